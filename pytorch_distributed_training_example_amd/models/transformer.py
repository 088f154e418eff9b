"""Transformer building blocks shared by ViT-B/16 and GPT-2 (north-star configs 3 and 4).

Not in the reference (LeNet only). MI355X-first choices:
  * every GEMM is a plain bf16 hipBLASLt GEMM (ops/linear.py: bias in the GEMM epilogue, bias
    gradient on the HIP column-strip kernel) with NO fused bias where an epilogue kernel
    follows: the MLP's first bias is applied inside the fused bias+GELU HIP kernel
    (ops/gelu.py), so the [tokens, 4·D] activation is read/written once;
  * LayerNorm is the wave-per-row HIP kernel (ops/layernorm.py) with fp32 parameters;
  * attention goes through ``ops.attention.attention`` ([B, H, T, Dh] bf16);
  * the LM / classifier loss is the fused softmax-cross-entropy kernel.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn

from ..config import SW
from ..ops.attention import attention_qkv
from ..ops.fp8 import add_layer_norm_fp8, fp8_input_slot, fp8_linear, fp8_mlp
from ..ops.gelu import bias_gelu
from ..ops.layernorm import LayerNorm, add_layer_norm
from ..ops.linear import linear as _linear
from ..ops.linear import linear_gelu


def linear(x, mod: nn.Linear, bias=True):
    """``mod``'s GEMM: fp8 when ``enable_fp8`` tagged it (ops/fp8.py), else bf16 (ops/linear.py).
    ``x`` may be an ``Fp8Act`` (already e4m3, from ``add_layer_norm_fp8``) for a tagged ``mod``."""
    b = mod.bias if bias else None
    fp8 = getattr(mod, "_fp8", None)
    if fp8 is not None:
        return fp8_linear(x, mod.weight, b, fp8[0], fp8[1])
    return _linear(x, mod.weight, b)


class SelfAttention(nn.Module):
    def __init__(self, dim: int, heads: int, causal: bool, bias: bool = True, dropout: float = 0.0):
        super().__init__()
        assert dim % heads == 0
        self.heads = heads
        self.causal = causal
        self.c_attn = nn.Linear(dim, 3 * dim, bias=bias)
        self.c_proj = nn.Linear(dim, dim, bias=bias)
        self.dropout = dropout

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        qkv = linear(x, self.c_attn)  # [B, T, 3D]; attention reads Q/K/V in place
        y = attention_qkv(qkv, self.heads, causal=self.causal, dropout_p=self.dropout if self.training else 0.0)
        return linear(y, self.c_proj)


class MLP(nn.Module):
    def __init__(self, dim: int, hidden: int, approximate: str = "none", bias: bool = True):
        super().__init__()
        self.c_fc = nn.Linear(dim, hidden, bias=bias)
        self.c_proj = nn.Linear(hidden, dim, bias=bias)
        self.approximate = approximate

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if getattr(self.c_fc, "_fp8", None) is not None:
            y = fp8_mlp(x, self.c_fc, self.c_proj, self.approximate)
            if y is not None:
                return y
        else:
            g = linear_gelu(x, self.c_fc.weight, self.c_fc.bias, self.approximate)  # PDT_LINEAR_EPILOGUE=1
            if g is not None:
                return linear(g, self.c_proj)
        h = linear(x, self.c_fc, bias=False)  # bias is fused into the GELU kernel
        b = self.c_fc.bias
        h = bias_gelu(h, b if b is None or b.dtype in (torch.float32, torch.bfloat16) else b.float(), self.approximate)
        return linear(h, self.c_proj)


class Block(nn.Module):
    """Pre-norm transformer block: x + attn(ln_1(x)), then x + mlp(ln_2(x))."""

    def __init__(self, dim: int, heads: int, mlp_ratio: float = 4.0, causal: bool = False,
                 approximate: str = "none", eps: float = 1e-5):
        super().__init__()
        self.ln_1 = LayerNorm(dim, eps=eps)
        self.attn = SelfAttention(dim, heads, causal)
        self.ln_2 = LayerNorm(dim, eps=eps)
        self.mlp = MLP(dim, int(dim * mlp_ratio), approximate)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x + self.attn(self.ln_1(x))
        x = x + self.mlp(self.ln_2(x))
        return x


def run_blocks(blocks, x: torch.Tensor, final_ln: nn.Module) -> torch.Tensor:
    """``final_ln(blocks(x))`` for pre-norm blocks, with every residual add fused into the
    LayerNorm that follows it (the block's ln_2, the next block's ln_1, finally ``final_ln``):
    one add+LN kernel per residual step forward and one LN-backward-with-accumulate backward,
    instead of separate add kernels each way (ops/layernorm.py add_layer_norm)."""
    blocks = list(blocks)
    if not blocks or not SW.fused_addln:
        for blk in blocks:
            x = blk(x)
        return final_ln(x)
    y = blocks[0].ln_1(x)
    for i, blk in enumerate(blocks):
        x, y = _add_ln(x, blk.attn(y), blk.ln_2, blk.mlp)
        nxt, cons = (blocks[i + 1].ln_1, blocks[i + 1].attn.c_attn) if i + 1 < len(blocks) else (final_ln, None)
        x, y = _add_ln(x, blk.mlp(y), nxt, cons)
    return y


def _add_ln(x, h, ln, consumer):
    """add_layer_norm, or its fp8-emitting form when ``consumer`` (the module the normalised output
    feeds) runs an fp8 GEMM on it (ops/fp8.py fp8_input_slot)."""
    if consumer is not None and getattr(ln, "weight", None) is not None and h.shape == x.shape:
        t = fp8_input_slot(consumer, x)
        if (t is not None and x.dtype == torch.bfloat16 and h.dtype == x.dtype and x.shape[-1] % 256 == 0
                and 2 <= x.shape[-1] // 256 <= 6 and ln.weight.dtype == torch.float32
                and ln.bias is not None and ln.bias.dtype == torch.float32 and len(ln.normalized_shape) == 1):
            return add_layer_norm_fp8(x, h, ln, t[0], t[1])
    return add_layer_norm(x, h, ln)


def init_weights(module: nn.Module, std: float = 0.02, n_layer: Optional[int] = None) -> None:
    for name, m in module.named_modules():
        if isinstance(m, nn.Linear):
            s = std
            if n_layer is not None and name.endswith("c_proj"):
                s = std / math.sqrt(2 * n_layer)  # GPT-2 residual-projection scaling
            nn.init.normal_(m.weight, 0.0, s)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, std)
