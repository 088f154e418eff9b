"""GPT-2 (north-star config 4: GPT-2-medium DDP, the sequence path).

GPT-2 medium: 24 layers, 16 heads, D=1024, context 1024, tanh-GELU, tied input/output
embedding. The vocabulary is padded from 50257 to 50304 (a multiple of 64) so the LM-head
GEMM and the fused cross-entropy rows are MFMA/vector aligned; padded logits are never a
target. Parameter names follow the nanoGPT layout of HF GPT-2 (``transformer.wte``,
``transformer.h.{i}.attn.c_attn``, ``ln_1``, ``mlp.c_fc`` …, weights as [out, in]).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn

from ..ops.cross_entropy import cross_entropy
from ..ops.embedding import token_position_embedding
from ..ops.layernorm import LayerNorm
from .transformer import Block, init_weights, run_blocks


@dataclass
class GPTConfig:
    n_layer: int = 24
    n_head: int = 16
    n_embd: int = 1024
    block_size: int = 1024
    vocab_size: int = 50304   # 50257 padded to a multiple of 64


class GPT(nn.Module):
    def __init__(self, cfg: GPTConfig = GPTConfig()):
        super().__init__()
        self.cfg = cfg
        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(cfg.vocab_size, cfg.n_embd),
            wpe=nn.Embedding(cfg.block_size, cfg.n_embd),
            h=nn.ModuleList([Block(cfg.n_embd, cfg.n_head, 4.0, causal=True, approximate="tanh")
                             for _ in range(cfg.n_layer)]),
            ln_f=LayerNorm(cfg.n_embd),
        ))
        self.lm_head = nn.Linear(cfg.n_embd, cfg.vocab_size, bias=False)
        self.lm_head.weight = self.transformer.wte.weight  # tied
        init_weights(self, n_layer=cfg.n_layer)

    def forward(self, idx: torch.Tensor, targets: torch.Tensor | None = None):
        # one fused gather pass forward, deterministic scatter backward (ops/embedding.py)
        x = token_position_embedding(idx, self.transformer.wte.weight, self.transformer.wpe.weight)
        x = run_blocks(self.transformer.h, x, self.transformer.ln_f)  # == ln_f(h[-1](...h[0](x)))
        logits = self.lm_head(x)
        if targets is None:
            return logits
        return cross_entropy(logits.reshape(-1, logits.shape[-1]), targets.reshape(-1))


def gpt2_medium(**kw) -> GPT:
    return GPT(GPTConfig(**kw))


def gpt2_small(**kw) -> GPT:
    return GPT(GPTConfig(n_layer=12, n_head=12, n_embd=768, **kw))


def gpt2_tiny(**kw) -> GPT:
    """Small config for tests."""
    kw.setdefault("vocab_size", 512)
    kw.setdefault("block_size", 64)
    return GPT(GPTConfig(n_layer=2, n_head=4, n_embd=256, **kw))


from . import register  # noqa: E402

register("gpt2_medium", gpt2_medium)
register("gpt2_small", gpt2_small)
register("gpt2_tiny", gpt2_tiny)
