"""ViT-B/16 (north-star config 3: ViT-B/16 DDP + AMP + gradient accumulation).

Standard ViT: 16×16 patch embedding (a stride-16 conv = one GEMM over non-overlapping
patches), learned position embedding, class token, 12 pre-norm blocks (D=768, 12 heads,
MLP 3072, exact-erf GELU), final LayerNorm, linear head on the class token. Parameter names
follow torchvision's ``vit_b_16`` layout loosely (``conv_proj``, ``class_token``,
``encoder.pos_embedding``, ``encoder.layers.{i}``, ``encoder.ln``, ``heads.head``).
"""
from __future__ import annotations

import torch
from torch import nn

from ..ops.conv import PatchConv2d
from ..ops.layernorm import LayerNorm
from .transformer import Block, init_weights, run_blocks


class _Encoder(nn.Module):
    def __init__(self, seq: int, dim: int, depth: int, heads: int, mlp_ratio: float):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq, dim).normal_(std=0.02))
        self.layers = nn.ModuleList([Block(dim, heads, mlp_ratio, causal=False, approximate="none", eps=1e-6)
                                     for _ in range(depth)])
        self.ln = LayerNorm(dim, eps=1e-6)

    def forward(self, x):
        x = x + self.pos_embedding.to(x.dtype)
        return run_blocks(self.layers, x, self.ln)  # == ln(layers[-1](...layers[0](x)))


class _Heads(nn.Module):
    def __init__(self, dim: int, num_classes: int):
        super().__init__()
        self.head = nn.Linear(dim, num_classes)

    def forward(self, x):
        return self.head(x)


class VisionTransformer(nn.Module):
    def __init__(self, image_size: int = 224, patch_size: int = 16, dim: int = 768, depth: int = 12,
                 heads: int = 12, mlp_ratio: float = 4.0, num_classes: int = 1000, **_):
        super().__init__()
        self.patch_size = patch_size
        n = (image_size // patch_size) ** 2
        # patchify + one GEMM on the GPU (ops/conv.py PatchConv2d; nn.Conv2d parameters / state_dict)
        self.conv_proj = PatchConv2d(3, dim, kernel_size=patch_size, stride=patch_size)
        self.class_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.encoder = _Encoder(n + 1, dim, depth, heads, mlp_ratio)
        self.heads = _Heads(dim, num_classes)
        init_weights(self)
        nn.init.zeros_(self.heads.head.weight)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.conv_proj(x)                      # [B, D, H/16, W/16]
        x = x.flatten(2).transpose(1, 2)           # [B, N, D]
        cls = self.class_token.to(x.dtype).expand(x.shape[0], -1, -1)
        x = torch.cat([cls, x], dim=1)
        x = self.encoder(x)
        return self.heads(x[:, 0])


def vit_b16(**kw) -> VisionTransformer:
    return VisionTransformer(patch_size=16, dim=768, depth=12, heads=12, **kw)


def vit_tiny(**kw) -> VisionTransformer:
    """Small config for tests."""
    return VisionTransformer(image_size=kw.pop("image_size", 32), patch_size=8, dim=256, depth=2, heads=4, **kw)


from . import register  # noqa: E402

register("vit_b16", vit_b16)
register("vit_tiny", vit_tiny)
