"""Flash-attention kernel timing on the north-star shapes: ours (csrc/kernels/attention.hip) vs
PyTorch SDPA, forward and forward+backward, with achieved TFLOP/s.

FLOPs: forward 4·B·H·T²·D (halved for causal), backward 2.5x forward (5 products vs 2).

usage: python tools/attn_bench.py
"""
import math
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402

SHAPES = [  # name, B, H, T, causal
    ("gpt2-medium", 8, 16, 1024, True),
    ("vit-b16", 128, 12, 197, False),
    ("long", 2, 16, 4096, True),
]


def timed(fn, it=10):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    C = native()
    D = 64
    print(f"{'shape':12s} | {'ours fwd us':>11} {'TF/s':>5} | {'ours bwd us':>11} {'TF/s':>5} | "
          f"{'sdpa fwd us':>11} {'TF/s':>5} | {'sdpa bwd us':>11} {'TF/s':>5}")
    for name, B, H, T, causal in SHAPES:
        q, k, v = (torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        scale = 1 / math.sqrt(D)
        out = torch.empty(B, H, T, D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B, H, T, device="cuda", dtype=torch.float32)
        fl = 4 * B * H * T * T * D * (0.5 if causal else 1.0)
        tf = timed(lambda: C.attn_fwd_out(q, k, v, out, lse, causal, scale))
        do = torch.randn_like(out)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        tb = timed(lambda: C.attn_bwd_out(do, q, k, v, out, lse, dq, dk, dv, causal, scale))
        qs, ks, vs = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
        sf = timed(lambda: F.scaled_dot_product_attention(qs, ks, vs, is_causal=causal, scale=scale))
        ys = F.scaled_dot_product_attention(qs, ks, vs, is_causal=causal, scale=scale)
        sb = timed(lambda: torch.autograd.grad(ys, (qs, ks, vs), do, retain_graph=True))
        print(f"{name:12s} | {tf:11.1f} {fl / tf / 1e6:5.0f} | {tb:11.1f} {2.5 * fl / tb / 1e6:5.0f} | "
              f"{sf:11.1f} {fl / sf / 1e6:5.0f} | {sb:11.1f} {2.5 * fl / sb / 1e6:5.0f}", flush=True)


if __name__ == "__main__":
    main()
