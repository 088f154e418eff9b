"""The fp8 producer kernels (csrc/kernels/fp8.hip, layernorm.hip) on the ViT-B/16 shapes: time per call
and achieved HBM bandwidth from the bytes each must move (bf16 in, e4m3 + transposed e4m3 out).

    python tools/fp8_cast_bench.py [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from pytorch_distributed_training_example_amd.ops._native import native
    C = native()
    M, D, H = 25216, 768, 3072

    from pytorch_distributed_training_example_amd.ops.fp8 import Fp8State

    def st():  # a striped state row, as the model's (Fp8State)
        s = Fp8State(1, history=16).cuda().state[0]
        s[1], s[2] = 16.0, 1 / 16.0
        return s
    h = torch.randn(M, H, device="cuda").bfloat16()
    dg = torch.randn(M, H, device="cuda").bfloat16()
    b = torch.randn(H, device="cuda")
    x = torch.randn(M, D, device="cuda").bfloat16()
    r = torch.randn(M, D, device="cuda").bfloat16()
    x3 = torch.randn(M, 3 * D, device="cuda").bfloat16()
    w, lb = torch.rand(D, device="cuda") + 0.5, torch.randn(D, device="cuda")
    s1 = st()
    cases = [
        ("gelu fwd -> e4m3 [25216, 3072]", lambda: C.fp8_gelu_cast(h, None, b, s1, False), M * H * (2 + 2)),
        ("gelu bwd -> e4m3 + db [25216, 3072]", lambda: C.fp8_gelu_cast(h, dg, b, s1, False), M * H * (4 + 2)),
        ("cast + colsum [25216, 768]", lambda: C.fp8_cast_colsum(x, s1, torch.bfloat16), M * D * (2 + 2)),
        ("cast + colsum [25216, 2304]", lambda: C.fp8_cast_colsum(x3, s1, torch.bfloat16), M * 3 * D * (2 + 2)),
        ("cast-transpose [25216, 768]", lambda: C.fp8_cast_transpose(x, s1, True), M * D * (2 + 2)),
        ("add + LayerNorm -> e4m3 [25216, 768]", lambda: C.ln_fwd_fp8(x, w, lb, 1e-6, r, s1), M * D * (2 + 2 + 2 + 2)),
        ("(ref) bias+GELU bf16 strip [25216, 3072]", lambda: C.bias_gelu_fwd(h, b, False), M * H * (2 + 2)),
        ("(ref) add + LayerNorm bf16 [25216, 768]", lambda: C.ln_fwd(x, w, lb, 1e-6, r), M * D * (2 + 2 + 2 + 2)),
    ]
    print(f"{'kernel':<44}{'us':>9}{'GB':>8}{'TB/s':>7}", flush=True)
    for name, fn, nbytes in cases:
        us = timeit(fn, a.reps)
        print(f"{name:<44}{us:9.1f}{nbytes / 1e9:8.3f}{nbytes / us / 1e6:7.2f}", flush=True)


if __name__ == "__main__":
    main()
