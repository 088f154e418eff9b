"""Transformer Linear weight gradient dW = dY^T X (K = tokens): one hipBLASLt GEMM vs split-K batched
GEMMs summed in fp32 (ops/conv.py _wgrad_splitk), on the ViT-B/16 and GPT-2-medium shapes.

    python tools/linear_wgrad_bench.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    from pytorch_distributed_training_example_amd.engine.gemm_tuning import use_repo_gemm_tuning
    from pytorch_distributed_training_example_amd.ops.conv import _wgrad_splitk
    use_repo_gemm_tuning()
    cases = []
    for name, T, d in (("vit128", 128 * 197, 768), ("vit32", 32 * 197, 768), ("gpt2m", 8 * 1024, 1024)):
        for dout, din in ((3 * d, d), (d, d), (4 * d, d), (d, 4 * d)):
            cases.append((name, T, dout, din))
    print(f"{'case':<8} {'T':>6} {'dout':>5} {'din':>5} | {'mm':>6} | " + " ".join(f"sk{s:<4}" for s in (2, 4, 8, 16)))
    for name, T, dout, din in cases:
        dy = torch.randn(T, dout, device="cuda").bfloat16()
        x = torch.randn(T, din, device="cuda").bfloat16()
        t_mm = timeit(lambda: dy.t() @ x)
        ts = []
        for s in (2, 4, 8, 16):
            ts.append(timeit(lambda: _wgrad_splitk(dy, x, s)) if T % s == 0 else float("nan"))
        print(f"{name:<8} {T:>6} {dout:>5} {din:>5} | {t_mm:6.0f} | " + " ".join(f"{t:6.0f}" for t in ts), flush=True)


if __name__ == "__main__":
    main()
