"""1x1-conv weight gradient dW = dY^T X (K = pixels, both operands pixel-major) as split-K batched
GEMMs on hipBLASLt, against MIOpen's kernel: can a [S, Co, M/S] x [S, M/S, Ci] bmm + a sum over S
reach the HBM floor where MIOpen runs at ~0.5 PF (ResNet-50 layer3/4 shapes)?

    python tools/wgrad_split_bench.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = [(1, 64, 64, 56), (4, 64, 256, 56), (2, 256, 64, 56), (1, 256, 128, 56), (4, 128, 512, 28), (3, 512, 128, 28), (1, 512, 256, 28), (6, 256, 1024, 14),
          (5, 1024, 256, 14), (1, 1024, 512, 14), (3, 512, 2048, 7), (2, 2048, 512, 7)]


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
    from pytorch_distributed_training_example_amd.engine.miopen_cache import use_repo_miopen_cache
    use_repo_miopen_cache()
    B = int(os.environ.get("BATCH", "512"))
    print(f"{'(n, Ci, Co, H)':<20} | miopen | " + " ".join(f"bmm{s:>3}" for s in (4, 8, 16, 32, 64)) + " | fp32out16 | floor")
    for n, ci, co, h in SHAPES:
        M = B * h * h
        x = torch.randn(B, ci, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        gy = torch.randn(B, co, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = torch.randn(co, ci, 1, 1, device="cuda").bfloat16()
        x2, g2 = x.permute(0, 2, 3, 1).reshape(M, ci), gy.permute(0, 2, 3, 1).reshape(M, co)
        ref = (g2.float().t() @ x2.float())
        t_mi = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [1, 1], [0, 0], [1, 1], False,
                                                                  [0, 0], 1, [False, True, False]))
        ts = []
        for s in (4, 8, 16, 32, 64):  # noqa: B007
            if M % s:
                ts.append(float("nan"))
                continue
            gb, xb = g2.view(s, M // s, co), x2.view(s, M // s, ci)
            f = lambda: torch.bmm(gb.transpose(1, 2), xb).float().sum(0)  # noqa: E731
            ts.append(timeit(f))
            err = ((f() - ref).norm() / ref.norm()).item()
            if err > 2e-2:
                print("  bad", s, err)
        t32 = float("nan")
        try:
            gb, xb = g2.view(16, M // 16, co), x2.view(16, M // 16, ci)
            f = lambda: torch.bmm(gb.transpose(1, 2), xb, out_dtype=torch.float32).sum(0)  # noqa: E731
            t32 = timeit(f)
        except Exception as e:  # noqa: BLE001
            t32 = -1.0
            print("  out_dtype unsupported:", str(e)[:80])
        floor = M * (ci + co) * 2 / 5.3e12 * 1e6
        print(f"{str((n, ci, co, h)):<20} | {t_mi:6.0f} | " + " ".join(f"{t:6.0f}" for t in ts) + f" | {t32:9.0f} | {floor:5.0f}",
              flush=True)


if __name__ == "__main__":
    main()
