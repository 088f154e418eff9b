"""1x1-conv weight gradient at ResNet-50 shapes (batch 1024 by default): our kernel
(csrc/kernels/conv1x1_wgrad.hip) vs MIOpen (aten convolution_backward) vs hipBLASLt split-K
(ops/conv.py _wgrad_splitk), with the HBM floor (bytes of dY + X at 5.5 TB/s).

    python tools/conv1x1_wgrad_bench.py [--batch 1024] [--wgs 0,512,1024]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_distributed_training_example_amd.ops._native import native  # noqa: E402
from pytorch_distributed_training_example_amd.ops.conv import _wgrad_splitk  # noqa: E402


def timeit(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--wgs", default="0")
    ap.add_argument("--variants", default="-1", help="pipeline variants (conv1x1_wgrad.hip kVarKP/kVarSlots)")
    ap.add_argument("--ilv", default="-1", help="interleaved split stages: 0,1 (-1 = by shape)")
    ap.add_argument("--miopen", type=int, default=1)
    ap.add_argument("--layer1-only", type=int, default=0)
    a = ap.parse_args()
    B = a.batch
    # (H, Ci, Co): layer-1 (56x56) and the layer-2 block-0 conv1 (256 -> 128 at 56x56), then layers 2-4
    shapes = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
              (14, 256, 1024), (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]
    C = native()
    if a.layer1_only:
        shapes = [sh for sh in shapes if sh[0] == 56]
    for H, Ci, Co in shapes:
        M = B * H * H
        x4 = torch.randn(B, Ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        g4 = torch.randn(B, Co, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = torch.randn(Co, Ci, 1, 1, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        x2 = x4.permute(0, 2, 3, 1).reshape(M, Ci)
        g2 = g4.permute(0, 2, 3, 1).reshape(M, Co)
        floor = (M * (Ci + Co) * 2) / 5.5e12 * 1e6
        row = [f"M={M:8d} {Ci:5d}->{Co:5d} floor {floor:7.1f} us"]
        ref = g2.float().t() @ x2.float()
        res = []
        for il in [int(t) for t in a.ilv.split(",")]:
            for v in [int(t) for t in a.variants.split(",")]:
                for wg in [int(t) for t in a.wgs.split(",")]:
                    C.conv1x1_wgrad_tune(wg, v, il)
                    d = C.conv1x1_wgrad(x2, g2)
                    err = ((d.float() - ref).abs().max() / ref.abs().max()).item()
                    assert err < 1e-2, err
                    res.append((timeit(lambda: C.conv1x1_wgrad(x2, g2)), il, v, wg))
        C.conv1x1_wgrad_tune(0, -1, -1)
        row.append(" ".join(f"i{il}v{v}w{wg}:{t:.0f}" for t, il, v, wg in res))
        t, il, v, wg = min(res)
        row.append(f"best ours ilv{il}/v{v}/wgs{wg} {t:7.1f} us")
        if a.miopen:
            mi = lambda: torch.ops.aten.convolution_backward(g4, x4, w, None, [1, 1], [0, 0], [1, 1], False,  # noqa
                                                              [0, 0], 1, [False, True, False])
            row.append(f"miopen {timeit(mi):7.1f} us")
        best = min((timeit(lambda sk=sk: _wgrad_splitk(g2, x2, sk)), sk) for sk in (8, 16, 32, 64) if M % sk == 0)
        row.append(f"splitk{best[1]} {best[0]:7.1f} us")
        print(" | ".join(row), flush=True)


if __name__ == "__main__":
    main()
