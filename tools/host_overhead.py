"""Host-side cost of one ResNet-50 training step vs its GPU time: perf_counter around the forward
(+ loss), the backward call and the optimizer step — none of which wait for the GPU — then one
device sync. If the host's phases add up to about the GPU step time, the GPU idles wherever the
host falls behind (the start of backward: profiles/r2 trace gaps).

    python tools/host_overhead.py [bench args]
"""
from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = bench.parse(sys.argv[1:])
    ctx = bench.setup(args)
    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)
    model, ddp, opt, precision = bench.build(args, ctx)
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    B = args.batch_size or bench.WORKLOADS[args.model][2]
    x = torch.randn(B, 3, args.image_size, args.image_size, device="cuda").bfloat16().contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device="cuda")
    for _ in range(args.warmup):
        opt.zero_grad(set_to_none=True)
        cross_entropy(ddp(x), y, label_smoothing=0.1).backward()
        opt.step()
    torch.cuda.synchronize()
    rows = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss = cross_entropy(ddp(x), y, label_smoothing=0.1)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        opt.step()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        rows.append((t1 - t0, t2 - t1, t3 - t2, t4 - t0))
    for r in rows:
        print("[host] fwd %.2f ms  bwd-call %.2f ms  opt %.2f ms  | host total %.2f  wall (synced) %.2f ms"
              % (r[0] * 1e3, r[1] * 1e3, r[2] * 1e3, (r[0] + r[1] + r[2]) * 1e3, r[3] * 1e3), flush=True)


if __name__ == "__main__":
    main()
