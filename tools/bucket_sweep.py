#!/usr/bin/env python3
"""RCCL bucket-size sweep (BASELINE.json config 5: "ResNet-50 DDP with hipGraph-captured train
step + RCCL bucket-size sweep").

Two sweeps, one process per GPU (launch with torchrun, 127.0.0.1 rendezvous):

  collectives : all-reduce latency / algorithm bandwidth / bus bandwidth per message size
                (64 KiB … 256 MiB, bf16) — where the per-link-bound ring regime starts on xGMI —
                for RCCL and for the one-shot P2P kernel (parallel/p2p.py) up to its capacity
  train       : full ResNet-50 DDP steps (bench.py's workload, eager or hipGraph) for each
                ``bucket_cap_mb`` — the end-to-end effect of bucket granularity on overlap

  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bucket_sweep.py --caps 1,5,10,25,50,100
  python tools/bucket_sweep.py --mode collectives --backend gloo   # CPU plumbing check
  python tools/bucket_sweep.py --nproc 8 --nchannels 4,8,16,32 --caps 10,25,50
      # third axis: RCCL channel count (NCCL_MIN/MAX_NCHANNELS, read once per process at communicator
      # creation, so each value runs as its own torchrun job; every JSON line carries "nchannels")

xGMI is point-to-point (7 links x ~153 GB/s per GPU): a single ring is bound by ONE link, so the
bucket size that hides the last bucket's all-reduce under backward and the number of RCCL channels
(parallel rings over different links) have to be chosen together.

The reference issues one un-bucketed fp32 all-reduce per parameter after backward
(/root/reference/train.py:34-39); its sizes are printed for comparison (--reference-sizes).
Each result is one JSON line on rank 0; ``--out`` also writes them to a file.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pytorch_distributed_training_example_amd.parallel import launcher  # noqa: E402

# per-parameter gradient sizes of the reference LeNet step
REFERENCE_SIZES = [150, 6, 2400, 16, 48000, 120, 10080, 84, 840, 10]


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def time_allreduce(numel: int, dtype, dev, iters: int, warmup: int) -> float:
    """Seconds per all-reduce (MAX over ranks)."""
    t = torch.ones(numel, dtype=dtype, device=dev)
    op = dist.ReduceOp.AVG if dist.get_backend() == "nccl" else dist.ReduceOp.SUM
    for _ in range(warmup):
        dist.all_reduce(t, op=op)
    _sync(dev)
    launcher.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(t, op=op)
    _sync(dev)
    el = (time.perf_counter() - t0) / iters
    m = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return float(m.item())


def time_p2p(p2p, numel: int, dtype, dev, iters: int, warmup: int, algo: int = 0) -> float:
    t = torch.ones(numel, dtype=dtype, device=dev)
    for _ in range(warmup):
        p2p.all_reduce(t, algo=algo)
    _sync(dev)
    launcher.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        p2p.all_reduce(t, algo=algo)
    _sync(dev)
    el = (time.perf_counter() - t0) / iters
    m = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return float(m.item())


def sweep_collectives(args, ctx, emit):
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[args.dtype]
    esize = torch.finfo(dtype).bits // 8
    n = ctx.world_size
    sizes = [int(s) for s in args.sizes.split(",")] if args.sizes else \
        [1 << k for k in range(16, 29, 2)]  # 64 KiB .. 256 MiB
    if args.reference_sizes:
        sizes = [s * 4 for s in REFERENCE_SIZES] + [sum(REFERENCE_SIZES) * 4]
        dtype, esize = torch.float32, 4
    p2p = None
    if args.p2p and ctx.device.type == "cuda":
        from pytorch_distributed_training_example_amd.parallel.p2p import P2PAllReduce
        p2p = P2PAllReduce(capacity_bytes=args.p2p_capacity_mb << 20)
    for nbytes in sizes:
        numel = max(1, nbytes // esize)
        sec = time_allreduce(numel, dtype, ctx.device, args.iters, args.warmup)
        algbw = numel * esize / sec / 1e9
        emit({"sweep": "collectives", "op": "all_reduce", "bytes": numel * esize, "dtype": str(dtype),
              "n_ranks": n, "us": round(sec * 1e6, 2), "algbw_GBps": round(algbw, 2),
              "busbw_GBps": round(algbw * 2 * (n - 1) / max(n, 1), 2), "backend": dist.get_backend()})
        if p2p is not None and numel % 8 == 0 and numel * esize <= p2p.capacity:
            for algo, name in ((0, "p2p_oneshot"), (1, "p2p_twoshot")):
                sec = time_p2p(p2p, numel, dtype, ctx.device, args.iters, args.warmup, algo)
                emit({"sweep": "collectives", "op": name, "bytes": numel * esize, "dtype": str(dtype),
                      "n_ranks": n, "us": round(sec * 1e6, 2), "algbw_GBps": round(numel * esize / sec / 1e9, 2)})
    if p2p is not None:
        p2p.check()


def sweep_train(args, ctx, emit):
    import bench  # noqa: E402  (repo root on sys.path)
    for cap in [float(c) for c in args.caps.split(",")]:
        bargs = bench.parse(["--gpus", str(ctx.world_size), "--steps", str(args.steps), "--warmup",
                             str(args.train_warmup), "--model", args.model, "--graph", str(args.graph),
                             "--bucket-cap-mb", str(cap)] + (["--batch-size", str(args.batch_size)]
                                                             if args.batch_size else []))
        res = bench.run(bargs, ctx)
        emit({"sweep": "train", "bucket_cap_mb": cap, "graph": bool(args.graph), "model": args.model,
              "n_gpus": ctx.world_size, "value": res["value"], "unit": res["unit"],
              "ms_per_step": res["ms_per_step"]})
        del res
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.empty_cache()


def channel_sweep(args, argv) -> int:
    """One torchrun job per RCCL channel count; the child jobs print JSON lines tagged with it."""
    import subprocess
    rest, skip = [], False
    for a in argv:  # drop --nchannels / --nproc and their values
        if skip:
            skip = False
            continue
        if a in ("--nchannels", "--nproc"):
            skip = True
            continue
        if a.startswith("--nchannels=") or a.startswith("--nproc="):
            continue
        rest.append(a)
    nproc = args.nproc or max(1, torch.cuda.device_count())
    rc = 0
    for ch in [int(c) for c in args.nchannels.split(",")]:
        env = dict(os.environ, NCCL_MIN_NCHANNELS=str(ch), NCCL_MAX_NCHANNELS=str(ch), PDT_SWEEP_NCHANNELS=str(ch),
                   MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", f"--master-port={launcher.find_free_port()}",
               os.path.abspath(__file__), *rest]
        rc |= subprocess.run(cmd, env=env).returncode
    return rc


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nchannels", default=None,
                    help="comma list of RCCL channel counts: one child job each (NCCL_MIN/MAX_NCHANNELS)")
    ap.add_argument("--nproc", type=int, default=None, help="ranks per child job (default: visible GPUs)")
    ap.add_argument("--mode", default="both", choices=["collectives", "train", "both"])
    ap.add_argument("--backend", default=None)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--sizes", default=None, help="comma list of message sizes in bytes")
    ap.add_argument("--reference-sizes", action="store_true", help="the reference's 10 per-param sizes (fp32)")
    ap.add_argument("--p2p", type=int, default=1, help="also time the one-shot xGMI P2P all-reduce (GPU)")
    ap.add_argument("--p2p-capacity-mb", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--caps", default="1,5,10,25,50,100", help="bucket_cap_mb values for the train sweep")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch-size", type=int, default=None)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--train-warmup", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    if args.nchannels and "WORLD_SIZE" not in os.environ:
        return channel_sweep(args, argv)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    gpu = torch.cuda.is_available() and args.backend in (None, "nccl")
    if args.mode != "collectives" and args.graph and gpu:
        from pytorch_distributed_training_example_amd.engine.graph import make_miopen_capture_safe
        make_miopen_capture_safe()
    os.environ.setdefault("PDT_FORCE_PG", "1")  # a group even at world 1 (collective timings)
    ctx = launcher.init_distributed(backend=args.backend, use_gpu=gpu)
    lines = []

    nch = os.environ.get("PDT_SWEEP_NCHANNELS")

    def emit(d):
        if nch:
            d = dict(d, nchannels=int(nch))
        lines.append(d)
        if ctx.rank == 0:
            print(json.dumps(d), flush=True)

    if args.mode in ("collectives", "both"):
        sweep_collectives(args, ctx, emit)
    if args.mode in ("train", "both") and gpu:
        sweep_train(args, ctx, emit)
    if ctx.rank == 0 and args.out:
        with open(args.out, "w") as f:
            for d in lines:
                f.write(json.dumps(d) + "\n")
    launcher.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
