"""Measure the P2P all-reduce crossovers that parallel/p2p.py and bench.py currently set by estimate:
``ONESHOT_MAX_BYTES`` (one-shot vs two-shot, p2p.py:41) and the DDP hook's cap (the bucket size up to which
the xGMI P2P kernel beats RCCL, bench.py ``--comm-hook p2p``). Needs >= 2 GPUs on one node (the round's
gpurun boxes have one, so the constants stay estimates there); run as

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29555 tools/p2p_crossover.py [--max-mb 64]

Rank 0 prints one JSON line per size: us per call (max over ranks) for one-shot, two-shot and RCCL, bf16,
and at the end the two crossovers it implies."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    t = torch.tensor([s.elapsed_time(e) * 1e3 / iters], device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mb", type=float, default=64.0)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl")
    world = dist.get_world_size()
    if world < 2:
        raise SystemExit("p2p_crossover needs >= 2 ranks (one GPU each)")
    from pytorch_distributed_training_example_amd.parallel.p2p import P2PAllReduce
    cap = int(a.max_mb * (1 << 20))
    p2p = P2PAllReduce(capacity_bytes=cap)
    rows, nbytes = [], 16 << 10
    while nbytes <= cap:
        x = torch.randn(nbytes // 2, device="cuda").bfloat16()
        r = {"bytes": nbytes, "world": world,
             "oneshot_us": timed(lambda: p2p.all_reduce(x, algo=0), a.iters),
             "twoshot_us": timed(lambda: p2p.all_reduce(x, algo=1), a.iters),
             "rccl_us": timed(lambda: dist.all_reduce(x), a.iters)}
        rows.append(r)
        if dist.get_rank() == 0:
            print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        nbytes *= 2
    if dist.get_rank() == 0:
        one = max((r["bytes"] for r in rows if r["oneshot_us"] <= r["twoshot_us"]), default=0)
        hook = max((r["bytes"] for r in rows if min(r["oneshot_us"], r["twoshot_us"]) <= r["rccl_us"]), default=0)
        print(json.dumps({"oneshot_max_bytes": one, "p2p_beats_rccl_up_to_bytes": hook,
                          "current": {"ONESHOT_MAX_BYTES": 256 << 10, "hook_max_bytes": 1 << 20}}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
