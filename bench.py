#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 DDP training throughput (images/sec, whole node) on MI355X.

BASELINE.json metric: "images/sec (whole node) ResNet-50 DDP at 1/2/4/8 MI355X". The reference
publishes no number, so ``vs_baseline`` is null.

  python bench.py --gpus N --steps K --warmup W            # launches N ranks itself (N>1)
  torchrun --nproc-per-node N ... bench.py --gpus N ...    # same, under an external launcher
                                                           # (WORLD_SIZE must equal N)

Each step is a full training step on synthetic data with random-init weights: forward, loss,
backward, bucketed RCCL all-reduce overlapped with backward, fused optimizer update. W
warm-up steps are untimed; exactly K steps are timed between barrier + device synchronize on
both sides; the reported time is the MAX over ranks; ``value`` is the total over all N GPUs
(weak scaling: per-GPU batch fixed; ``--global-batch G`` = strong scaling with the reference's
global-batch semantics, ceil(G/N) per rank, train.py:82).

--model resnet50 (default, headline) | vit_b16 | gpt2_medium (other north-star configs)
        | lenet (the reference's own LeNet/MNIST workload, fp32, Adadelta)
--impl ours       : this framework (DDP reducer, HIP BN/LN/GELU/CE/optimizer kernels, bf16 params +
                    fp32 master weights)
--impl torch_ddp  : stock torch.nn.parallel.DistributedDataParallel + autocast bf16 + stock
                    nn modules + torch optimizer (baseline B0)
--impl reference  : the reference's algorithm — per-parameter all-reduce after backward (B1)
"""
from __future__ import annotations

import argparse
import contextlib
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from pytorch_distributed_training_example_amd.parallel import launcher  # noqa: E402

WORKLOADS = {
    # name: (metric, unit, default per-GPU batch, optimizer)
    # 1024 images per GPU: sized for 288 GB of HBM (round 1: bs 256: 9.29k, 384: 9.57k, 512: 10.04k
    # img/s, tools/gpu_batchsweep.sh; round 2: 512: 12.24k, 1024: 13.08k, tools/gpu_bsz.sh) and a 4x
    # larger compute window per all-reduce at N > 1 than 256
    # metric string verbatim from BASELINE.json:2 (the driver computes the scaling efficiency)
    "resnet50": ("images/sec (whole node) ResNet-50 DDP at 1/2/4/8 MI355X; scaling efficiency",
                 "images/sec", 1024, "sgd"),
    "vit_b16": ("images/sec (whole node) ViT-B/16 DDP", "images/sec", 128, "adamw"),
    "gpt2_medium": ("tokens/sec (whole node) GPT-2-medium DDP", "tokens/sec", 8, "adamw"),
    # the reference's own workload (train.py:82-105): LeNet on MNIST-shaped data, fp32, Adadelta,
    # nll_loss on softmax probabilities, global batch 1024 = 128 per GPU at 8 GPUs
    "lenet": ("images/sec (whole node) LeNet-MNIST DDP (reference workload)", "images/sec", 128, "adadelta"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet50", choices=sorted(WORKLOADS))
    ap.add_argument("--batch-size", type=int, default=None, help="per-GPU batch (default per model)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling with the reference's semantics (train.py:82): per-rank batch = "
                         "ceil(G / N); overrides --batch-size")
    ap.add_argument("--grad-accum", type=int, default=1, help="micro-batches per step (no_sync)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--impl", default="ours", choices=["ours", "torch_ddp", "reference"])
    ap.add_argument("--graph", type=int, default=0,
                    help="1: hipGraph-capture the step (ours: forward, backward, the bucket all-reduce and the optimizer "
                         "replayed; excludes the capture-unsafe MIOpen solvers). Default 0: at 1024/GPU the captured "
                         "step measures the same as eager (15,455-15,468 vs 15,467-15,487 img/s on one box, "
                         "profiles/r6/ab_graph_b1024.txt); it pays at small per-GPU batches (launch-bound)")
    ap.add_argument("--bucket-cap-mb", default="auto",
                    help="MiB cap per gradient bucket, or 'auto' (ours): the comm-model plan whose last-filling "
                         "bucket is <= 2 MiB (parallel/buckets.py plan_auto); torch_ddp uses 25 for 'auto'")
    ap.add_argument("--reduce-single-rank", type=int, default=1,
                    help="ours at N=1: still pack buckets and issue the (1-rank RCCL) all-reduce, as torch "
                         "DDP does, so N=1 carries the same per-step reducer work as N>1")
    ap.add_argument("--comm-hook", default="none", choices=["none", "p2p"],
                    help="p2p: one-shot xGMI P2P all-reduce for buckets <= 1 MiB, RCCL above (ours, N>1)")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp8", "amp_bf16", "fp32"],
                    help="fp8: transformer-block GEMMs on e4m3 with delayed scaling (ViT/GPT-2)")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--cudnn-benchmark", type=int, default=1, help="MIOpen find mode for conv algorithms")
    ap.add_argument("--deterministic", type=int, default=0, help="MIOpen deterministic solvers (slow)")
    ap.add_argument("--backend", default=None, help="process-group backend (default: nccl = RCCL on GPU)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


def build(args, ctx):
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.models.precision import apply_precision
    dev = ctx.device
    torch.manual_seed(1234)
    kw = {}
    if args.model.startswith("resnet"):
        kw["norm"] = "pdt" if args.impl == "ours" else "torch"  # stock baseline uses nn.BatchNorm2d
    if args.model == "lenet":  # ours: fused kernels + reference loss from logits; stock: cnn.py as-is
        kw = dict(output="logits") if args.impl == "ours" else dict(output="probs", fused=False)
    model = get_model(args.model, **kw).to(dev)
    if args.model.startswith("resnet"):
        model = model.to(memory_format=torch.channels_last)
    precision = args.precision
    if args.model == "lenet":
        precision = "fp32"  # the reference trains LeNet in fp32
    if args.impl != "ours" and precision == "bf16":
        precision = "amp_bf16"  # stock path: fp32 params + autocast (what torch users run)
    model = apply_precision(model, precision)
    world = ctx.world_size
    opt_name = WORKLOADS[args.model][3]
    lr = args.lr if args.lr is not None else (0.1 if opt_name in ("sgd", "adadelta") else 1e-4)
    if args.impl == "ours":
        from pytorch_distributed_training_example_amd.optim import FusedAdadelta, FusedAdamW, FusedSGD
        from pytorch_distributed_training_example_amd.parallel import DistributedDataParallel
        ddp = DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb, broadcast_buffers=False,
                                      gradient_as_bucket_view=True,
                                      reduce_single_rank=bool(args.reduce_single_rank))
        if args.comm_hook == "p2p" and world > 1:
            from pytorch_distributed_training_example_amd.parallel.p2p import (P2PAllReduce, P2PHookState,
                                                                                p2p_allreduce_hook)
            ddp.register_comm_hook(P2PHookState(P2PAllReduce(capacity_bytes=2 << 20), max_bytes=1 << 20),
                                   p2p_allreduce_hook)
        if opt_name == "sgd":
            opt = FusedSGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
        elif opt_name == "adadelta":
            opt = FusedAdadelta(model.parameters(), lr=lr)
        else:
            opt = FusedAdamW(model.parameters(), lr=lr, weight_decay=0.1)
    else:
        if args.impl == "torch_ddp" and world > 1:
            ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index],
                                                            bucket_cap_mb=(25.0 if args.bucket_cap_mb == "auto"
                                                                           else float(args.bucket_cap_mb)),
                                                            broadcast_buffers=False, gradient_as_bucket_view=True)
        else:
            ddp = model
        if opt_name == "sgd":
            opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
        elif opt_name == "adadelta":
            opt = torch.optim.Adadelta(model.parameters(), lr=lr)
        else:
            opt = torch.optim.AdamW(model.parameters(), lr=lr, weight_decay=0.1, fused=True)
    return model, ddp, opt, precision


def setup(args):
    """Environment + process group (once per process)."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if args.impl != "ours":
        # stock baseline: every op (BN, LN, GELU, attention, CE) on PyTorch's own kernels
        os.environ["PDT_DISABLE_NATIVE"] = "1"
        from pytorch_distributed_training_example_amd.config import SW
        SW.reload()  # switches are read once per process
    if args.impl == "ours" and args.graph:
        # two MIOpen CK solvers replay wrong gradients under capture (tools/diag_conv_graph.py);
        # MIOpen reads the switch once, so this must precede the first convolution
        from pytorch_distributed_training_example_amd.engine.graph import make_miopen_capture_safe
        make_miopen_capture_safe()
    from pytorch_distributed_training_example_amd.engine.miopen_cache import use_repo_miopen_cache
    use_repo_miopen_cache()  # persisted conv-algorithm find-db + kernel cache (after the solver switches)
    # measured hipBLASLt/rocBLAS solution per GEMM shape (read-only table), same predicate as cli.py
    from pytorch_distributed_training_example_amd.engine.gemm_tuning import (use_repo_gemm_tuning,
                                                                             wants_gemm_tuning)
    if args.impl == "ours" and wants_gemm_tuning(args.model, args.grad_accum, args.graph):
        use_repo_gemm_tuning()
    return launcher.init_distributed(backend=args.backend or ("nccl" if torch.cuda.is_available() else "gloo"),
                                     use_gpu=torch.cuda.is_available())


def run(args, ctx):
    """Build the workload, warm up, time ``args.steps`` steps; returns the result dict (all ranks)."""
    dev = ctx.device
    world = ctx.world_size
    # device sync (a no-op for CPU/gloo rehearsals of the multi-rank path)
    dsync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    metric, unit, default_b, _ = WORKLOADS[args.model]
    B = args.batch_size or default_b
    if args.global_batch:  # the reference's --batch-size is global: ceil(1024 / N) per rank (train.py:82)
        B = -(-args.global_batch // world)
    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)
    det = max(args.deterministic, 0)
    torch.backends.cudnn.deterministic = bool(det)
    model, ddp, opt, precision = build(args, ctx)
    from pytorch_distributed_training_example_amd.ops.cross_entropy import cross_entropy
    from pytorch_distributed_training_example_amd.parallel.reference import average_gradients

    g = torch.Generator(device=dev).manual_seed(100 + ctx.rank)
    is_lm = args.model.startswith("gpt")
    S, T = args.image_size, args.seq_len
    assert B % args.grad_accum == 0, "batch must be divisible by grad-accum"
    in_dtype = torch.bfloat16 if precision in ("bf16", "fp8") else torch.float32
    pool = []
    for _ in range(2):
        if is_lm:
            x = torch.randint(0, 50257, (B, T), device=dev, generator=g)
            y = torch.randint(0, 50257, (B, T), device=dev, generator=g)
        elif args.model == "lenet":
            x = torch.randn(B, 1, 28, 28, device=dev, generator=g)
            y = torch.randint(0, 10, (B,), device=dev, generator=g)
        else:
            x = torch.randn(B, 3, S, S, device=dev, generator=g).to(in_dtype)
            if args.model.startswith("resnet"):
                x = x.contiguous(memory_format=torch.channels_last)
            y = torch.randint(0, 1000, (B,), device=dev, generator=g)
        pool.append((x, y))
    autocast = precision == "amp_bf16"
    ls = 0.1 if args.model.startswith("resnet") else 0.0

    def loss_of(out, y):
        if args.model == "lenet":  # reference loss: nll_loss on softmax probabilities (train.py:48)
            if args.impl == "ours":
                from pytorch_distributed_training_example_amd.ops.lenet import softmax_nll
                return softmax_nll(out, y, "prob_nll")
            return torch.nn.functional.nll_loss(out, y)
        if is_lm:
            out, y = out.reshape(-1, out.shape[-1]), y.reshape(-1)
        if args.impl == "ours":
            return cross_entropy(out, y, label_smoothing=ls)
        return torch.nn.functional.cross_entropy(out.float(), y, label_smoothing=ls)

    def step(x, y):
        opt.zero_grad(set_to_none=True)
        xs, ys = x.chunk(args.grad_accum), y.chunk(args.grad_accum)
        total = None
        for i, (xm, ym) in enumerate(zip(xs, ys)):
            last = i == len(xs) - 1
            sync = ddp.no_sync() if (not last and hasattr(ddp, "no_sync")) else contextlib.nullcontext()
            with sync:
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
                    out = ddp(xm)
                loss = loss_of(out, ym) / len(xs)
                loss.backward()
            total = loss.detach() if total is None else total + loss.detach()
        if args.impl == "reference" and world > 1:
            average_gradients(model)
        opt.step()
        return total

    runner = None
    if args.impl == "ours" and args.graph:
        from pytorch_distributed_training_example_amd.engine.graph import StaticStep
        runner = StaticStep(step, list(pool[0]), warmup=max(3, min(args.warmup, 5)))

    def run(i):
        x, y = pool[i % 2]
        return runner(x, y) if runner is not None else step(x, y)

    tw = time.perf_counter()
    for i in range(args.warmup):
        loss = run(i)
        if ctx.rank == 0:  # progress (first steps include MIOpen's conv-algorithm search)
            dsync()
            print(f"[bench] warmup step {i + 1}/{args.warmup} done at {time.perf_counter() - tw:.1f}s",
                  file=sys.stderr, flush=True)
    dsync()
    launcher.barrier()
    dsync()
    timing = args.impl == "ours" and runner is None and hasattr(ddp, "enable_comm_timing") and dev.type == "cuda"
    if timing:  # events only (no host sync inside the timed region)
        ddp.enable_comm_timing(True)
    if dev.type == "cuda":
        torch.cuda.nvtx.range_push("timed")
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = run(i)
    dsync()
    launcher.barrier()
    dsync()
    elapsed = time.perf_counter() - t0
    if dev.type == "cuda":
        torch.cuda.nvtx.range_pop()
    exposed = ddp.comm_exposed_ms() if timing else None
    leads = ddp.bucket_ready_lead_ms() if timing else None
    if timing:
        ddp.enable_comm_timing(False)
    # which device every rank bound, as RCCL saw it: one distinct GPU per rank (train.py:138,147 uses
    # every visible GPU, one process each)
    pg_size = dist.get_world_size() if dist.is_initialized() else 1
    dev_idx = torch.tensor([dev.index if dev.type == "cuda" else -1], device=dev, dtype=torch.int64)
    if world > 1:
        gathered = [torch.zeros_like(dev_idx) for _ in range(world)]
        dist.all_gather(gathered, dev_idx)
        rank_devices = [int(t.item()) for t in gathered]
    else:
        rank_devices = [int(dev_idx.item())]
    if dev.type == "cuda" and len(set(rank_devices)) != len(rank_devices):
        raise RuntimeError(f"ranks share GPUs: rank->device {rank_devices}")
    if world > 1:
        t = torch.tensor([elapsed, exposed if exposed is not None else -1.0], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        exposed = float(t[1].item()) if t[1].item() >= 0 else None
    ms = elapsed / args.steps * 1e3
    per_step = B * (T if is_lm else 1)
    value = per_step * world * args.steps / elapsed
    result = {
        "metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "strong" if args.global_batch else "weak", "vs_baseline": None, "dtype": {"fp32": "fp32", "fp8": "fp8_e4m3+bf16"}.get(precision, "bf16"),
        "data": "synthetic (random inputs and labels, random-init weights)",
        "config": {"model": args.model, "global_batch": B * world, "per_gpu_batch": B,
                   "seq_len": T if is_lm else None, "image_size": None if is_lm else S,
                   "parallelism": f"dp{world}", "grad_accum": args.grad_accum, "impl": args.impl,
                   "graph": bool(runner is not None), "precision": precision, "bucket_cap_mb": args.bucket_cap_mb,
                   "comm_hook": args.comm_hook, "reducer_active": bool(getattr(ddp, "_active", lambda: False)()),
                   # exposed (not overlapped) communication per step, max over ranks: the compute stream's
                   # wait on the all-reduces after backward (parallel/ddp.py enable_comm_timing)
                   "comm_exposed_ms": None if exposed is None else round(exposed, 3),
                   "bucket_mb": ([round(b / 2 ** 20, 2) for b in ddp.bucket_bytes()]
                                 if hasattr(ddp, "bucket_bytes") else None),
                   # per bucket (launch order), rank 0: ms between the compute-stream point where the
                   # bucket's all-reduce could start and the end of backward's compute (overlap window)
                   "bucket_ready_lead_ms": None if leads is None else [round(v, 3) for v in leads],
                   "pg_size": pg_size, "pg_backend": dist.get_backend() if dist.is_initialized() else None,
                   "rank_devices": rank_devices,
                   "deterministic": bool(det), "final_loss": round(float(loss.float().item()), 4)},
    }
    return result


def self_launch(args, argv) -> int | None:
    """``--gpus N`` is authoritative: one command uses N GPUs, like the reference's
    ``spawn(..., nprocs=torch.cuda.device_count())`` (/root/reference/train.py:138,147).

    * under a launcher (``WORLD_SIZE`` set): the world size must equal N, else exit non-zero —
      a silent mismatch would report an N-GPU number measured on another rank count;
    * no launcher and N > 1: start ``torch.distributed.run`` with N ranks on 127.0.0.1 as a CHILD
      process (never exec: nothing here has touched the GPU, and the ranks own their devices) and
      return its exit code. Rank 0's JSON line comes out on this process's stdout.
    Returns None when this process should run the benchmark itself."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={env_world}: refusing to report a "
                  f"{env_world}-rank measurement as {args.gpus} GPUs", file=sys.stderr, flush=True)
            return 2
        return None
    if args.gpus <= 1:
        return None
    # device_count() does not initialise HIP on this image (the children bind their own GPUs)
    ngpu = torch.cuda.device_count()
    if ngpu and ngpu < args.gpus and (args.backend in (None, "nccl")):
        print(f"[bench] --gpus {args.gpus} but only {ngpu} visible GPU(s): RCCL needs one GPU per rank",
              file=sys.stderr, flush=True)
        return 2
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(launcher.find_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.setdefault("OMP_NUM_THREADS", "4")
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    rc = self_launch(args, argv)
    if rc is not None:
        return rc
    if os.environ.get("PDT_STACK_DUMP"):  # periodic Python stacks: where a slow warm-up spends time
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["PDT_STACK_DUMP"]), repeat=True)
    ctx = setup(args)
    result = run(args, ctx)
    if ctx.rank == 0:
        print(json.dumps(result), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(result, f)
    launcher.destroy()
    if not math.isfinite(result["config"]["final_loss"]):
        # a step that trains to NaN/inf measures nothing (round 6: a graphed run looked faster while
        # its loss was NaN, profiles/r6/graph_colsum_bwd.txt) — fail the run instead of reporting it
        print(f"[bench] final loss is {result['config']['final_loss']}: the timed steps are not valid",
              file=sys.stderr, flush=True)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
