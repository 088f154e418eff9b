"""Command-line training driver (``python train.py ...``).

Reference CLI (/root/reference/train.py:113-133): ``--batch-size`` (GLOBAL, default 1024),
``--epochs`` (20), ``--lr`` (0.1), ``--gamma`` (0.9), ``--no-cuda``, ``--dry-run``, ``--seed`` (5),
``--log-interval`` (15), ``--save-model``. All nine are kept with identical names, defaults and
meaning; running with no flags trains the reference's LeNet on MNIST (real IDX files under
``./data`` if present, else deterministic synthetic MNIST) with Adadelta + StepLR on every
visible GPU, prints the reference's log lines and, with ``--save-model``, writes
``mnist_cnn.pt`` in the reference's format.

Launch: one process per GPU. Under ``torchrun`` (RANK/WORLD_SIZE in the env) the process
trains directly; otherwise it spawns ``--world-size`` ranks itself (default: all visible
GPUs), like the reference's ``spawn`` (train.py:138-147). Without a GPU the reference exits
(train.py:139-142); here it trains on CPU with gloo instead.
"""
from __future__ import annotations

import argparse
import math
import os
import sys
from typing import Optional

import torch

from .parallel import launcher


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X-native distributed training (PyTorch MNIST Example superset)")
    # --- the reference's nine flags (train.py:113-133) ---
    p.add_argument("--batch-size", type=int, default=1024, metavar="N",
                   help="GLOBAL input batch size for training (default: 1024)")
    p.add_argument("--epochs", type=int, default=20, metavar="N", help="number of epochs to train (default: 20)")
    p.add_argument("--lr", type=float, default=1e-1, metavar="LR", help="learning rate (default: 0.1)")
    p.add_argument("--gamma", type=float, default=0.9, metavar="M", help="Learning rate step gamma (default: 0.9)")
    p.add_argument("--no-cuda", action="store_true", default=False, help="disables GPU training")
    p.add_argument("--dry-run", action="store_true", default=False, help="quickly check a single pass")
    p.add_argument("--seed", type=int, default=5, metavar="S", help="random seed (default: 5)")
    p.add_argument("--log-interval", type=int, default=15, metavar="N",
                   help="how many batches to wait before logging training status")
    p.add_argument("--save-model", action="store_true", default=False, help="For Saving the current Model")
    # --- extensions ---
    p.add_argument("--model", default="lenet", help="lenet | mlp | resnet50 | resnet18 | vit_b16 | gpt2_medium | ...")
    p.add_argument("--world-size", type=int, default=None, help="ranks to spawn (default: visible GPUs, 1 on CPU)")
    p.add_argument("--backend", default=None, help="nccl (RCCL) | gloo")
    p.add_argument("--loss", default=None, help="cross_entropy | nll_on_probs (reference) | prob_nll (reference loss from logits) | mse")
    p.add_argument("--optimizer", default=None, help="adadelta | sgd | adamw | adam")
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--weight-decay", type=float, default=0.0)
    p.add_argument("--scheduler", default="step", help="step (StepLR per epoch) | cosine | none")
    p.add_argument("--precision", default="fp32", help="fp32 | bf16 | fp8 (transformer GEMMs) | amp_bf16 | amp_fp16")
    p.add_argument("--grad-accum", type=int, default=1, help="micro-batches per optimizer step (no_sync)")
    p.add_argument("--clip-grad", type=float, default=0.0)
    p.add_argument("--reducer", default="ddp", help="ddp (ours) | torch_ddp | reference (per-param)")
    p.add_argument("--bucket-cap-mb", type=float, default=25.0)
    p.add_argument("--sharding", default="split", help="split (reference SplitDataset) | sampler (DistributedSampler)")
    p.add_argument("--loader", default="resident", help="resident (whole shard in HBM) | reference (DataLoader)")
    p.add_argument("--synthetic", default="auto", help="auto | yes | no (MNIST source)")
    p.add_argument("--data-dir", default="./data")
    p.add_argument("--train-samples", type=int, default=None, help="synthetic dataset size override")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--seq-len", type=int, default=1024)
    p.add_argument("--steps-per-epoch", type=int, default=None)
    p.add_argument("--no-eval-reduce", action="store_true", help="reference eval: rank 0 reports its own shard")
    p.add_argument("--no-eval", action="store_true")
    p.add_argument("--save-path", default="mnist_cnn.pt")
    p.add_argument("--checkpoint", default=None, help="full resume checkpoint path (written every epoch)")
    p.add_argument("--resume", action="store_true", help="resume from --checkpoint if it exists")
    p.add_argument("--metrics", default=None, help="JSONL metrics path (rank 0)")
    p.add_argument("--check-sync", action="store_true", help="verify replicas are identical after each epoch")
    p.add_argument("--channels-last", action="store_true")
    p.add_argument("--timeout", type=float, default=600.0, help="process-group timeout (s)")
    p.add_argument("--amp", default=None, choices=["off", "bf16", "fp8"],
                   help="alias: off=fp32, bf16=bf16 params+fp32 master, fp8=bf16+e4m3 transformer GEMMs")
    p.add_argument("--hipgraph", action="store_true",
                   help="replay each train step as one hipGraph (static shapes; MIOpen capture-safe solvers)")
    p.add_argument("--profile", default=None, metavar="DIR",
                   help="torch.profiler trace of a few steps of epoch 1 into DIR (rank 0), roctx ranges on")
    return p


MODEL_DEFAULTS = {
    # the reference's loss: nll_loss on softmax probabilities (train.py:48), values in [-1, 0];
    # computed from the logits by one fused kernel (--loss cross_entropy for the usual loss)
    "lenet": dict(optimizer="adadelta", loss="nll_on_probs"),
    "mlp": dict(optimizer="sgd", loss="mse"),
}


def _datasets(args, rank, world):
    from .data import RandomTensorDataset, mnist
    if args.model == "lenet":
        syn = {"auto": None, "yes": True, "no": False}[args.synthetic]
        tr = mnist(args.data_dir, True, synthetic=syn, n=args.train_samples, seed=0)
        te = mnist(args.data_dir, False, synthetic=syn, n=(args.train_samples // 6 if args.train_samples else None),
                   seed=0)
        return tr, te
    if args.model == "mlp":
        return RandomTensorDataset(args.train_samples or 4096, seed=0), RandomTensorDataset(512, seed=1)
    return None, None


def _shard(ds, args, rank, world, shuffle=True):
    from .parallel import DistributedSampler, rank_partition
    if ds is None:
        return None, None
    if args.sharding == "sampler":
        return ds, DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=shuffle, seed=args.seed)
    return rank_partition(ds, rank, world), None


def _loader(ds, sampler, per_rank_batch, args, device, shuffle=True, seed=0):
    from .data import ResidentLoader, reference_loader
    if args.loader == "resident" and sampler is None and hasattr(getattr(ds, "dataset", ds), "tensors"):
        base = getattr(ds, "dataset", ds)
        x, y = base.tensors()
        off = ds.offset() if hasattr(ds, "offset") else 0
        n = len(ds)
        return ResidentLoader(x[off:off + n], y[off:off + n], per_rank_batch, device, shuffle=shuffle, seed=seed)
    return reference_loader(ds, per_rank_batch, shuffle=shuffle, sampler=sampler,
                            num_workers=0 if device.type == "cpu" else 4,
                            pin_memory=device.type == "cuda")


def run(rank: int, world: int, args) -> dict:
    from .engine.checkpoint import load_checkpoint, save_checkpoint, save_model
    from .engine.trainer import StepConfig, TrainStep, evaluate, make_loss_fn, train_epoch
    from .models import get_model
    from .models.precision import apply_precision
    from .optim import build_optimizer, build_scheduler
    from .parallel import DistributedDataParallel
    from .parallel.debug import check_replicas_in_sync
    from .utils.metrics import MetricsWriter

    ctx = launcher.context()
    device = ctx.device
    torch.manual_seed(args.seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(args.seed)
    defaults = MODEL_DEFAULTS.get(args.model, dict(optimizer="sgd", loss="cross_entropy"))
    loss_kind = args.loss or defaults["loss"]
    opt_name = args.optimizer or defaults["optimizer"]
    per_rank = math.ceil(args.batch_size / world)  # reference: ceil(global / world) (train.py:82)

    if args.model == "lenet":
        if loss_kind == "nll_on_probs":
            # the reference's loss (nll on softmax probabilities, train.py:48), computed from the
            # logits by one fused kernel: identical values, no separate softmax round trip
            loss_kind = "prob_nll"
        model = get_model("lenet", output="logits")
    else:
        model = get_model(args.model)
    model = model.to(device)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    model = apply_precision(model, args.precision)

    if args.reducer == "ddp" and world >= 1 and launcher.context().distributed:
        wrapped = DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb)
    elif args.reducer == "torch_ddp" and launcher.context().distributed:
        wrapped = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[device.index] if device.type == "cuda" else None, bucket_cap_mb=args.bucket_cap_mb)
    else:
        wrapped = model
    opt_kw = {}
    if opt_name == "sgd":
        opt_kw = dict(momentum=args.momentum, weight_decay=args.weight_decay)
    elif opt_name in ("adamw", "adam", "adadelta"):
        opt_kw = dict(weight_decay=args.weight_decay)
    optimizer = build_optimizer(opt_name, model.parameters(), lr=args.lr, **opt_kw)
    scheduler = build_scheduler(args.scheduler, optimizer, gamma=args.gamma, step_size=1,
                                total_steps=args.epochs)
    scaler = None
    if args.precision == "amp_fp16":
        from .engine.amp import GradScaler
        scaler = GradScaler(device=str(device))
    step = TrainStep(wrapped, optimizer, make_loss_fn(loss_kind),
                     StepConfig(precision=args.precision, grad_accum=args.grad_accum,
                                reducer=args.reducer if launcher.context().distributed else "none",
                                clip_grad=args.clip_grad), scaler=scaler, raw_model=model)
    if args.hipgraph and device.type == "cuda":
        step.enable_graph()

    train_ds, test_ds = _datasets(args, rank, world)
    train_shard, train_sampler = _shard(train_ds, args, rank, world)
    test_shard, test_sampler = _shard(test_ds, args, rank, world, shuffle=False)
    in_dtype = torch.bfloat16 if args.precision in ("bf16", "fp8") else None
    if train_shard is not None:
        train_loader = _loader(train_shard, train_sampler, per_rank, args, device, seed=args.seed + rank)
        test_loader = _loader(test_shard, test_sampler, per_rank, args, device, shuffle=False)
    else:
        from .data import SyntheticBatches
        steps = args.steps_per_epoch or 10
        if args.model.startswith("gpt"):
            train_loader = SyntheticBatches((per_rank, args.seq_len), 50257, steps, device, seed=args.seed + rank,
                                            int_inputs=True)
        else:
            train_loader = SyntheticBatches((per_rank, 3, args.image_size, args.image_size), 1000, steps, device,
                                            dtype=in_dtype or torch.float32, channels_last=args.channels_last,
                                            seed=args.seed + rank)
        test_loader = None

    start_epoch = 1
    if args.checkpoint and args.resume and os.path.exists(args.checkpoint):
        ck = load_checkpoint(args.checkpoint, model, optimizer, scheduler, scaler, sampler=train_sampler,
                             map_location=device)
        start_epoch = int(ck["epoch"]) + 1
        if rank == 0:
            print(f"resumed from {args.checkpoint} at epoch {start_epoch}", flush=True)
    metrics = MetricsWriter(args.metrics, rank)
    from .parallel.fault import FaultInjector
    injector = FaultInjector(rank=rank)
    gstep = [0]

    prof = None
    if args.profile and rank == 0:
        from .utils.profiling import torch_profiler
        prof = torch_profiler(args.profile)
        prof.__enter__()

    def on_step(epoch, batch_idx):
        gstep[0] += 1
        injector.maybe_fail(gstep[0])
        if prof is not None:
            prof.step()

    result = {}
    for epoch in range(start_epoch, args.epochs + 1):
        if train_sampler is not None:
            train_sampler.set_epoch(epoch)
        if hasattr(train_loader, "set_epoch"):
            train_loader.set_epoch(epoch)
        stats = train_epoch(step, train_loader, device, epoch, args.log_interval, args.dry_run, rank, metrics,
                            max_steps=args.steps_per_epoch, input_dtype=in_dtype, channels_last=args.channels_last,
                            on_step=on_step)
        result["train"] = stats
        metrics.log({"event": "epoch", "epoch": epoch, **stats})
        if test_loader is not None and not args.no_eval:
            result["eval"] = evaluate(wrapped, test_loader, device, loss_kind, rank,
                                      reduce_across_ranks=not args.no_eval_reduce, input_dtype=in_dtype,
                                      channels_last=args.channels_last)
            metrics.log({"event": "eval", "epoch": epoch, **result["eval"]})
        scheduler.step()
        if args.check_sync:
            check_replicas_in_sync(list(model.parameters()))
        if args.checkpoint:
            save_checkpoint(args.checkpoint, model, optimizer, scheduler, scaler, train_sampler, epoch=epoch)
    if prof is not None:
        prof.__exit__(None, None, None)
        print(f"profiler trace written to {args.profile}", flush=True)
    if args.save_model:
        save_model(model, args.save_path, rank)
    metrics.close()
    return result


def configure_process(args) -> None:
    """Per-rank library settings, applied once LOCAL_RANK is known and before the first conv or
    GEMM: MIOpen's in-tree find-db (local rank 0 only; other ranks get private copies) and the
    measured GEMM table copied for THIS rank's device. Called in each rank, never in a
    spawning parent, whose environment every child would inherit."""
    from .engine.miopen_cache import use_repo_miopen_cache
    use_repo_miopen_cache()  # persisted conv-algorithm find-db (engine/miopen_cache.py)
    from .engine.gemm_tuning import use_repo_gemm_tuning, wants_gemm_tuning
    if wants_gemm_tuning(args.model, args.grad_accum, getattr(args, "hipgraph", False)):
        use_repo_gemm_tuning()  # measured GEMM solutions (engine/gemm_tuning.py), read-only


def _entry(rank: int, world: int, args) -> None:
    configure_process(args)
    run(rank, world, args)


def main(argv: Optional[list] = None) -> int:
    args = build_parser().parse_args(argv)
    if args.amp is not None:
        args.precision = {"off": "fp32", "bf16": "bf16", "fp8": "fp8"}[args.amp]
    if args.hipgraph:
        # MIOpen reads its solver switches once per process: set before any convolution
        from .engine.graph import make_miopen_capture_safe
        make_miopen_capture_safe()
    if args.profile:
        from .utils import profiling
        profiling.enable_ranges(True)
    use_gpu = not args.no_cuda and torch.cuda.is_available()
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:  # torchrun
        configure_process(args)
        ctx = launcher.init_distributed(backend=args.backend, use_gpu=use_gpu, timeout_s=args.timeout)
        try:
            run(ctx.rank, ctx.world_size, args)
        finally:
            launcher.destroy()
        return 0
    if args.world_size is not None:
        world = args.world_size
    elif use_gpu:
        world = torch.cuda.device_count()
    else:
        print("No available GPU instance! Training on CPU with gloo.", flush=True)
        world = 1
    backend = args.backend or ("nccl" if use_gpu else "gloo")
    launcher.spawn(_entry, world, args=(args,), backend=backend, use_gpu=use_gpu, timeout_s=args.timeout)
    return 0


if __name__ == "__main__":
    sys.exit(main())
