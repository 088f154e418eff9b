"""Train / eval loops (reference-compatible output) and the step function.

Reference: ``train()`` (/root/reference/train.py:42-57) — per batch: H2D copy, zero_grad,
forward, ``F.nll_loss``, backward, per-parameter gradient averaging, ``optimizer.step()``,
rank-0 log every ``log_interval`` batches, ``--dry-run`` breaks after one batch;
``test()`` (train.py:60-76) — no_grad eval with per-batch ``.item()`` syncs, rank 0 prints
only its own shard's metrics.

Here the same loops and the same log lines, plus:
  * the step goes through the bucketed/overlapped DDP reducer (or the reference's
    per-parameter algorithm when ``reducer='reference'``);
  * gradient accumulation with ``no_sync`` (communication only on the last micro-batch);
  * AMP (bf16 autocast or bf16 params + fp32 master weights; fp16 with a device loss scaler);
  * eval metrics accumulate on the device and are all-reduced across ranks (one host sync
    per epoch); ``eval_reduce=False`` reproduces the reference's rank-0-shard-only report;
  * per-step timing, throughput and JSONL metrics (utils/metrics.py).
"""
from __future__ import annotations

import contextlib
import time
from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist
from torch import nn

from ..ops.cross_entropy import cross_entropy, nll_on_probs
from ..ops.lenet import eval_metrics_, softmax_nll
from ..parallel import launcher
from ..parallel.reference import average_gradients
from ..utils.profiling import range as prof_range
from .amp import autocast_ctx


def make_loss_fn(kind: str) -> Callable[[torch.Tensor, torch.Tensor], torch.Tensor]:
    if kind == "nll_on_probs":  # reference: softmax output + nll_loss (train.py:48)
        return lambda out, y: nll_on_probs(out.float(), y)
    if kind == "prob_nll":  # the reference's loss computed from logits (ops/lenet.py, one fused kernel)
        return lambda out, y: softmax_nll(out, y, "prob_nll")
    if kind == "cross_entropy":
        # small class counts (LeNet's 10): one wave per row, loss and gradient in one pass
        return lambda out, y: softmax_nll(out, y, "ce") if out.dim() == 2 and out.shape[-1] <= 64 \
            else cross_entropy(out, y)
    if kind.startswith("cross_entropy_ls"):
        ls = float(kind.split("=")[1]) if "=" in kind else 0.1
        return lambda out, y: cross_entropy(out, y, label_smoothing=ls)
    if kind == "mse":
        return lambda out, y: nn.functional.mse_loss(out.float(), y.float())
    raise ValueError(kind)


@dataclass
class StepConfig:
    precision: str = "fp32"          # fp32 | bf16 (params bf16 + fp32 master) | amp_bf16 | amp_fp16
    grad_accum: int = 1
    reducer: str = "ddp"             # ddp | torch_ddp | reference | none
    clip_grad: float = 0.0


class TrainStep:
    """One optimizer step over ``grad_accum`` micro-batches."""

    def __init__(self, model: nn.Module, optimizer, loss_fn, cfg: StepConfig, scaler=None, raw_model=None):
        self.model = model
        self.raw_model = raw_model if raw_model is not None else model
        self.opt = optimizer
        self.loss_fn = loss_fn
        self.cfg = cfg
        self.scaler = scaler

        self._graphs = None  # {input signature: StaticStep} when hipGraph mode is on

    def zero_grad(self):
        self.opt.zero_grad(set_to_none=True)

    def enable_graph(self, warmup: int = 3) -> None:
        """Replay the whole step (forward, backward, bucket all-reduces, optimizer) as one hipGraph
        per input shape (engine/graph.py). Host-side lr changes are pushed to the optimizer's
        device lr tensors before each replay."""
        self._graphs = {}
        self._graph_warmup = warmup

    def __call__(self, xs, ys) -> torch.Tensor:
        """xs/ys: a tensor (one micro-batch) or a list of micro-batches."""
        if self._graphs is not None and torch.is_tensor(xs) and xs.is_cuda:
            return self._replay(xs, ys)
        return self._eager(xs, ys)

    def _replay(self, x, y) -> torch.Tensor:
        from .graph import StaticStep
        key = (tuple(x.shape), x.dtype, tuple(y.shape), y.dtype)
        runner = self._graphs.get(key)
        if runner is None:
            runner = StaticStep(self._eager, [x, y], warmup=self._graph_warmup)
            self._graphs[key] = runner
        if hasattr(self.opt, "sync_lr"):
            self.opt.sync_lr()
        return runner(x, y)

    def _eager(self, xs, ys) -> torch.Tensor:
        if torch.is_tensor(xs):
            xs, ys = [xs], [ys]
        self.zero_grad()
        n = len(xs)
        total = None
        for i, (x, y) in enumerate(zip(xs, ys)):
            last = i == n - 1
            ctx = self.model.no_sync() if (not last and hasattr(self.model, "no_sync")) else contextlib.nullcontext()
            with ctx:
                with prof_range("forward"), autocast_ctx(self.cfg.precision):
                    out = self.model(x)
                    loss = self.loss_fn(out, y)
                l = loss / n if n > 1 else loss
                with prof_range("backward"):  # includes the overlapped bucket all-reduces
                    (self.scaler.scale(l) if self.scaler is not None else l).backward()
            total = loss.detach() if total is None else total + loss.detach()
        if self.cfg.reducer == "reference" and launcher.get_world_size() > 1:
            average_gradients(self.raw_model)
        if self.cfg.clip_grad > 0:
            from ..ops.multi_tensor import clip_grad_norm_
            if self.scaler is not None:
                self.scaler.unscale_(self.opt)
            clip_grad_norm_([p.grad for p in self.raw_model.parameters() if p.grad is not None], self.cfg.clip_grad)
        with prof_range("optimizer"):
            if self.scaler is not None:
                self.scaler.step(self.opt)
                self.scaler.update()
            else:
                self.opt.step()
        return total / n


def train_epoch(step: TrainStep, loader, device, epoch: int, log_interval: int = 15, dry_run: bool = False,
                rank: Optional[int] = None, metrics=None, max_steps: Optional[int] = None,
                input_dtype: Optional[torch.dtype] = None, channels_last: bool = False,
                on_step: Optional[Callable[[int, int], None]] = None) -> dict:
    """Reference-compatible train loop (log line format of train.py:52-55).

    ``on_step(epoch, batch_idx)`` runs after every optimizer step (fault injection, profiling)."""
    rank = launcher.get_rank() if rank is None else rank
    step.model.train()
    nb = len(loader)
    t0 = time.perf_counter()
    seen = 0
    for batch_idx, (data, target) in enumerate(loader):
        data = data.to(device, non_blocking=True)
        target = target.to(device, non_blocking=True)
        if input_dtype is not None and data.is_floating_point():
            data = data.to(input_dtype)
        if channels_last and data.dim() == 4:
            data = data.contiguous(memory_format=torch.channels_last)
        if step.cfg.grad_accum > 1:
            xs, ys = list(data.chunk(step.cfg.grad_accum)), list(target.chunk(step.cfg.grad_accum))
        else:
            xs, ys = data, target
        loss = step(xs, ys)
        seen += data.shape[0]
        if on_step is not None:
            on_step(epoch, batch_idx)
        if batch_idx % log_interval == 0 and rank == 0:
            print("Train Epoch: {} [{}/{} ({:.0f}%)]\tLoss: {:.6f}".format(
                epoch, batch_idx * len(data), len(loader.dataset), 100.0 * batch_idx / nb, loss.item()),
                flush=True)
            if metrics is not None:
                metrics.log({"event": "train", "epoch": epoch, "batch": batch_idx, "loss": float(loss.item()),
                             "lr": float(step.opt.param_groups[0]["lr"])})
        if dry_run or (max_steps is not None and batch_idx + 1 >= max_steps):
            break
    if torch.cuda.is_available() and str(device).startswith("cuda"):
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"samples": seen, "seconds": dt, "samples_per_sec": seen / max(dt, 1e-9)}


@torch.no_grad()
def evaluate(model: nn.Module, loader, device, loss_kind: str = "cross_entropy", rank: Optional[int] = None,
             reduce_across_ranks: bool = True, print_result: bool = True, input_dtype=None,
             channels_last: bool = False, autocast: str = "fp32") -> dict:
    """Reference-compatible eval (train.py:60-76) with on-device accumulation."""
    rank = launcher.get_rank() if rank is None else rank
    model.eval()
    dev = torch.device(device)
    acc = torch.zeros(3, dtype=torch.float64, device=dev)  # loss_sum, correct, count
    for data, target in loader:
        data, target = data.to(dev, non_blocking=True), target.to(dev, non_blocking=True)
        if input_dtype is not None and data.is_floating_point():
            data = data.to(input_dtype)
        if channels_last and data.dim() == 4:
            data = data.contiguous(memory_format=torch.channels_last)
        with autocast_ctx(autocast):
            out = model(data)
        if loss_kind in ("cross_entropy", "prob_nll") and out.dim() == 2 and out.shape[-1] <= 1024:
            # fused on-device loss-sum / correct / count (one kernel, no per-batch sync)
            eval_metrics_(acc, out, target, "ce" if loss_kind == "cross_entropy" else "prob_nll")
            continue
        if loss_kind == "nll_on_probs":
            l = nll_on_probs(out.float(), target, reduction="sum")
        else:
            l = cross_entropy(out, target, reduction="sum")
        pred = out.argmax(dim=1)
        acc[0] += l.double()
        acc[1] += (pred == target).sum().double()
        acc[2] += target.numel()
    local_n = float(len(loader.dataset))
    if reduce_across_ranks and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(acc)
        n = float(acc[2].item())
    else:
        n = local_n
    loss_sum, correct = float(acc[0].item()), int(acc[1].item())
    res = {"loss": loss_sum / max(n, 1), "correct": correct, "total": int(n), "accuracy": correct / max(n, 1)}
    if print_result and rank == 0:
        print("\nTest set on {}: Average loss: {:.4f}, Accuracy: {}/{} ({:.0f}%)\n".format(
            rank, res["loss"], correct, int(n), 100.0 * correct / max(n, 1)), flush=True)
    model.train()
    return res
