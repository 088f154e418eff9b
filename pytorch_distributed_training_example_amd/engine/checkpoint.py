"""Checkpointing: reference-compatible model save + full resume checkpoints.

Reference: rank 0 saves ``torch.save(model.state_dict(), "mnist_cnn.pt")`` once after the last
epoch; no optimizer/scheduler/RNG state, no load path (/root/reference/train.py:107-108).

Here:
  * ``save_model`` writes exactly that format (plain state_dict of the *unwrapped* module, so
    keys are ``ConvNet.1.weight`` … with no ``module.`` prefix) — files interchange with the
    reference's and with torchvision/torch-DDP checkpoints;
  * ``load_model`` accepts plain or ``module.``-prefixed (torch DDP) state_dicts, with
    ``weights_only=True`` (never unpickles code);
  * ``save_checkpoint`` / ``load_checkpoint`` add optimizer (torch-compatible layout),
    scheduler, grad scaler, epoch/step, sampler position and RNG states for exact resume;
    rank 0 writes atomically (tmp + rename), every rank then barriers.
"""
from __future__ import annotations

import os
import random
from typing import Any, Dict, Optional

import numpy as np
import torch
from torch import nn

from ..parallel import launcher
from ..parallel.ddp import unwrap


def _unwrapped_state(model: nn.Module) -> Dict[str, torch.Tensor]:
    m = unwrap(model)
    for mod in m.modules():
        if hasattr(mod, "sync_num_batches_tracked"):
            mod.sync_num_batches_tracked()
    return m.state_dict()


def strip_prefix(sd: Dict[str, Any], prefix: str = "module.") -> Dict[str, Any]:
    if sd and all(k.startswith(prefix) for k in sd):
        return {k[len(prefix):]: v for k, v in sd.items()}
    return sd


def save_model(model: nn.Module, path: str = "mnist_cnn.pt", rank: Optional[int] = None) -> None:
    """Reference format: plain state_dict of the unwrapped model, written by rank 0."""
    rank = launcher.get_rank() if rank is None else rank
    if rank == 0:
        sd = {k: v.detach().cpu() for k, v in _unwrapped_state(model).items()}
        tmp = path + ".tmp"
        torch.save(sd, tmp)
        os.replace(tmp, path)


def load_model(model: nn.Module, path: str, strict: bool = True, map_location="cpu"):
    sd = torch.load(path, map_location=map_location, weights_only=True)
    sd = strip_prefix(sd)
    return unwrap(model).load_state_dict(sd, strict=strict)


def rng_state() -> Dict[str, Any]:
    name, keys, pos, has_gauss, cached = np.random.get_state()
    st = {"python": random.getstate(), "numpy": (name, keys.tolist(), int(pos), int(has_gauss), float(cached)),
          "torch": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st: Dict[str, Any]) -> None:
    random.setstate(st["python"])
    name, keys, pos, has_gauss, cached = st["numpy"]
    np.random.set_state((name, np.asarray(keys, dtype=np.uint32), pos, has_gauss, cached))
    torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


def save_checkpoint(path: str, model: nn.Module, optimizer=None, scheduler=None, scaler=None,
                    sampler=None, epoch: int = 0, step: int = 0, extra: Optional[dict] = None) -> None:
    rank = launcher.get_rank()
    if rank == 0:
        ck = {
            "format": "pdt-amd-ckpt-v1",
            "model": {k: v.detach().cpu() for k, v in _unwrapped_state(model).items()},
            "optimizer": optimizer.state_dict() if optimizer is not None else None,
            "scheduler": scheduler.state_dict() if scheduler is not None else None,
            "scaler": scaler.state_dict() if scaler is not None else None,
            "sampler": sampler.state_dict() if sampler is not None and hasattr(sampler, "state_dict") else None,
            "epoch": epoch,
            "step": step,
            "world_size": launcher.get_world_size(),
            "rng": rng_state(),
            "extra": extra or {},
        }
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        torch.save(ck, tmp)
        os.replace(tmp, path)
    launcher.barrier()


def load_checkpoint(path: str, model: nn.Module, optimizer=None, scheduler=None, scaler=None, sampler=None,
                    map_location="cpu", restore_rng: bool = True) -> Dict[str, Any]:
    ck = torch.load(path, map_location=map_location, weights_only=True)
    unwrap(model).load_state_dict(strip_prefix(ck["model"]))
    if optimizer is not None and ck.get("optimizer") is not None:
        optimizer.load_state_dict(ck["optimizer"])
    if scheduler is not None and ck.get("scheduler") is not None:
        scheduler.load_state_dict(ck["scheduler"])
    if scaler is not None and ck.get("scaler") is not None:
        scaler.load_state_dict(ck["scaler"])
    if sampler is not None and ck.get("sampler") is not None and hasattr(sampler, "load_state_dict"):
        sampler.load_state_dict(ck["sampler"])
    if restore_rng and ck.get("rng") is not None:
        try:
            set_rng_state(ck["rng"])
        except Exception:
            pass
    return ck
