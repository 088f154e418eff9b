"""Loader for the in-tree gfx950 extension (``_C``).

GPU tensors always go through the HIP kernels: if the extension is missing or fails to load,
GPU calls raise immediately (no silent eager/PyTorch fallback). CPU tensors use the pure
PyTorch reference implementations in each op module (tests on the CPU-only container).
Set ``PDT_DISABLE_NATIVE=1`` to force the reference path (A/B benchmarking only).
"""
from __future__ import annotations

import importlib

from ..config import SW

_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return _mod
    try:
        import torch  # noqa: F401  (libc10 / libtorch must be loaded first)
        _mod = importlib.import_module("pytorch_distributed_training_example_amd._C")
        import os
        if os.environ.get("PDT_BN_TILES_FUSED", "1") == "0":  # A/B: the two-launch BN tile finalize
            _mod.bn_tiles_fused(0)
        if os.environ.get("PDT_POOL_BWD_V2", "1") == "0":  # A/B: the per-position max-pool gradient kernel
            _mod.maxpool_bwd_v2(0)
        if os.environ.get("PDT_BN_APPLY_WGS"):  # A/B: one grid cap (workgroups per CU) for every BN apply pass
            _mod.bn_apply_wgs(int(os.environ["PDT_BN_APPLY_WGS"]))
        if os.environ.get("PDT_CONV1X1_PROBE"):  # A/B / diagnosis only (conv1x1.hip ApArgs::probe)
            _mod.conv1x1_probe(int(os.environ["PDT_CONV1X1_PROBE"]))
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e
    return _mod


def available() -> bool:
    return _load() is not None


_CUDA_OK: list = []


def cuda_available() -> bool:
    """``torch.cuda.is_available()``, asked once per process: it re-enumerates the devices on every call
    (~130 us on the MI355X box), and the optimizer / DDP reducer asked it every step (cProfile of the
    LeNet eager step, round 4)."""
    if not _CUDA_OK:
        import torch
        _CUDA_OK.append(torch.cuda.is_available())
    return _CUDA_OK[0]


def disabled() -> bool:
    return SW.disable_native


def native():
    """The extension module, or a RuntimeError explaining how to build it."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "pytorch_distributed_training_example_amd._C (gfx950 HIP kernels) is not built or failed to "
            f"load: {_err!r}. Build it with `python -m pytorch_distributed_training_example_amd._build`.")
    return m


def use_native(*tensors) -> bool:
    """True when these tensors must take the HIP path (any on GPU and native not disabled)."""
    on_gpu = any(t is not None and getattr(t, "is_cuda", False) for t in tensors)
    if not on_gpu:
        return False
    if disabled():
        return False
    native()  # raise loudly if missing
    return True
