"""MI355X-native distributed data-parallel training framework.

Capabilities of ownzonefeng/pytorch-distributed-training-example,
re-designed for AMD Instinct MI355X (gfx950): one process per GPU over RCCL/xGMI, a
bucketed backward-overlapped DDP reducer, hand-written HIP/CDNA4 kernels for the per-step
hot path, hipGraph step capture.
"""
__version__ = "0.1.0"

from . import parallel  # noqa: F401
