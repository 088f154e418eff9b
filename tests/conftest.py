import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# MIOpen reads its solver switches once per process: exclude the capture-unsafe solvers before
# any test runs a convolution so the hipGraph tests see the same solver set as bench --graph 1
from pytorch_distributed_training_example_amd.engine.graph import make_miopen_capture_safe  # noqa: E402
from pytorch_distributed_training_example_amd.engine.miopen_cache import use_repo_miopen_cache  # noqa: E402

make_miopen_capture_safe()
use_repo_miopen_cache()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
