import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# the ALG backward paths at the tests' small batches too (by default they need >= 50176 output pixels per conv)
os.environ.setdefault("PDT_BWD_ALG_MIN_M", "0")
# MIOpen reads its solver switches once per process: exclude the capture-unsafe solvers before
# any test runs a convolution so the hipGraph tests see the same solver set as bench --graph 1
from pytorch_distributed_training_example_amd.engine.graph import make_miopen_capture_safe  # noqa: E402
from pytorch_distributed_training_example_amd.engine.miopen_cache import use_repo_miopen_cache  # noqa: E402

make_miopen_capture_safe()
use_repo_miopen_cache()


@pytest.fixture(autouse=True)
def _reload_switches():
    """Switches are read once per process (config.SW): re-read them after every test so a test's
    env changes (monkeypatch, undone at teardown) never leak into the next one."""
    yield
    from pytorch_distributed_training_example_amd.config import SW
    SW.reload()


@pytest.fixture
def switch(monkeypatch):
    """switch("PDT_X", "v"): set a PDT_* switch for this test (env + config.SW reload)."""
    from pytorch_distributed_training_example_amd.config import SW

    def set_(name, value):
        monkeypatch.setenv(name, value)
        SW.reload()
    yield set_
    monkeypatch.undo()
    SW.reload()


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
