"""Host logic of the native extension under AddressSanitizer + UndefinedBehaviorSanitizer
(csrc/host/host_selftest.cpp, built with the sanitizers on the host half only): multi-tensor launch
metadata packing, the 3x3 weight-gradient tiling / halo bounds (brute force over every tile), the
BatchNorm reduction geometry and the embedding workspace arithmetic. CPU only."""
import os
import shutil
import subprocess

import pytest

pytestmark = pytest.mark.skipif(shutil.which(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")) is None,
                                reason="hipcc not available")


def test_host_selftest_asan_ubsan():
    from pytorch_distributed_training_example_amd import _build
    exe = _build.build_host_selftest()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "all passed" in p.stdout
