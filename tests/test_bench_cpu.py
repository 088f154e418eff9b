"""bench.py driver contract, rehearsed on CPU/gloo: the launch line the driver uses
(torch.distributed.run, 127.0.0.1, one rank per device), one JSON line from rank 0 with the
whole-job aggregate, the BASELINE.json metric and the dp<N> parallelism tag."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _run(nproc, port, extra=(), self_launch=False):
    env = dict(os.environ, OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    args = ["--steps", "2", "--warmup", "1", "--image-size", "32", *extra]
    if not any(a in ("--batch-size", "--global-batch") for a in extra):
        args += ["--batch-size", "2"]
    if nproc == 1 or self_launch:
        cmd = [sys.executable, "bench.py", "--gpus", str(nproc), *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", f"--master-port={port}", "bench.py", "--gpus", str(nproc), *args]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("nproc,port", [(1, 0), (4, 29671)])
def test_bench_json_contract(nproc, port):
    r = _run(nproc, port)
    assert KEYS <= set(r)
    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert r["metric"] == baseline["metric"]
    assert r["n_gpus"] == nproc and r["steps"] == 2 and r["warmup"] == 1
    assert r["config"]["model"] == "resnet50" and r["config"]["parallelism"] == f"dp{nproc}"
    assert r["config"]["global_batch"] == 2 * nproc
    assert r["scaling"] == "weak" and r["higher_is_better"] is True and r["dtype"] == "bf16"
    # value is the whole-job aggregate derived from the (max over ranks) step time
    assert r["value"] == pytest.approx(2 * nproc / (r["ms_per_step"] / 1e3), rel=1e-2)


def test_bench_gpus_flag_self_launches():
    """``python bench.py --gpus 4`` (no launcher) must run 4 ranks itself, like the reference's one
    command that uses every GPU (train.py:138,147)."""
    r = _run(4, 0, self_launch=True)
    assert r["n_gpus"] == 4 and r["config"]["parallelism"] == "dp4"
    assert r["config"]["global_batch"] == 8


def test_bench_world_size_mismatch_refused():
    env = dict(os.environ, OMP_NUM_THREADS="2", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "1", "--warmup", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=200)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_global_batch_strong_scaling():
    """--global-batch G: per-rank ceil(G/N) (train.py:82), reported as strong scaling."""
    r = _run(2, 0, extra=("--global-batch", "5"), self_launch=True)
    assert r["scaling"] == "strong" and r["config"]["per_gpu_batch"] == 3
    assert r["config"]["global_batch"] == 6 and r["n_gpus"] == 2


def test_bench_fails_on_non_finite_loss():
    """A run whose loss ends NaN is not a measurement: bench.py exits 3 (round 6: a graphed run looked
    faster while training to NaN, profiles/r6/graph_colsum_bwd.txt)."""
    env = dict(os.environ, OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "bench.py", "--model", "lenet", "--steps", "3", "--warmup", "2",
                        "--lr", "1e30"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "not valid" in p.stderr
