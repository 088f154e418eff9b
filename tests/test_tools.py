"""Tool plumbing on CPU: the RCCL bucket-size sweep runs its collective sweep over gloo."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bucket_sweep_collectives_gloo_two_ranks(tmp_path):
    from pytorch_distributed_training_example_amd.parallel.launcher import find_free_port
    out = tmp_path / "sweep.jsonl"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(find_free_port()),
           os.path.join(ROOT, "tools", "bucket_sweep.py"), "--mode", "collectives", "--backend", "gloo",
           "--iters", "2", "--warmup", "1", "--sizes", "4096,262144", "--out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [json.loads(l) for l in out.read_text().splitlines()]
    assert [d["bytes"] for d in rows] == [4096, 262144]
    assert all(d["n_ranks"] == 2 and d["us"] > 0 and d["busbw_GBps"] == d["algbw_GBps"] for d in rows)


def test_bucket_sweep_channel_axis_gloo(tmp_path):
    """--nchannels: one child job per RCCL channel count (NCCL_MIN/MAX_NCHANNELS in its env), every
    JSON line tagged with the count; rehearsed over gloo (the env is simply unused there)."""
    cmd = [sys.executable, os.path.join(ROOT, "tools", "bucket_sweep.py"), "--nproc", "2", "--nchannels", "4,16",
           "--mode", "collectives", "--backend", "gloo", "--iters", "1", "--warmup", "1", "--sizes", "4096"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path),
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(d["nchannels"] for d in rows) == [4, 16]
    assert all(d["n_ranks"] == 2 and d["bytes"] == 4096 for d in rows)
