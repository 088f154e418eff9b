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


def _load_tool(name):
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(name, os.path.join(root, "tools", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_prof_categories_families():
    """The kernel-family map the committed category tables are built with (tools/prof_categories.py)."""
    f = _load_tool("prof_categories").family
    ns = "(anonymous namespace)::"
    assert f(f"void {ns}conv1x1_kernel<{ns}G1<256, 4, 4>, false, false, false, false, false, true>(unsigned short const*)") \
        .startswith("1x1 GEMM + BN")
    assert f(f"void {ns}conv1x1_kernel<{ns}G1<128, 4, 2>, false, true, false, false, false, false>(unsigned short)") \
        .startswith("our 1x1 conv GEMM")
    assert f(f"void {ns}conv1x1_bwd_fused_kernel<{ns}FB<256, 64, true, false> >({ns}FBArgs)").startswith("fused conv3")
    assert f(f"void {ns}bn_bwd_apply_kernel<true, false, 1>(unsigned short const*)").startswith("our BN")
    assert f(f"{ns}weight_prep_kernel({ns}PrepBatch)") == "batched weight transforms"
    assert f("Cijk_Ailk_Bjlk_BBS_BH_Bias_HA_S_SAV_UserArgs_MT256x128x64").startswith("hipBLASLt")


def test_prof_calls_last_step(tmp_path):
    """tools/prof_calls.py: the last of `steps` equal launch groups inside the marker range, in launch order."""
    d = tmp_path / "trace"
    d.mkdir()
    with open(d / "run_kernel_trace.csv", "w") as f:
        f.write("Kernel_Name,Start_Timestamp,End_Timestamp,Workgroup_Size_X,Grid_Size_X\n")
        t = 1000
        for step in range(2):
            for k in ("void (anonymous namespace)::a_kernel(int)", "b_kernel(float)"):
                f.write(f"\"{k}\",{t},{t + 500 * (step + 1)},256,{256 * 4}\n")
                t += 1000
        f.write(f"\"late_kernel(int)\",{t + 10_000_000},{t + 10_000_500},64,64\n")  # outside the range
    with open(d / "run_marker_api_trace.csv", "w") as f:
        f.write("Function,Start_Timestamp,End_Timestamp\n")
        f.write(f"timed,0,{t + 5}\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "prof_calls.py"), str(d), "timed", "2"],
                         capture_output=True, text=True, check=True).stdout
    rows = [line for line in out.splitlines() if line.startswith("| ") and "`" in line]
    assert len(rows) == 2 and "a_kernel`" in rows[0] and "b_kernel`" in rows[1]
    assert "| 1.0 | 4 | 256 |" in rows[0]  # the second step's 1000-ns launch, 4 workgroups of 256
    assert "2 launches, 0.00 ms busy" in out
