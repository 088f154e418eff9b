"""GEMM tuning table plumbing (engine/gemm_tuning.py): merge semantics and the read-only
TunableOp environment each rank gets. CPU-only (no GEMM runs)."""
import os

from pytorch_distributed_training_example_amd.engine import gemm_tuning


def _write(path, lines):
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def test_merge_tables_union_later_wins(tmp_path):
    a, b, out = tmp_path / "a.csv", tmp_path / "b.csv", tmp_path / "o" / "m.csv"
    _write(a, ["Validator,PT_VERSION,2.10.0", "GemmTunableOp_BFloat16_TN,tn_1_2_3,Gemm_Hipblaslt_1,0.5",
               "GemmTunableOp_BFloat16_NN,nn_4_5_6,Gemm_Rocblas_2,0.7"])
    _write(b, ["Validator,PT_VERSION,9.9.9", "GemmTunableOp_BFloat16_TN,tn_1_2_3,Gemm_Hipblaslt_9,0.4"])
    assert gemm_tuning.merge_tables([str(a), str(b)], str(out)) == 2
    text = out.read_text().splitlines()
    assert text[0] == "Validator,PT_VERSION,2.10.0" and len([t for t in text if t.startswith("Validator")]) == 1
    assert "GemmTunableOp_BFloat16_TN,tn_1_2_3,Gemm_Hipblaslt_9,0.4" in text
    assert "GemmTunableOp_BFloat16_NN,nn_4_5_6,Gemm_Rocblas_2,0.7" in text


def test_read_only_env_and_per_device_copy(tmp_path, monkeypatch):
    for k in list(os.environ):
        if k.startswith("PYTORCH_TUNABLEOP_") or k.startswith("PDT_TUNE") or k == "PDT_GEMM_TUNING":
            monkeypatch.delenv(k, raising=False)
    table = tmp_path / "t.csv"
    _write(table, ["Validator,PT_VERSION,2.10.0", "GemmTunableOp_BFloat16_TN,tn_1_2_3,Gemm_Hipblaslt_1,0.5"])
    monkeypatch.setattr(gemm_tuning.tempfile, "gettempdir", lambda: str(tmp_path))
    pattern = gemm_tuning.use_repo_gemm_tuning(device_index=3, table=str(table))
    assert pattern is not None and pattern.endswith("tunableop%d.csv")
    assert os.environ["PYTORCH_TUNABLEOP_ENABLED"] == "1"
    assert os.environ["PYTORCH_TUNABLEOP_TUNING"] == "0"  # never searches inside a timed run
    copy = pattern.replace("%d", "3")
    assert open(copy).read() == table.read_text()


def test_disabled_and_explicit_env_win(tmp_path, monkeypatch, switch):
    table = tmp_path / "t.csv"
    _write(table, ["Validator,PT_VERSION,2.10.0"])
    switch("PDT_GEMM_TUNING", "0")
    assert gemm_tuning.use_repo_gemm_tuning(table=str(table)) is None
    monkeypatch.delenv("PDT_GEMM_TUNING")
    monkeypatch.setenv("PYTORCH_TUNABLEOP_ENABLED", "0")
    assert gemm_tuning.use_repo_gemm_tuning(table=str(table)) is None


def test_committed_table_has_validators_and_entries():
    lines = open(gemm_tuning.TABLE).read().splitlines()
    assert any(l.startswith("Validator,GCN_ARCH_NAME,gfx950") for l in lines)
    assert sum(not l.startswith("Validator") for l in lines if l) >= 10


def test_conv1x1_decision_table_roundtrip(tmp_path, monkeypatch):
    """Measured 1x1-conv decisions (ops/conv.py) load from / dump to a JSON table; a key in the
    table is used without timing (no GPU needed to pick)."""
    from pytorch_distributed_training_example_amd.ops import conv as C
    monkeypatch.setattr(C, "_CHOICE", {})
    monkeypatch.setattr(C, "_TABLE_LOADED", [True])
    C._CHOICE[("fwd", "bf16", 802816, 64, 256)] = "gemm"
    C._CHOICE[("bwd_weight", "bf16", 802816, 64, 256)] = "miopen"
    p = tmp_path / "t.json"
    C.dump_table(str(p))
    C._CHOICE.clear()
    assert C.load_table(str(p)) == 2
    assert C._pick(("fwd", "bf16", 802816, 64, 256), {"miopen": None, "gemm": None}) == "gemm"
    assert C._pick(("bwd_weight", "bf16", 802816, 64, 256), {"miopen": None, "gemm": None}) == "miopen"
    import json
    tab = json.load(open(C.TABLE))  # the committed table parses and holds only valid choices
    assert set(tab.values()) <= {"miopen", "gemm", "ours", "splitk8", "splitk16", "splitk32", "splitk64"}
    # split-K weight-gradient decisions load and are picked when the candidate exists
    key = ("bwd_weight", "bf16", 100352, 256, 1024)
    C._CHOICE.clear()
    C.load_table(C.TABLE)
    assert C._pick(key, {"miopen": None, "gemm": None, "splitk32": None}) == tab["bwd_weight,bf16,100352,256,1024"]


def test_wgrad_splitk_matches_mm():
    """The split-K batched-GEMM weight gradient equals dY^T X (CPU, fp32)."""
    import torch
    from pytorch_distributed_training_example_amd.ops import conv as C
    g = torch.randn(512, 24)
    x = torch.randn(512, 40)
    torch.testing.assert_close(C._wgrad_splitk(g, x, 8), g.t() @ x, rtol=1e-4, atol=1e-4)


def test_conv1x1_table_covers_bench_default_resnet50():
    """Every stride-1 1x1 convolution of the headline bench (ResNet-50, 224x224, bench.py's default
    per-GPU batch) has all three directions in the committed table, so a fresh box never times
    MIOpen against GEMM (or runs MIOpen's search for a GEMM-decided shape) inside warm-up."""
    import json

    import torch

    import bench
    from pytorch_distributed_training_example_amd.models import get_model
    from pytorch_distributed_training_example_amd.ops import conv as C
    batch = bench.WORKLOADS["resnet50"][2]
    model = get_model("resnet50").eval()
    shapes = set()

    def hook(mod, inp, out):
        if isinstance(mod, C.Conv1x1) and mod.stride == (1, 1):
            n, ci, h, w = inp[0].shape
            shapes.add((batch * h * w, ci, mod.out_channels))

    hs = [m.register_forward_hook(hook) for m in model.modules()]
    with torch.no_grad():
        model(torch.zeros(1, 3, 224, 224))
    for h in hs:
        h.remove()
    assert len(shapes) >= 10
    tab = json.load(open(C.TABLE))
    missing = [f"{d},bf16,{m},{ci},{co}" for (m, ci, co) in sorted(shapes)
               for d in ("fwd", "bwd_data", "bwd_weight") if f"{d},bf16,{m},{ci},{co}" not in tab]
    assert not missing, missing


def test_conv1x1_table_keyed_by_dtype_and_arch(tmp_path, monkeypatch):
    """A bf16 decision never decides an fp32 conv of the same shape, and the committed (gfx950)
    table is not loaded on any other device (here: no GPU at all)."""
    from pytorch_distributed_training_example_amd.ops import conv as C
    monkeypatch.setattr(C, "_CHOICE", {})
    monkeypatch.setattr(C, "_TABLE_LOADED", [False])
    C._ensure_table()
    assert C._CHOICE == {}  # no gfx950 device here: nothing loaded
    C.load_table()
    assert C._CHOICE and all(k[1] == "bf16" for k in C._CHOICE)
    k = next(iter(C._CHOICE))
    assert ("fwd", "fp32", *k[2:]) not in C._CHOICE
