"""Per-rank library environment of a self-spawned job (cli.configure_process): every rank sees the
measured GEMM table under its own device index, and only local rank 0 uses the in-tree MIOpen
find-db (the others work on private copies). CPU/gloo, world_size 2."""
import argparse
import json
import os

from pytorch_distributed_training_example_amd.engine import miopen_cache
from pytorch_distributed_training_example_amd.parallel import launcher

_KEYS = ("PYTORCH_TUNABLEOP_FILENAME", "MIOPEN_USER_DB_PATH", "MIOPEN_CUSTOM_CACHE_DIR")


def _probe(rank, world, out_dir):
    from pytorch_distributed_training_example_amd import cli
    cli.configure_process(argparse.Namespace(model="resnet50", grad_accum=1))
    env = {k: os.environ.get(k) for k in _KEYS}
    env["local_rank"] = os.environ["LOCAL_RANK"]
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(env, f)


def test_spawned_ranks_get_own_gemm_table_and_private_miopen_db(tmp_path, monkeypatch, switch):
    for k in list(os.environ):
        if k.startswith(("PYTORCH_TUNABLEOP_", "MIOPEN_", "PDT_")):
            monkeypatch.delenv(k, raising=False)
    cache = tmp_path / "miopen"
    switch("PDT_MIOPEN_CACHE", str(cache))
    launcher.spawn(_probe, 2, args=(str(tmp_path),), backend="gloo", use_gpu=False)
    envs = [json.load(open(tmp_path / f"r{r}.json")) for r in range(2)]
    for r, env in enumerate(envs):
        assert env["local_rank"] == str(r)
        table = env["PYTORCH_TUNABLEOP_FILENAME"].replace("%d", str(r))
        assert os.path.exists(table), (r, table)  # rank r's device reads tunableop<r>.csv
    assert envs[0]["MIOPEN_USER_DB_PATH"] == str(cache / "db")
    assert not envs[1]["MIOPEN_USER_DB_PATH"].startswith(str(cache))  # private copy, never the tree
    assert envs[1]["MIOPEN_CUSTOM_CACHE_DIR"] != envs[0]["MIOPEN_CUSTOM_CACHE_DIR"]
    assert os.environ.get("MIOPEN_USER_DB_PATH") is None  # the parent set nothing for its children


def test_parent_main_does_not_configure_libraries(monkeypatch):
    """cli.main's spawn path leaves the library environment to the ranks."""
    from pytorch_distributed_training_example_amd import cli
    called = []
    monkeypatch.setattr(cli.launcher, "spawn", lambda *a, **k: called.append("spawn"))
    monkeypatch.setattr(miopen_cache, "use_repo_miopen_cache", lambda *a, **k: called.append("miopen"))
    for k in ("RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    cli.main(["--model", "resnet50", "--no-cuda", "--world-size", "2"])
    assert called == ["spawn"]
