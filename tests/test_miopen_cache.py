"""MIOpen find-db / kernel-cache placement (engine/miopen_cache.py). CPU-only: checks the
environment each process gets, not MIOpen itself."""
import os

from pytorch_distributed_training_example_amd.engine import miopen_cache
from pytorch_distributed_training_example_amd.engine.graph import CAPTURE_UNSAFE_MIOPEN_SOLVERS


def _clean(monkeypatch):
    for k in ("MIOPEN_USER_DB_PATH", "MIOPEN_CUSTOM_CACHE_DIR", "PDT_MIOPEN_CACHE", "LOCAL_RANK",
              *CAPTURE_UNSAFE_MIOPEN_SOLVERS):
        monkeypatch.delenv(k, raising=False)


def test_rank0_uses_tree_dir(tmp_path, monkeypatch):
    _clean(monkeypatch)
    d = miopen_cache.use_repo_miopen_cache(str(tmp_path / "mc"))
    assert d == str(tmp_path / "mc")
    assert os.environ["MIOPEN_USER_DB_PATH"] == str(tmp_path / "mc" / "db")
    assert os.environ["MIOPEN_CUSTOM_CACHE_DIR"] == str(tmp_path / "mc" / "kcache")


def test_capture_safe_solver_set_gets_its_own_db(tmp_path, monkeypatch):
    _clean(monkeypatch)
    monkeypatch.setenv(CAPTURE_UNSAFE_MIOPEN_SOLVERS[0], "0")
    d = miopen_cache.use_repo_miopen_cache(str(tmp_path / "mc"))
    assert d == str(tmp_path / "mc" / "capture_safe")


def test_other_local_ranks_get_private_copies(tmp_path, monkeypatch):
    _clean(monkeypatch)
    src = tmp_path / "mc"
    (src / "db").mkdir(parents=True)
    (src / "db" / "x.ufdb.txt").write_text("entry")
    monkeypatch.setenv("LOCAL_RANK", "3")
    monkeypatch.setattr(miopen_cache.tempfile, "gettempdir", lambda: str(tmp_path / "tmp"))
    d = miopen_cache.use_repo_miopen_cache(str(src))
    assert d != str(src) and d.startswith(str(tmp_path / "tmp"))
    assert open(os.path.join(d, "db", "x.ufdb.txt")).read() == "entry"  # starts from rank 0's db
    assert os.environ["MIOPEN_USER_DB_PATH"] == os.path.join(d, "db")


def test_explicit_env_and_off_switch(tmp_path, monkeypatch):
    _clean(monkeypatch)
    monkeypatch.setenv("MIOPEN_USER_DB_PATH", "/custom/db")
    miopen_cache.use_repo_miopen_cache(str(tmp_path / "mc"))
    assert os.environ["MIOPEN_USER_DB_PATH"] == "/custom/db"
    assert miopen_cache.use_repo_miopen_cache("off") is None
