"""Persistent MIOpen find-db / kernel cache that travels with the repository.

``torch.backends.cudnn.benchmark = True`` makes MIOpen search every convolution's algorithms
(and compile the winning kernels) the first time a shape is seen. On a fresh MI355X box that
search is minutes of warm-up for ResNet-50 (measured: first step 204 s cold, 55 s with this
cache). MIOpen keeps its results in a user find-db (``MIOPEN_USER_DB_PATH``) and compiled code
objects in a kernel cache (``MIOPEN_CUSTOM_CACHE_DIR``); pointing both at an in-tree directory
lets one GPU run populate them and every later run on a fresh box reuse them (the directory is
git-ignored, like the built extension, and shipped with the tree).

Multi-process jobs: only local rank 0 uses (and may update) the in-tree directory; every other
rank works on a private copy under the temp dir, so N ranks never write one sqlite / text db
concurrently.

Processes that restricted MIOpen's solver set for hipGraph capture (engine/graph.py) use a
separate ``capture_safe`` sub-directory.

Must run after ``make_miopen_capture_safe`` (when used) and before the first convolution (MIOpen reads these variables once per process).
Explicit ``MIOPEN_*`` settings in the environment always win.
"""
from __future__ import annotations

import os
import shutil
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_DIR = os.path.join(ROOT, "miopen_cache")


def use_repo_miopen_cache(path: str | None = None) -> str | None:
    """Point MIOpen's user db and kernel cache at ``path`` (default ``<repo>/miopen_cache``,
    or ``$PDT_MIOPEN_CACHE``). Returns the directory used, or None when disabled/unwritable."""
    path = path or os.environ.get("PDT_MIOPEN_CACHE") or DEFAULT_DIR
    if path in ("0", "off", "none"):
        return None
    from .graph import CAPTURE_UNSAFE_MIOPEN_SOLVERS
    if any(os.environ.get(k) == "0" for k in CAPTURE_UNSAFE_MIOPEN_SOLVERS):
        # a solver set restricted for hipGraph capture gets its own find-db, so a db entry
        # found without the restriction is never replayed under capture
        path = os.path.join(path, "capture_safe")
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if local_rank > 0:
        private = os.path.join(tempfile.gettempdir(), f"pdt_miopen_{os.getpid()}_r{local_rank}")
        try:
            if os.path.isdir(path):
                shutil.copytree(path, private, dirs_exist_ok=True)
        except OSError:
            pass
        path = private
    db, kc = os.path.join(path, "db"), os.path.join(path, "kcache")
    try:
        os.makedirs(db, exist_ok=True)
        os.makedirs(kc, exist_ok=True)
    except OSError:
        return None
    if not (os.access(db, os.W_OK) and os.access(kc, os.W_OK)):
        return None
    os.environ.setdefault("MIOPEN_USER_DB_PATH", db)
    os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", kc)
    return path
