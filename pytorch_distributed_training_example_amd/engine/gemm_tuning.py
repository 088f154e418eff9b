"""Measured GEMM solution selection (PyTorch TunableOp over hipBLASLt / rocBLAS), shipped in-tree.

hipBLASLt picks a kernel for each GEMM shape by heuristic. PyTorch's TunableOp instead times
every hipBLASLt and rocBLAS solution for the shape once and records the fastest in a CSV
(operator, shape, solution, time). Measured on one MI355X (`tools/gpu_tunableop.sh`):
ViT-B/16 4,251 -> 4,910 img/s (+15%) from the tuned block GEMMs; GPT-2-medium +1%.

The tuned table for this framework's workloads is committed at ``tuning/tunableop_gfx950.csv``
(its Validator lines pin the PyTorch / HIP / hipBLASLt / rocBLAS versions; TunableOp rejects it
on any other stack). ``use_repo_gemm_tuning()`` enables TunableOp in READ-ONLY mode against it:
a shape that is in the table runs its measured solution, any other shape runs the default
heuristic pick — never a surprise search inside a timed run. ``PDT_TUNE_GEMMS=1`` turns the
search on for unseen shapes (results are written to ``$PDT_TUNE_GEMMS_OUT`` or the temp copy)
to extend the table.

TunableOp reads ``<name><device ordinal>.csv``; each process gets a private copy named for its
own device, so every rank of a multi-GPU job sees the table. Must run before the first GEMM.
"""
from __future__ import annotations

import os
import shutil
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TABLE = os.path.join(ROOT, "tuning", "tunableop_gfx950.csv")


def wants_gemm_tuning(model: str, grad_accum: int, hipgraph: bool) -> bool:
    """One predicate for every entry point (bench.py, cli.py): the measured table pays off for big
    GEMMs only. TunableOp's per-call host lookup costs more than it saves on launch-bound models
    (LeNet, MLP: 177k -> 131k img/s) and on eager micro-batched steps (ViT 4 x 32: 3,190 -> 2,999);
    a hipGraph replay pays the lookup once, at capture."""
    return model not in ("lenet", "mlp") and (grad_accum == 1 or bool(hipgraph))


def use_repo_gemm_tuning(device_index: int | None = None, table: str | None = None) -> str | None:
    """Enable TunableOp with the committed table. Returns the filename pattern used, or None
    when disabled (``PDT_GEMM_TUNING=0``) or when the table is missing. Explicit
    ``PYTORCH_TUNABLEOP_*`` settings in the environment win."""
    if os.environ.get("PDT_GEMM_TUNING", "1") == "0" or "PYTORCH_TUNABLEOP_ENABLED" in os.environ:
        return None
    table = table or TABLE
    tune = os.environ.get("PDT_TUNE_GEMMS", "0") == "1"
    if not os.path.exists(table) and not tune:
        return None
    if device_index is None:
        device_index = int(os.environ.get("LOCAL_RANK", "0"))
    out_dir = os.environ.get("PDT_TUNE_GEMMS_OUT") if tune else None
    d = out_dir or os.path.join(tempfile.gettempdir(), f"pdt_tunableop_{os.getpid()}")
    os.makedirs(d, exist_ok=True)
    if os.path.exists(table):
        shutil.copyfile(table, os.path.join(d, f"tunableop{device_index}.csv"))
    pattern = os.path.join(d, "tunableop%d.csv")
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1" if tune else "0"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = pattern
    if tune:
        os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "20")
        os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS", "5")
    return pattern


def merge_tables(paths: list[str], out: str) -> int:
    """Union of TunableOp CSVs (validators from the first; later files win on duplicate keys).
    Returns the number of tuned entries written."""
    validators: list[str] = []
    entries: dict[tuple[str, str], str] = {}
    for i, p in enumerate(paths):
        with open(p) as f:
            for line in f:
                line = line.rstrip("\n")
                if not line:
                    continue
                parts = line.split(",")
                if parts[0] == "Validator":
                    if i == 0:
                        validators.append(line)
                    continue
                entries[(parts[0], parts[1])] = line
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        for v in validators:
            f.write(v + "\n")
        for k in sorted(entries):
            f.write(entries[k] + "\n")
    return len(entries)
