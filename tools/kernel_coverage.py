"""Kernel-name coverage gate: which kernels of the bench's steady-state step did the GPU tests launch?

The GPU test tier is run under ``rocprofv3 --kernel-trace`` (tools/gpu_coverage.sh); this compares the
kernel names in that trace against a step window's per-kernel table (tools/prof_window.py output, e.g.
profiles/r5/steady_resnet50_b1024_kernels.csv). Template instantiations count separately: a test that
runs ``conv1x1_kernel<G1<128,4,2>,...>`` does not cover the 16-wave ``G1<256,4,4>`` variant of the same
epilogue (round-4 VERDICT: the largest kernel family of the step was never hit by a test).

    python tools/kernel_coverage.py <tests_kernel_trace.csv> <step_kernels.csv> [--out report.md] [--strict]

Library kernels (hipBLASLt ``Cijk_*``, aten ``at::native``) are listed but never required.
Exit status 1 with --strict when one of OUR kernels of the step is not covered.
"""
from __future__ import annotations

import argparse
import csv
import re
import sys


def norm(name: str) -> str:
    """Kernel identity without the argument list (template arguments kept)."""
    name = re.sub(r"\(anonymous namespace\)::", "", name.strip().strip('"'))
    depth = 0
    for i, ch in enumerate(name):  # cut at the '(' that opens the parameter list (outside template <>)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            name = name[:i]
            break
    return name.replace("void ", "", 1).strip()


def library(n: str) -> bool:
    return n.startswith(("Cijk_", "Custom_Cijk")) or "at::native" in n or n.startswith("__amd_rocclr")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("step")
    ap.add_argument("--out", default=None)
    ap.add_argument("--strict", action="store_true")
    a = ap.parse_args(argv)
    seen = set()
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            seen.add(norm(r.get("Kernel_Name") or r.get("Name") or ""))
    rows = []
    with open(a.step) as f:
        for r in csv.DictReader(f):
            n = norm(r["Name"])
            rows.append((n, float(r["TotalDurationNs"]), int(r["Calls"])))
    ms_total = sum(t for _, t, _ in rows) or 1.0
    lines = ["| step kernel | share of step | covered by a GPU test |", "|---|---:|---|"]
    missing = []
    for n, t, _ in sorted(rows, key=lambda x: -x[1]):
        cov = n in seen
        tag = "yes" if cov else ("library (not required)" if library(n) else "**NO**")
        if not cov and not library(n):
            missing.append(n)
        lines.append(f"| `{n[:150]}` | {100 * t / ms_total:.2f} % | {tag} |")
    ours = [n for n, _, _ in rows if not library(n)]
    summary = (f"{len(ours) - len(missing)} of {len(ours)} of our step kernels launched by the GPU tests "
               f"({100 * sum(t for n, t, _ in rows if n in seen and not library(n)) / ms_total:.1f} % of the step's "
               f"kernel time); library kernels are not required.")
    text = summary + "\n\n" + "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(summary)
    for n in missing:
        print("  not covered:", n)
    return 1 if (a.strict and missing) else 0


if __name__ == "__main__":
    sys.exit(main())
