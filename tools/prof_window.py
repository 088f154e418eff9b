"""Aggregate rocprofv3 kernel-trace rows that fall inside a roctx range (default "timed").

usage: python tools/prof_window.py <rocprof_out_dir> <out_prefix> [range_name] [steps] [occurrence]
(occurrence: which of several ranges of that name, 0-based; default the last)
Writes <out_prefix>_kernels.csv (per-kernel totals inside the window) and <out_prefix>.md.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d, out = sys.argv[1], sys.argv[2]
    name = sys.argv[3] if len(sys.argv) > 3 else "timed"
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True)
    occ = int(sys.argv[5]) if len(sys.argv) > 5 else -1
    lo, hi = 0, float("inf")
    if mt:
        ranges = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(mt[0]))
                        if name in (r.get("Function", "") + r.get("Message", "") + r.get("Name", "")))
        if ranges:
            lo, hi = ranges[occ]
    agg = defaultdict(lambda: [0, 0])
    t_first, t_last = None, None
    for r in csv.DictReader(open(kt[0])):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < lo or e > hi:
            continue
        k = r["Kernel_Name"]
        agg[k][0] += 1
        agg[k][1] += e - s
        t_first = s if t_first is None else min(t_first, s)
        t_last = e if t_last is None else max(t_last, e)
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for _, v in rows) or 1
    with open(out + "_kernels.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for k, (c, t) in rows:
            w.writerow([k, c, t, t / c, 100.0 * t / tot])
    span = (t_last - t_first) if t_first is not None else 0
    with open(out + ".md", "w") as f:
        f.write(f"Window '{name}': {len(rows)} distinct kernels, busy {tot/1e6:.2f} ms, span {span/1e6:.2f} ms "
                f"over {steps} steps -> {tot/1e6/steps:.2f} ms/step busy, {span/1e6/steps:.2f} ms/step span\n\n")
        f.write("| kernel | calls/step | ms/step | avg us | % |\n|---|---:|---:|---:|---:|\n")
        for k, (c, t) in rows[:40]:
            f.write(f"| `{k[:100]}` | {c/steps:.1f} | {t/1e6/steps:.3f} | {t/c/1e3:.1f} | {100*t/tot:.1f} |\n")
    print(open(out + ".md").read()[:4000])


if __name__ == "__main__":
    main()
