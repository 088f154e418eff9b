"""Per-call view of one step inside a rocprofv3 kernel trace: every kernel launch of the LAST timed step
(the window split into `steps` equal parts by launch count) with its duration, grid and workgroup sizes,
in launch order — to find under-filled grids (workgroups < 256 CUs x occupancy) at small batches.

usage: python tools/prof_calls.py <rocprof_out_dir> [range_name] [steps] [min_us]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "timed"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    min_us = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    mt = glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True)
    lo, hi = 0, float("inf")
    if mt:
        rs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(mt[0]))
                    if name in (r.get("Function", "") + r.get("Message", "") + r.get("Name", "")))
        if rs:
            lo, hi = rs[-1]
    rows = [r for r in csv.DictReader(open(kt)) if int(r["Start_Timestamp"]) >= lo and int(r["End_Timestamp"]) <= hi]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per = len(rows) // max(steps, 1)
    last = rows[-per:] if per else rows
    tot = 0.0
    print("| # | us | workgroups | wg size | kernel |\n|---:|---:|---:|---:|---|")
    for i, r in enumerate(last):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += us
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        if us >= min_us:
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            k = k[:k.find("(")] if "(" in k else k
            print(f"| {i} | {us:.1f} | {grid // max(wg, 1)} | {wg} | `{k[:100]}` |")
    print(f"\n{len(last)} launches, {tot / 1e3:.2f} ms busy in the step")


if __name__ == "__main__":
    main()
