"""Measured roofline of a training step from rocprofv3 --pmc runs (tools/gpu_step_roofline.sh).

--reduce <counter_collection.csv> <out.csv>: per dispatch (Dispatch_Id, kernel, duration, counter
    values summed over the dimension rows), keeping the last 2 bench steps (the dispatches after the
    second-to-last launch of the step's first kernel, the stem conv).
--join <pass1.csv> <pass2.csv> [read_scale]: per kernel family (tools/prof_categories.py) and in total: time,
    HBM bytes read / written, achieved TB/s, MFMA bf16 TFLOP/s (SQ_INSTS_VALU_MFMA_MOPS_BF16 counts
    units of 512 FLOPs).

read_scale: rocprofv3's derived FETCH_SIZE assumes 32/64-B read requests; on gfx950 it reports
exactly HALF the bytes of kernels whose reads are known (bn_reduce3 over the 1.64 GB stem output:
0.822 GB; the 256->64 1x1 conv reading a 1.64 GB input: 0.822 GB; the 3x3 wst kernel's 0.41 GB
input: 0.213 GB), i.e. the TCC issues 128-B requests it counts as 64 B. Default 2.0 corrects that;
WRITE_SIZE matches the known output sizes (1.64 GB + the 0.1 GB ReLU mask -> 1.755 GB) unscaled.
"""
import csv
import os
import sys
from collections import OrderedDict, defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def reduce(src, dst):
    per = OrderedDict()
    for r in csv.DictReader(open(src)):
        d = int(r["Dispatch_Id"])
        e = per.setdefault(d, {"name": r["Kernel_Name"], "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    starts = [i for i in ids if "stem_conv_kernel" in per[i]["name"]]
    lo = starts[-2] if len(starts) >= 2 else ids[0]
    keep = [i for i in ids if i >= lo]
    cols = sorted({k for i in keep for k in per[i] if k not in ("name", "ns")})
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["dispatch", "name", "ns"] + cols)
        for i in keep:
            w.writerow([i, per[i]["name"], per[i]["ns"]] + [per[i].get(c, 0.0) for c in cols])
    print(f"{src}: {len(keep)} dispatches kept of {len(ids)}", file=sys.stderr)


def join(p1, p2, read_scale=2.0):
    from prof_categories import family
    a = list(csv.DictReader(open(p1)))
    b = list(csv.DictReader(open(p2)))
    n = min(len(a), len(b))
    steps = max(1, sum(1 for r in a[:n] if "stem_conv_kernel" in r["name"]))
    agg = defaultdict(lambda: [0.0, 0.0, 0.0, 0.0])
    mism = 0
    for ra, rb in zip(a[:n], b[:n]):
        if ra["name"] != rb["name"]:
            mism += 1
        f = family(ra["name"])
        g = agg[f]
        g[0] += float(ra["ns"]) / 2 + float(rb["ns"]) / 2
        g[1] += float(ra.get("FETCH_SIZE", 0)) * 1024 * read_scale
        g[2] += float(rb.get("WRITE_SIZE", 0)) * 1024
        g[3] += float(ra.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0)) * 512
    print(f"steps in window: {steps}; dispatches joined: {n} (name mismatches: {mism}); "
          f"FETCH_SIZE x {read_scale} (see the module docstring)\n")
    print("| family | ms/step | GB read | GB written | TB/s | MFMA bf16 TFLOP/s |\n|---|---:|---:|---:|---:|---:|")
    tot = [0.0, 0.0, 0.0, 0.0]
    for k, g in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        t = g[0] / 1e9
        print(f"| {k} | {g[0] / 1e6 / steps:.2f} | {g[1] / 1e9 / steps:.1f} | {g[2] / 1e9 / steps:.1f} | "
              f"{(g[1] + g[2]) / max(t, 1e-12) / 1e12:.2f} | {g[3] / max(t, 1e-12) / 1e12:.0f} |")
        for j in range(4):
            tot[j] += g[j]
    t = tot[0] / 1e9
    print(f"| **step** | {tot[0] / 1e6 / steps:.2f} | {tot[1] / 1e9 / steps:.1f} | {tot[2] / 1e9 / steps:.1f} | "
          f"{(tot[1] + tot[2]) / max(t, 1e-12) / 1e12:.2f} | {tot[3] / max(t, 1e-12) / 1e12:.0f} |")
    print("\n(durations are from the counter-collection runs, which serialise kernels; FETCH_SIZE / "
          "WRITE_SIZE are KB at the L2-HBM interface, so L2 / MALL hits are not counted as HBM traffic)")


if __name__ == "__main__":
    if sys.argv[1] == "--reduce":
        reduce(sys.argv[2], sys.argv[3])
    else:
        join(sys.argv[2], sys.argv[3], float(sys.argv[4]) if len(sys.argv) > 4 else 2.0)
