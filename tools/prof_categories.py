"""Group a prof_window.py *_kernels.csv by kernel family (ms per step)."""
import csv
import re
import sys


def family(n):
    if "conv1x1_bwd_fused" in n or "fb_reduce" in n:
        return "fused conv3 + BN3 backward (dgrad + wgrad + BN apply/reduction)"
    m = re.search(r"conv1x1_kernel<.*?G1<[^>]*>,(.*?)>\s*\(", n)  # <Cf, ACC, STATS, NT, BSTATS, ATR, APPLY[, STR]>
    if m and [f.strip() for f in m.group(1).split(",")][5:6] == ["true"]:
        return "1x1 GEMM + BN(+res)+ReLU apply epilogue (recomputed conv3)"
    m = re.search(r"conv1x1p_kernel<.*?G1<[^>]*>,(.*?)>\s*\(", n)  # persistent: <Cf, ACC, STATS, BSTATS, ATR, APPLY, STR>
    if m and [f.strip() for f in m.group(1).split(",")][4:5] == ["true"]:
        return "1x1 GEMM + BN(+res)+ReLU apply epilogue (recomputed conv3)"
    if "conv1x1_wgrad" in n:
        return "our 1x1 weight gradient (MFMA)"
    if "weight_prep" in n:
        return "batched weight transforms"
    if "bn_" in n or "maxpool" in n:
        return "our BN (+ReLU/residual/pool)"
    if "conv3x3" in n:
        return "our 3x3 conv (MFMA)"
    if "conv1x1_kernel" in n or "conv1x1p_kernel" in n:
        return "our 1x1 conv GEMM (MFMA, fused BN-stats epilogues)"
    if "stem_" in n:
        return "our 7x7 stem conv (MFMA)"
    if "Cijk" in n:
        return "hipBLASLt GEMM (1x1 convs, fc)"
    if any(s in n for s in ("igemm", "ck::", "_ZN2ck", "naive_conv", "SubTensor", "fillBuffer", "ranspose")):
        return "MIOpen conv (+fills)"
    if any(s in n for s in ("ce_", "mt_kernel", "sgd", "strip", "colsum")):
        return "our CE / optimizer"
    return "other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    cat = {}
    other = []
    for r in rows:
        ms = float(r["TotalDurationNs"]) / 1e6 / steps
        f = family(r["Name"])
        cat[f] = cat.get(f, 0.0) + ms
        if f == "other":
            other.append((ms, r["Name"][:80]))
    print("| family | ms/step |\n|---|---:|")
    for k, v in sorted(cat.items(), key=lambda x: -x[1]):
        print(f"| {k} | {v:.2f} |")
    print(f"| total busy | {sum(cat.values()):.2f} |")
    for ms, n in sorted(other, reverse=True)[:8]:
        print(f"  other: {ms:.3f} {n}", file=sys.stderr)


if __name__ == "__main__":
    main()
