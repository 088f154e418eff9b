"""Per-kernel difference of two prof_window.py outputs (<prefix>_kernels.csv, same step count).

usage: python tools/prof_diff.py A_kernels.csv B_kernels.csv [steps] [top]
"""
import csv
import sys


def load(p):
    return {r["Name"]: (int(r["Calls"]), int(r["TotalDurationNs"])) for r in csv.DictReader(open(p))}


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    keys = set(a) | set(b)
    rows = []
    for k in keys:
        ca, ta = a.get(k, (0, 0))
        cb, tb = b.get(k, (0, 0))
        rows.append((tb - ta, k, ca, ta, cb, tb))
    rows.sort(key=lambda r: -abs(r[0]))
    ta_tot = sum(v[1] for v in a.values()) / 1e6 / steps
    tb_tot = sum(v[1] for v in b.values()) / 1e6 / steps
    print(f"total busy ms/step: A {ta_tot:.2f}  B {tb_tot:.2f}  diff {tb_tot - ta_tot:+.2f}")
    print("| kernel | A calls | A ms | B calls | B ms | B-A ms |\n|---|---:|---:|---:|---:|---:|")
    for d, k, ca, ta, cb, tb in rows[:top]:
        print(f"| `{k[:90]}` | {ca / steps:.0f} | {ta / 1e6 / steps:.3f} | {cb / steps:.0f} | {tb / 1e6 / steps:.3f} | "
              f"{d / 1e6 / steps:+.3f} |")


if __name__ == "__main__":
    main()
