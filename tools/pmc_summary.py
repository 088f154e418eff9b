"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel name (filtered), per counter,
the value of the last dispatch (steady state) and the kernel duration from the trace."""
import csv
import glob
import sys
from collections import defaultdict

pat = sys.argv[2] if len(sys.argv) > 2 else "conv3x3s1"
vals = defaultdict(dict)
for f in sorted(glob.glob(sys.argv[1] + "/*/*_counter_collection.csv")):
    rows = [r for r in csv.DictReader(open(f)) if pat in r["Kernel_Name"]]
    if not rows:
        continue
    last = max(int(r["Dispatch_Id"]) for r in rows)
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            vals[r["Kernel_Name"][:60]][r["Counter_Name"]] = float(r["Counter_Value"])
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {v:16.0f}")
