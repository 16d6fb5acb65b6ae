#!/usr/bin/env python3
"""Print the per-kernel PMC averages of gpurun_out/pmc<TAG>_<pass>/ directories.
usage: python tools/pmc_print.py TAG"""
import csv, glob, os, sys
from collections import defaultdict
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc{tag}_*", "run_counter_collection.csv"))):
    for row in csv.DictReader(open(path)):
        acc[row["Kernel_Name"][:60]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.4g}   (n={len(v)})")
