"""Per-wave PMC of the iterate (solve) kernel from tools/gpu_pmc_iterate.sh's
passes: the last `steps` dispatches of each pass (the timed step loop of
tools/pmc_iterate.py), counters divided by SQ_WAVES.
usage: python tools/summarize_pmc_iterate.py gpurun_out [steps]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d, steps):
    rows = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if "cmpc_solve" not in r["Kernel_Name"]:
            continue
        did = int(r["Dispatch_Id"])
        rows[did][r["Counter_Name"]] = rows[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[did] = (r["Kernel_Name"], r["VGPR_Count"], r["Scratch_Size"])
    ids = sorted(rows)[-steps:]
    agg = defaultdict(float)
    for i in ids:
        for k, v in rows[i].items():
            agg[k] += v / len(ids)
    return agg, meta[ids[-1]] if ids else None, len(ids)


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    tags = sorted({os.path.basename(p)[len("pmcit_"):-2] for p in glob.glob(os.path.join(root, "pmcit_*_a"))})
    for t in tags:
        a, meta, n = load(os.path.join(root, f"pmcit_{t}_a"), steps)
        b, _, _ = load(os.path.join(root, f"pmcit_{t}_b"), steps)
        c = {**a, **b}
        waves = a.get("SQ_WAVES", 0.0) or 1.0
        print(f"{t}: {meta[0] if meta else '?'} vgpr={meta[1] if meta else '?'} "
              f"scratch={meta[2] if meta else '?'} dispatches={n} waves={waves:.0f}")
        for k in sorted(c):
            if k == "SQ_WAVES":
                continue
            print(f"  {k:24s} per wave {c[k] / waves:12.1f}   per dispatch {c[k]:14.0f}")


if __name__ == "__main__":
    main()
