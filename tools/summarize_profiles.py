#!/usr/bin/env python3
"""Copy the rocprofv3 summaries of one GPU round into profiles/ (tracked).

usage: python tools/summarize_profiles.py TAG ROUND [BATCH]

  gpurun_out/prof_TAG/run_kernel_stats.csv      -> profiles/ROUND_kernel_stats.csv
  gpurun_out/cfgprof_TAG/run_kernel_stats.csv   -> profiles/ROUND_configs_kernel_stats.csv
                                                 (+ that run's configs line)
  gpurun_out/pmcTAG_{sq1,sq2,fetch,write}/...   -> profiles/ROUND_pmc.json
                                                 + profiles/pmc_build_coop_p50.json

Counters are the median over a kernel's dispatches.  HBM bytes per launch
follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a 16-byte-per-lane coalesced streaming read (the build kernel's record
loads are exactly that), so it is doubled; WRITE_SIZE is taken as is.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def counters(tag, name):
    path = os.path.join(OUT, f"pmc{tag}_{name}", "run_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    acc = defaultdict(lambda: defaultdict(list))
    for row in csv.DictReader(open(path)):
        acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    # the median over a kernel's dispatches: a launch right after one that
    # left many dirty L2 lines (e.g. a traced solve) is charged their
    # write-back, which the mean would spread over the others
    def med(v):
        v = sorted(v)
        n = len(v)
        return v[n // 2] if n % 2 else 0.5 * (v[n // 2 - 1] + v[n // 2])
    return {k: {c: med(v) for c, v in d.items()} | {"_dispatches": len(next(iter(d.values())))}
            for k, d in acc.items()}


def main():
    tag, rnd = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    os.makedirs(PROF, exist_ok=True)
    ks = os.path.join(OUT, f"prof_{tag}", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(PROF, f"{rnd}_kernel_stats.csv"))
        print("copied", ks)
    cs = os.path.join(OUT, f"cfgprof_{tag}", "run_kernel_stats.csv")
    if os.path.exists(cs):  # bench.py --configs-only under rocprofv3 --stats
        shutil.copy(cs, os.path.join(PROF, f"{rnd}_configs_kernel_stats.csv"))
        shutil.copy(os.path.join(OUT, f"cfgprof_{tag}.json"), os.path.join(PROF, f"{rnd}_configs_bench.json"))
        print("copied", cs)
    merged = defaultdict(dict)
    for name in ("sq1", "sq2", "fetch", "write"):
        for k, d in counters(tag, name).items():
            merged[k].update(d)
    if not merged:
        return
    summary = {"note": __doc__.strip().splitlines()[0], "batch_scenarios": batch, "kernels": {}}
    for k, d in merged.items():
        e = dict(d)
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            e["hbm_read_bytes"] = 2.0 * d["FETCH_SIZE"] * 1024.0
            e["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024.0
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        if "SQ_WAVES" in d and d["SQ_WAVES"]:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
                if c in d:
                    e[c + "_per_wave"] = d[c] / d["SQ_WAVES"]
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in d:
                    e[c + "_frac"] = d[c] / d["SQ_WAVE_CYCLES"]
        summary["kernels"][k] = e
    json.dump(summary, open(os.path.join(PROF, f"{rnd}_pmc.json"), "w"), indent=1)
    bk = "cmpc_build_rows_kernel" if "cmpc_build_rows_kernel" in summary["kernels"] else "cmpc_build_kernel"
    b = summary["kernels"].get(bk, {})
    if "hbm_bytes_per_launch" in b:
        # the hash of the bench kernel's machine code the PMC pass ran, as that
        # run's bench line printed it (the tree here may have moved on since)
        h = None
        try:
            h = json.load(open(os.path.join(OUT, f"pmc{tag}_fetch.json")))["roofline"]["traffic_provenance"][
                "current_code_hash"]
        except (OSError, ValueError, KeyError, TypeError):
            sys.path.insert(0, ROOT)
            sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
            from bench import bench_kernel_code_hash
            h = bench_kernel_code_hash()
        json.dump({"batch": batch, "round": rnd, "kernel": bk, "build_kernel_code_hash": h,
                   "hbm_bytes_per_launch": b["hbm_bytes_per_launch"],
                   "hbm_read_bytes": b["hbm_read_bytes"], "hbm_write_bytes": b["hbm_write_bytes"],
                   "source": f"profiles/{rnd}_pmc.json"},
                  open(os.path.join(PROF, "pmc_build_coop_p50.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1)[:3000])


if __name__ == "__main__":
    main()
