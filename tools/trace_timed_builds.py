#!/usr/bin/env python3
"""Kernel-trace durations of the bench's timed steps: in a rocprofv3
--kernel-trace CSV of `bench.py --steps N`, the timed region is the first
host-synchronised block of exactly N build + N iterate launches (the settle
blocks have 16, the iterate-timing pass comes after a download).  Prints the
average build and iterate durations there, for comparison with the bench
line's HIP-event averages.
usage: python tools/trace_timed_builds.py TRACE_CSV N"""
import csv
import json
import sys

path, n = sys.argv[1], int(sys.argv[2])
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
            for r in csv.DictReader(open(path)))
blocks, cur, prev = [], [], None
for s, e, name in ks:
    if prev is not None and s - prev > 30000:  # > 30 us idle: a host synchronisation
        blocks.append(cur)
        cur = []
    cur.append((s, e, name))
    prev = e
blocks.append(cur)
for b in blocks:
    bu = [(e - s) / 1e6 for s, e, name in b if "build" in name]
    it = [(e - s) / 1e6 for s, e, name in b if "solve" in name]
    if len(bu) == n and len(it) == n:
        print(json.dumps({"timed_launches": n, "build_trace_avg_ms": sum(bu) / n,
                          "iterate_trace_avg_ms": sum(it) / n,
                          "step_span_ms": (b[-1][1] - b[0][0]) / 1e6 / n}))
        break
else:
    sys.exit("no block of %d build + %d iterate launches" % (n, n))
