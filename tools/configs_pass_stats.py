"""Kernel statistics of the configs section's event-timed passes, cut from a
rocprofv3 kernel trace of `bench.py --configs-only` (which brackets each
config's event-timed pass with torch.cuda._sleep launches), against the event
times (kernels_ms) of an unprofiled bench line (the profiled run's own events
are perturbed by the tracer; without a reference line they are used).
usage: python tools/configs_pass_stats.py <run_kernel_trace.csv> <profiled bench json>
       [<reference bench json>] [out.csv]"""
import csv
import json
import sys
from collections import defaultdict


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    refb = sys.argv[3] if len(sys.argv) > 3 else bench
    out = sys.argv[4] if len(sys.argv) > 4 else None
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin" in r["Kernel_Name"] or "sleep" in r["Kernel_Name"]]
    lines = [json.loads(x) for x in open(bench).read().splitlines() if x.strip().startswith("{")]
    cfgs = lines[-1]["configs"]
    rl = [json.loads(x) for x in open(refb).read().splitlines() if x.strip().startswith("{")]
    ref = rl[-1]["configs"]
    keys = [k for k in ("2", "3", "5") if k in cfgs and "error" not in cfgs[k]]
    if len(marks) != 2 * len(keys):
        sys.exit(f"expected {2 * len(keys)} marker launches, found {len(marks)}")
    table = []
    for n, key in enumerate(keys):
        a, b = marks[2 * n], marks[2 * n + 1]
        dur = defaultdict(list)
        for r in rows[a + 1:b]:
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        km = ref[key]["kernels_ms"]
        for name, d in dur.items():
            role = ("fused_step" if "build" in name and "fused_step" in km else
                    "build" if "build" in name else "iterate" if "solve" in name else None)
            ev = km.get(role) * 1e3 if role in km else None
            avg = sum(d) / len(d)
            table.append({"config": key, "kernel": name, "calls": len(d), "rocprof_avg_us": round(avg, 3),
                          "bench_event_us": round(ev, 3) if ev else None,
                          "ratio": round(avg / ev, 4) if ev else None,
                          "bench_ms_per_step_us": round(ref[key]["ms_per_step"] * 1e3, 3)})
    for t in table:
        print(t)
    if out:
        with open(out, "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(table[0]))
            w.writeheader()
            w.writerows(table)


if __name__ == "__main__":
    main()
