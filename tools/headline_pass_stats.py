"""Kernel statistics of the headline's own launches, cut from a rocprofv3
kernel trace of `bench.py --headline-only --markers`.

The bench brackets two passes with torch.cuda._sleep marker launches:
  pass 1: the timed steps (build with events, the iterate without),
  pass 2: the same step loop again with events on the iterate only.
The build's rocprof averages over both passes are compared with the bench
line's roofline.avg_launch_ms, the iterate's over pass 2 with
kernels_ms_per_step.iterate: the profiled run's own events (`run_event_us`,
`run_ratio`: the same launches under the same profiler) and, when given, an
unprofiled reference line's (`bench_event_us`, `ratio`; without one these
repeat the run's own).  A last row takes the timed pass's event-stamped
build launches alone (every build_event_stride-th), against the same run's
events.
usage: python tools/headline_pass_stats.py <kernel_trace.csv> <profiled bench json>
       [<reference bench json>] [out.csv]"""
import csv
import json
import sys
from collections import defaultdict


def short(name):
    """The kernel's name without its signature: rocprofv3 -T already
    truncates; full names may carry a "(anonymous namespace)::" prefix."""
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def last_line(path):
    return [json.loads(x) for x in open(path).read().splitlines() if x.strip().startswith("{")][-1]


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    run = last_line(bench)
    ref = last_line(sys.argv[3]) if len(sys.argv) > 3 else run
    out = sys.argv[4] if len(sys.argv) > 4 else None
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin" in r["Kernel_Name"] or "sleep" in r["Kernel_Name"]]
    if len(marks) != 4:
        sys.exit(f"expected 4 marker launches, found {len(marks)}")
    def events(line):
        return {"build": line["roofline"]["avg_launch_ms"] * 1e3,
                "iterate": line["kernels_ms_per_step"]["iterate"] * 1e3}

    ev, ev_run = events(ref), events(run)
    table = []
    for n, (pname, role_of_pass) in enumerate((("timed_steps", "build"), ("iterate_event_pass", "iterate"))):
        a, b = marks[2 * n], marks[2 * n + 1]
        dur = defaultdict(list)
        for r in rows[a + 1:b]:
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for name, d in dur.items():
            role = "build" if "build" in name else "iterate" if "solve" in name else None
            avg = sum(d) / len(d)
            # the build runs in both passes (the iterate pass replays the same
            # steps): both are compared with the build's events
            cmp = role == role_of_pass or role == "build"
            e = ev.get(role) if cmp else None
            er = ev_run.get(role) if cmp else None
            table.append({"pass": pname, "kernel": name, "calls": len(d), "rocprof_avg_us": round(avg, 3),
                          "bench_event_us": round(e, 3) if e else None,
                          "ratio": round(avg / e, 4) if e else None,
                          "run_event_us": round(er, 3) if er else None,
                          "run_ratio": round(avg / er, 4) if er else None})
    # the timed pass's build launches the bench stamped with events (every
    # build_event_stride-th from the first): rocprof and events on the same
    # launches of the same run
    stride = int(run["kernels_ms_per_step"].get("build_event_stride", 1) or 1)
    a, b = marks[0], marks[1]
    builds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
              for r in rows[a + 1:b] if "build" in short(r["Kernel_Name"])]
    stamped = builds[::stride]
    if stamped:
        avg = sum(stamped) / len(stamped)
        table.append({"pass": "timed_steps_stamped", "kernel": "cmpc_build_rows_kernel", "calls": len(stamped),
                      "rocprof_avg_us": round(avg, 3), "bench_event_us": None, "ratio": None,
                      "run_event_us": round(ev_run["build"], 3), "run_ratio": round(avg / ev_run["build"], 4)})
    for t in table:
        print(t)
    if out:
        with open(out, "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(table[0]))
            w.writeheader()
            w.writerows(table)


if __name__ == "__main__":
    main()
