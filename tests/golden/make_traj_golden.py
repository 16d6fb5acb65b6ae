#!/usr/bin/env python3
"""Extract the first records of the reference's closed-loop trajectories into
tests/golden/traj_<plant>_<cfg>.json (SURVEY.md §4 record layout: t, plant
state x, controller output u (before the input delay line), plant output y,
wall-ns, blank line).

Run once in the build container (needs /root/reference; the GPU box never
reads the reference).  Data only.  These pin the plant simulation
(SimulationSystem::Integrate, simulation_system.h:108-116, TimeDelay,
time_delay.h:41-58): driven by the recorded u(t), a faithful simulation
reproduces the recorded x(t) and y(t) to the printed 6 digits, whatever the
controller's (missing) observer gain was.
"""
import json
import os

REF = "/root/reference/results"
HERE = os.path.dirname(os.path.abspath(__file__))
N_RECORDS = 160  # 8 s at Ts = 0.05: covers the 40-sample delay-line onset at t = 2 s
CASES = [("parallel", "centralized"), ("parallel", "coop9"), ("parallel", "ncoop9"),
         ("serial", "centralized"), ("serial", "coop9"), ("serial", "ncoop9")]


def records(path, n):
    out = []
    with open(path) as f:
        lines = f.read().split("\n")
    i = 0
    while len(out) < n and i + 5 <= len(lines):
        t = float(lines[i])
        x = [float(v) for v in lines[i + 1].split()]
        u = [float(v) for v in lines[i + 2].split()]
        y = [float(v) for v in lines[i + 3].split()]
        out.append({"t": t, "x": x, "u": u, "y": y})
        i += 6
    return out


def main():
    for plant, cfg in CASES:
        path = os.path.join(REF, plant, "run1", cfg + ".dat")
        recs = records(path, N_RECORDS)
        with open(path) as f:  # the first two records verbatim (the writer's format)
            raw = f.read().split("\n")[:12]
        name = os.path.join(HERE, f"traj_{plant[:3]}_{cfg}.json")
        with open(name, "w") as f:
            json.dump({"source": f"results/{plant}/run1/{cfg}.dat", "records": recs,
                       "raw_first_records": raw}, f, separators=(",", ":"))
        print(name, len(recs))


if __name__ == "__main__":
    main()
