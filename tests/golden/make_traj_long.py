#!/usr/bin/env python3
"""Extract the whole recorded closed-loop trajectories of the reference (all
10 000 records, 500 s at Ts = 0.05) into tests/golden/traj_long.npz: per
configuration the controller output u(t) and the plant output y(t) as
float32 (the .dat files print 6 significant digits; float32 holds every
6-digit decimal exactly enough to print it back unchanged, FLT_DIG = 6).

Run once in the build container (needs /root/reference; the GPU box never
reads the reference).  Data only.  SURVEY.md §4: every run and every
coop1..9 / ncoop1..9 file of a (plant, controller) holds the same trajectory,
so run1's coop9 / ncoop9 / centralized stand for all of them.

With the harness's observer gain identified as M = [0; I] (tools/
fit_observer_gain.py), the device closed loop reproduces these records
(tests/test_closed_loop_golden.py).
"""
import os

import numpy as np

REF = "/root/reference/results"
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = [("parallel", "centralized"), ("parallel", "coop9"), ("parallel", "ncoop9"),
         ("serial", "centralized"), ("serial", "coop9"), ("serial", "ncoop9")]


def records(path):
    with open(path) as f:
        lines = f.read().split("\n")
    t, u, y = [], [], []
    i = 0
    while i + 5 <= len(lines) and lines[i].strip():
        t.append(float(lines[i]))
        u.append([float(v) for v in lines[i + 2].split()])
        y.append([float(v) for v in lines[i + 3].split()])
        i += 6
    return np.array(t), np.array(u), np.array(y)


def main():
    out = {}
    for plant, cfg in CASES:
        t, u, y = records(os.path.join(REF, plant, "run1", cfg + ".dat"))
        assert np.allclose(t, 0.05 * np.arange(len(t)), atol=1e-9), (plant, cfg)
        name = f"{plant[:3]}_{cfg}"
        u32, y32 = u.astype(np.float32), y.astype(np.float32)
        for a, b in ((u, u32), (y, y32)):   # the 6-digit values survive float32
            assert all("%.6g" % p == "%.6g" % float(q) for p, q in zip(a.ravel(), b.ravel()))
        out[name + "_u"], out[name + "_y"] = u32, y32
        print(name, len(t))
    np.savez_compressed(os.path.join(HERE, "traj_long.npz"), **out)


if __name__ == "__main__":
    main()
