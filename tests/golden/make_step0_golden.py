#!/usr/bin/env python3
"""Extract the reference's step-0 golden records into tests/golden/step0.json.

Run once in the build container (needs /root/reference; the GPU box never
reads the reference).  The fixture holds data only:

* the t=0 record of results/<plant>/run1/<cfg>.dat: plant state x (line 2),
  applied control input u (line 3), plant output y (line 4) — the record
  layout is SURVEY.md §4; all five runs agree to the printed 6 digits;
* the run parameters of setup/setup-<cfg>-<plant>: n-iterations, yref, uwt,
  ywt (one block per sub-controller for the distributed types), constraints,
  simulation (segments: plant-input offset change, end time).

The t=0 input is independent of the (missing) observer gain M, because the
first ObserveAPosteriori adds M*(y - y_old - C*0) = 0
(libs/observer.cc:24-40, libs/distributed_controller.cc:27-43).
"""
import json
import os
import sys

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "step0.json")


KEYS = ("n-iterations", "n-timing-iterations", "folder-name", "output-filename",
        "yref", "uwt", "ywt", "constraints-lower", "constraints-upper",
        "constraints-rate-lower", "constraints-rate-upper", "simulation")


def read_setup(path):
    """Key/value blocks as in include/read_files.h:13-81 (blank-line separated)."""
    blocks, key = {}, None
    for line in open(path):
        s = line.strip()
        if not s or s.startswith("#"):
            continue
        toks = s.split()
        if toks[0] in KEYS:
            key = toks[0]
            blocks.setdefault(key, [])
            continue
        if key is not None:
            blocks[key].append([float(t) if _isnum(t) else t for t in toks])
    return blocks


def _isnum(t):
    try:
        float(t)
        return True
    except ValueError:
        return False


def first_record(path):
    with open(path) as fh:
        lines = [next(fh) for _ in range(5)]
    vec = lambda l: [float(t) for t in l.split()]
    return {"t": float(lines[0]), "x": vec(lines[1]), "u": vec(lines[2]),
            "y": vec(lines[3]), "wall_ns": float(lines[4])}


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present")
    out = {"source": "katie-jones/compressor-mpc results/*/run1/*.dat t=0 records + setup/*",
           "configs": {}}
    for plant, pdir in (("par", "parallel"), ("ser", "serial")):
        for ctype, fname in (("cent", "centralized.dat"), ("coop", "coop9.dat"),
                             ("ncoop", "ncoop9.dat")):
            setup = read_setup(os.path.join(REF, "setup", f"setup-{ctype}-{plant}"))
            rec = first_record(os.path.join(REF, "results", pdir, "run1", fname))
            # all five runs agree at t=0 (determinism check)
            for run in range(2, 6):
                r2 = first_record(os.path.join(REF, "results", pdir, f"run{run}", fname))
                assert r2["u"] == rec["u"] and r2["y"] == rec["y"], (plant, ctype, run)
            flat = lambda rows: [v for r in rows for v in r]
            cfg = {
                "plant": pdir,
                "controller": ctype,
                "n_iterations": int(setup["n-iterations"][0][0]),
                "yref": flat(setup["yref"]),
                "uwt": flat(setup["uwt"]),
                "ywt": flat(setup["ywt"]),
                "constraints_lower": flat(setup["constraints-lower"]),
                "constraints_upper": flat(setup["constraints-upper"]),
                "rate_lower": flat(setup["constraints-rate-lower"]),
                "rate_upper": flat(setup["constraints-rate-upper"]),
                "simulation": flat(setup["simulation"]),
                "x0": rec["x"], "u0": rec["u"], "y0": rec["y"],
            }
            out["configs"][f"{ctype}-{plant}"] = cfg
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
