"""Shared construction of the reference's step-0 golden cases
(tests/golden/step0.json, written by tests/golden/make_step0_golden.py)."""
import json
import os

import numpy as np

from cmpc.configs import PLANT_N_INPUTS, SetupFile, reference_config
from cmpc.problem import controller_arrays

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "step0.json")
NAMES = ("cent-par", "coop-par", "ncoop-par", "cent-ser", "coop-ser", "ncoop-ser")


def load():
    return json.load(open(GOLDEN))["configs"]


def case(name, p=None):
    g = load()[name]
    ctype, plant = name.split("-")
    cfg = reference_config(plant, ctype) if p is None else reference_config(plant, ctype, p=p)
    blk = cfg.ny * cfg.ny
    yw = g["ywt"]
    ywt = [yw[i * blk:(i + 1) * blk] for i in range(cfg.S)] if len(yw) == blk * cfg.S else [yw] * cfg.S
    setup = SetupFile(n_iterations=g["n_iterations"], yref=g["yref"], uwt=g["uwt"], ywt=ywt,
                      constraints_lower=g["constraints_lower"],
                      constraints_upper=g["constraints_upper"],
                      rate_lower=g["rate_lower"], rate_upper=g["rate_upper"],
                      segments=segments(cfg, g["simulation"]))
    return cfg, setup, controller_arrays(cfg, setup), g


def segments(cfg, flat):
    """The `simulation` block as [(offset change (n_inputs), end time)]."""
    n = PLANT_N_INPUTS[cfg.plant] + 1
    assert len(flat) % n == 0, flat
    return [(flat[i:i + n - 1], flat[i + n - 1]) for i in range(0, len(flat), n)]


def step0_records(cfg, dims, layout, lin_record_fn, x0, u_full, y):
    """Lin records of the t=0 step: linearisation at (x0, u_offset), zero
    augmented deviation (dx_init = 0, ObserveAPosteriori adds 0), measured y."""
    recs = []
    for s in range(cfg.S):
        r = lin_record_fn(cfg, dims, s, x0, u_full)
        r[layout.off_x:layout.off_x + layout.naug] = 0.0
        r[layout.off_y:layout.off_y + cfg.ny] = np.asarray(y)[cfg.out_idx[s]]
        recs.append(r)
    return np.ascontiguousarray(np.stack(recs))


def assert_six_digits(u, golden):
    """results/*.dat print %g with 6 significant digits."""
    for a, b in zip(u, golden):
        if b == 0.0:
            assert abs(a) <= 1e-12, (u, golden)
        else:
            assert float("%.6g" % a) == b, (u, golden)
