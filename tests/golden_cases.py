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


def _six(v):
    return 0.0 if abs(v) < 1e-12 else float("%.6g" % v)


def six_digit_rows(got, ref, boundary_rel=1e-9):
    """Records of a closed loop against the reference's printed ones (%.6g;
    |v| < 1e-12 counts as 0).  Returns (bad rows, tie rows): a value of `got`
    within boundary_rel of a %.6g rounding boundary (x.xxxxx5 in the 7th
    digit) prints as either neighbour under the last ulp of rounding order, so
    there a reference value one unit away in the 6th digit is a tie, not a
    difference (the solver's arithmetic order is this repository's own, not
    qpOASES'; no decision depends on it)."""
    got = np.asarray(got, dtype=np.float64).reshape(len(got), -1)
    ref = np.asarray(ref, dtype=np.float64).reshape(len(ref), -1)
    bad, tie = set(), set()
    for k in range(len(got)):
        for a, r in zip(got[k], ref[k]):
            sa, sr = _six(a), _six(float(r))
            if sa == sr:
                continue
            if a != 0.0 and abs(a) >= 1e-12:
                e = np.floor(np.log10(abs(a)))
                unit = 10.0 ** (e - 5)
                frac = abs(a) / unit
                near = abs(frac - np.floor(frac) - 0.5) * unit <= boundary_rel * abs(a)
                if near and abs(sa - sr) <= 1.01 * unit:
                    tie.add(k)
                    continue
            bad.add(k)
    return np.array(sorted(bad), dtype=int), np.array(sorted(tie), dtype=int)


def six_digit_strings_ok(printed, ref, full=None, boundary_rel=1e-9):
    """A printed record (strings, %g) against the reference's: equal to 6
    digits, or a rounding-boundary tie.  The printed text cannot tell a tie
    from a real last-digit difference, so a tie needs the full-precision
    values `full` the harness wrote beside it (with_timing's .full file): each
    differing value must lie within boundary_rel of a %.6g rounding boundary
    and one unit of the 6th digit from the reference, the rule of
    six_digit_rows.  Without `full` no tie is accepted.  Returns (equal, tie)."""
    a = [_six(float(v)) for v in printed]
    b = [_six(float(v)) for v in ref]
    if a == b:
        return True, False
    if full is None or len(full) != len(a):
        return False, False
    if [_six(float(v)) for v in full] != a:
        return False, False  # the .full values are not the printed record's
    bad, tie = six_digit_rows([list(map(float, full))], [list(map(float, ref))], boundary_rel)
    return False, bool(len(tie)) and not len(bad)


def read_full(path):
    """with_timing's .full sidecar: per record the u and y values at %.17g."""
    out = []
    for ln in open(path).read().splitlines():
        u, y = ln.split("|")
        out.append(([float(v) for v in u.split()], [float(v) for v in y.split()]))
    return out
