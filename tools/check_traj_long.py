#!/usr/bin/env python3
"""Run the device closed loop (cmpc/driver.py, observer gain M = [0; g I]) of
the six reference configurations for the whole recorded horizon and compare
u(t) and y(t) with the reference's records (tests/golden/traj_long.npz, 6
printed digits).  Reports the first differing record, the number of records
that differ and the largest relative difference.
The setup files' `simulation` segments step the plant-input offset at 50 s
(driver.ClosedLoop.set_segments); `shift` moves that step by whole samples
(to test when the harness applied it).
usage: python tools/check_traj_long.py [steps] [gain] [shift]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np  # noqa: E402

CASES = [("par", "cent", "par_centralized"), ("par", "coop", "par_coop9"), ("par", "ncoop", "par_ncoop9"),
         ("ser", "cent", "ser_centralized"), ("ser", "coop", "ser_coop9"), ("ser", "ncoop", "ser_ncoop9")]


def six(a):
    """6 printed digits; |v| < 1e-12 as 0 (the parallel plant's y[2] is a
    difference of two equal compressors' values: 0 up to one ulp of
    cancellation, printed by the reference as 0 or +-2.22045e-16)."""
    return np.array([0.0 if abs(v) < 1e-12 else float("%.6g" % v) for v in np.ravel(a)]).reshape(np.shape(a))


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    g = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    shift = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    import torch
    torch.cuda.init()
    import cmpc
    from cmpc._abi import CmpcDims
    from cmpc.configs import reference_setup
    from cmpc.driver import ClosedLoop
    gold = np.load(os.path.join(ROOT, "tests", "golden", "traj_long.npz"))
    for plant, ctype, name in CASES:
        ur = gold[name + "_u"].astype(np.float64)
        yr = gold[name + "_y"].astype(np.float64)
        n = min(steps, len(ur))
        cfg = cmpc.reference_config(plant, ctype)
        setup = reference_setup(plant, ctype)
        arr = cmpc.controller_arrays(cfg, setup)
        L = cmpc.layout_of(CmpcDims.from_config(cfg, 1))
        x0, u0 = cmpc.plant_default(cfg.plant)
        Mg = np.zeros((L.nobs, 4))
        Mg[cfg.ns:cfg.ns + cfg.ndist, :cfg.ndist] = g * np.eye(cfg.ndist)
        loop = ClosedLoop(cfg, arr, [Mg] * cfg.S, x0[None, :], u0[None, :], setup.n_iterations)
        loop.set_segments([(d, te + shift * 0.05) for d, te in setup.segments], u0)
        ub = torch.zeros(n, 4, dtype=torch.float64, device="cuda")
        yb = torch.zeros(n, 4, dtype=torch.float64, device="cuda")
        t0 = time.perf_counter()
        loop.initialize()
        for k in range(n):
            _, y = loop.step()
            ub[k].copy_(loop.u_ctrl[0])
            yb[k].copy_(y[0])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        loop.close()
        u, y = ub.cpu().numpy(), yb.cpu().numpy()
        bad_u = np.any(six(u) != six(ur[:n]), axis=1)
        bad_y = np.any(six(y) != six(yr[:n]), axis=1)
        rel = lambda a, b: float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-3)))
        print(json.dumps({"case": name, "gain": g, "shift": shift, "steps": n,
                          "first_u_diff": int(np.argmax(bad_u)) if bad_u.any() else None,
                          "first_y_diff": int(np.argmax(bad_y)) if bad_y.any() else None,
                          "u_records_differing": int(bad_u.sum()), "y_records_differing": int(bad_y.sum()),
                          "max_rel_u": rel(u, ur[:n]), "max_rel_y": rel(y, yr[:n]),
                          "y_diff_examples": [(int(k), six(y[k]).tolist(), yr[k].tolist())
                                              for k in np.flatnonzero(bad_y)[:3]],
                          "seconds": round(el, 2)}), flush=True)


if __name__ == "__main__":
    main()
