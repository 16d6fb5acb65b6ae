#!/usr/bin/env python3
"""The reference's closed-loop timing executables (tests/<ctrl>-<plant>-with-
timing.cc + the missing common-simulation.inc), batched on one MI355X:
B identical or perturbed scenarios of plant + NerveCenter, scenario 0
written in the reference's results/*.dat format.

usage: run_closed_loop.py <par|ser> <cent|coop|ncoop> [--setup FILE] [--steps N]
                          [--batch B] [--p P] [--out FILE] [--gain G] [--perturb E]

The observer gain of the reference harness is unknown (its
common-simulation.inc is missing); --gain G uses the disturbance-only gain
[0; G I] (offset-free MPC convention).  Record 0 and the plant state of
record 1 do not depend on it and equal the reference's results (tests/
test_sim.py); later records do.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("plant", choices=["par", "ser"])
    ap.add_argument("ctype", choices=["cent", "coop", "ncoop"])
    ap.add_argument("--setup", help="setup file in the reference's format (default: the reference's values)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--p", type=int, default=100)
    ap.add_argument("--out", default=None, help=".dat output for scenario 0")
    ap.add_argument("--gain", type=float, default=0.5)
    ap.add_argument("--perturb", type=float, default=0.0, help="relative perturbation of x0 per scenario")
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    import cmpc
    from cmpc._abi import CmpcDims
    from cmpc.configs import SetupFile, reference_setup
    from cmpc.driver import ClosedLoop, DatWriter
    cfg = cmpc.reference_config(args.plant, args.ctype, p=args.p)
    setup = (SetupFile.parse(open(args.setup).read(), cfg) if args.setup
             else reference_setup(args.plant, args.ctype))
    arr = cmpc.controller_arrays(cfg, setup)
    L = cmpc.layout_of(CmpcDims.from_config(cfg, 1))
    x0, u0 = cmpc.plant_default(cfg.plant)
    no = 4
    Mg = np.zeros((L.nobs, no))
    Mg[cfg.ns:cfg.ns + cfg.ndist, :cfg.ndist] = args.gain * np.eye(cfg.ndist)
    B = args.batch
    rng = np.random.default_rng(0)
    xs = np.tile(x0, (B, 1))
    if args.perturb:
        xs[1:] *= 1 + args.perturb * rng.standard_normal((B - 1, len(x0)))
    loop = ClosedLoop(cfg, arr, [Mg] * cfg.S, xs, np.tile(u0, (B, 1)), setup.n_iterations)
    writer = DatWriter(args.out) if args.out else None
    try:
        loop.initialize()
        t0 = time.perf_counter()
        per_step = loop.run(args.steps, writer)
        wall = time.perf_counter() - t0
        _, st, _ = loop.ctx.download()
        _, _, _, sst = loop.sim.download()
    finally:
        if writer:
            writer.close()
        loop.close()
    print(json.dumps({
        "config": f"{args.ctype}-{args.plant} p={args.p} K={setup.n_iterations}",
        "scenarios": B, "steps": args.steps, "ms_per_step": per_step * 1e3,
        "scenario_steps_per_s": B / per_step, "wall_s": wall,
        "qp_status_ok_fraction_last_step": float((st == 0).mean()),
        "plant_step_failures": int(sst.sum()),
        "observer_gain": f"[0; {args.gain} I] (disturbance-only)"}))


if __name__ == "__main__":
    main()
