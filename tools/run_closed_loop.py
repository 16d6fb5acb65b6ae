#!/usr/bin/env python3
"""The reference's closed-loop timing executables (tests/<ctrl>-<plant>-with-
timing.cc + the missing common-simulation.inc), batched on one MI355X:
B identical or perturbed scenarios of plant + NerveCenter, scenario 0
written in the reference's results/*.dat format.

usage: run_closed_loop.py <par|ser> <cent|coop|ncoop> [--setup FILE] [--steps N]
                          [--batch B] [--p P] [--out FILE] [--gain G] [--perturb E]

The observer gain defaults to the reference runs' M = [0; I]
(cmpc.reference_observer_gain, identified from their records); --gain G uses
[0; G I] instead.  The setup's `simulation` segments step the plant-input
offset (ClosedLoop.set_segments).  With the defaults and --steps 10000 the
written records equal the reference's results/<plant>/run1/<cfg>.dat to the
printed digits except the wall-time line (tests/test_closed_loop_golden.py).
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
    ap.add_argument("--gain", type=float, default=None)
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
    Mg = cmpc.reference_observer_gain(cfg)
    if args.gain is not None:
        Mg = Mg * args.gain
    assert Mg.shape[0] == L.nobs
    B = args.batch
    rng = np.random.default_rng(0)
    xs = np.tile(x0, (B, 1))
    if args.perturb:
        xs[1:] *= 1 + args.perturb * rng.standard_normal((B - 1, len(x0)))
    loop = ClosedLoop(cfg, arr, [Mg] * cfg.S, xs, np.tile(u0, (B, 1)), setup.n_iterations)
    writer = DatWriter(args.out) if args.out else None
    try:
        if setup.segments:
            loop.set_segments(setup.segments, u0)
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
        "observer_gain": f"[0; {1.0 if args.gain is None else args.gain} I]"}))


if __name__ == "__main__":
    main()
