"""Closed-loop stress with the device observer: status histogram per step.
usage: closed_loop_observer.py [B] [steps] [M scale ...]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np
import torch
torch.cuda.init()
import cmpc
from cmpc.configs import reference_setup
from cmpc.synthetic import synthetic_operating_points, synthetic_u_old

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
# gain kinds: a number = random gain of that scale; "distA" = disturbance-only
# gain [0; A*I] (offset-free MPC convention)
scales = sys.argv[3:] or ["0", "0.01"]
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
S, K = cfg.S, 9
xs, us, ys = synthetic_operating_points(cfg, B, seed=77, n_distinct=min(B, 2048))
tx, tu, ty = (torch.from_numpy(a).cuda() for a in (xs, us, ys))
for ms in scales:
    for uo_kind in ("zero", "synthetic"):
        with cmpc.Context(cfg, B) as ctx:
            ctx.configure(arr)
            rng = np.random.default_rng(79)
            for s in range(S):
                nobs, no = ctx.layout.nobs, ys.shape[1]
                if ms.startswith("dist"):
                    Mg = np.zeros((nobs, no))
                    Mg[cfg.ns:cfg.ns + cfg.ndist, :cfg.ndist] = float(ms[4:]) * np.eye(cfg.ndist, no).T[:cfg.ndist, :]
                else:
                    Mg = float(ms) * rng.standard_normal((nobs, no))
                ctx.set_observer(s, Mg)
            u0 = np.zeros((B * S, cfg.nu_tot)) if uo_kind == "zero" else synthetic_u_old(cfg, B, np.random.default_rng(78))
            ctx.set_state(u0, np.zeros((B * S, cfg.nV)), np.zeros(B * S, np.uint32))
            ctx.observer_init(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
            ctx.build(); ctx.init_warmstart()
            line = []
            for t in range(steps):
                if t:
                    ctx.observe_step(tu.data_ptr(), ty.data_ptr())
                    ctx.build()
                ctx.iterate(K)
                _, st, _ = ctx.download()
                ctx.observe_apply()
                line.append("%d:%s" % (t, dict(zip(*np.unique(st, return_counts=True)))))
            uo, _, _ = ctx.get_state()
            print(f"M={ms} u_old0={uo_kind}: " + " ".join(line), flush=True)
            print(f"   |u_old| max {np.abs(uo).max():.3g}", flush=True)
