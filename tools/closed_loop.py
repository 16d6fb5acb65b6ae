"""Closed-loop (device-resident) steps: produce -> build -> iterate(K, apply
move), reporting per step the iterate time, active fraction and mean
working-set changes.  Plant states are synthetic and held fixed (no plant
simulation), so the applied moves accumulate: a stress test of the solver."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np
import torch
import cmpc
from cmpc.configs import reference_setup
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
from cmpc.synthetic import synthetic_operating_points, synthetic_u_old
xs, us, ys = synthetic_operating_points(cfg, B, seed=3, n_distinct=min(B, 2048))
tx, tu, ty = (torch.from_numpy(a).cuda() for a in (xs, us, ys))
S = cfg.S
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr)
    ctx.set_state(synthetic_u_old(cfg, B, np.random.default_rng(4)), np.zeros((B * S, cfg.nV)),
                  np.zeros(B * S, np.uint32))
    ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
    ctx.build(); ctx.init_warmstart()
    ctx.enable_timing(True)
    for t in range(steps):
        ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
        ctx.build()
        ctx.iterate(9, cmpc.CMPC_APPLY_MOVE)
        du, st, nw = ctx.download()
        ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
        ctx.enable_timing(False); ctx.enable_timing(True)
        _, _, ws = ctx.get_state()
        print(f"step {t}: iterate {ms:.4f} ms  ok {np.mean(st == 0):.4f}  active {np.mean(ws != 0):.3f}"
              f"  mean nwsr(last) {nw.mean():.2f}  max {nw.max()}", flush=True)
