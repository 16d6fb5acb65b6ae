"""Config 5 (cent-par p = 200, 1 024 QPs, K = 1): per-step wall time of cmpc_step
in a Python loop with and without binding a second batch per step and with
and without CMPC_APPLY_MOVE (host issue time beside it).  GPU only.
usage: python tools/time_apply_move.py [split]"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "compressor-mpc_amd"))
import numpy as np, torch
import cmpc
from cmpc.configs import reference_setup
from cmpc.synthetic import synthetic_batch
cfg = cmpc.reference_config("par", "cent", p=200)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "cent"))
B, NB = 1024, 2
recs, sts = [], []
for b in range(NB):
    lin, u, du, w = synthetic_batch(cfg, B, seed=4000 + 31 * b, n_distinct=1024)
    recs.append(torch.from_numpy(lin).cuda()); sts.append(tuple(torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (u, du, w.view(np.int32))))
ctx = cmpc.Context(cfg, B); ctx.configure(arr)
if len(sys.argv) > 1 and sys.argv[1] == "split":  # build + iterate launches instead of AUTO
    ctx.set_step_variant(cmpc.CMPC_STEP_SPLIT)
def bind(i):
    st = sts[i % NB]; ctx.bind_lin(recs[i % NB].data_ptr()); ctx.bind_state(st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr())
for b in range(NB):
    bind(b); ctx.build(); ctx.init_warmstart()
def run(n, dobind, flags):
    ctx.synchronize(); t0 = time.perf_counter(); th = 0.0
    for k in range(n):
        a = time.perf_counter()
        if dobind: bind(k)
        ctx.step(1, flags)
        th += time.perf_counter() - a
    ctx.synchronize(); return (time.perf_counter() - t0) / n * 1e6, th / n * 1e6
for _ in range(3): run(200, True, 0)
for dobind in (False, True):
    for flags in (0, cmpc.CMPC_APPLY_MOVE):
        print("bind", dobind, "flags", flags, "us/step, host us/step: %.1f %.1f" % run(200, dobind, flags), flush=True)
