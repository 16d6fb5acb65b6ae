"""Would a placement that groups scenarios by their active working sets make
the headline's iterate faster?  The bench's step loop (NB resident batches,
step i on batch i % NB, build + K iterations, the move applied) after the
settle steps, timed with the iterate's events, twice from the same states:
as drawn, and with every batch's scenarios permuted (records and controller
state alike) so that scenarios whose QPs hold active constraints are
adjacent.  The permutation is an experiment on the host; each QP is solved
identically wherever it sits.  GPU only.
usage: python tools/iterate_sorted_ab.py [B] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 40
NB, K = 4, 9
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
S = cfg.S
host = []
for b in range(NB):
    lin, u, du, w = synthetic_batch(cfg, B, seed=1002 + b, n_distinct=min(B, 2048))
    host.append([lin, u, du, w.view(np.int32)])
ctx = cmpc.Context(cfg, B)
ctx.configure(arr)


def upload(hb):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in hb]


def run(dev, label):
    def bind(i):
        d = dev[i % NB]
        ctx.bind_lin(d[0].data_ptr())
        ctx.bind_state(d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr())

    for i in range(32):  # warm the clock
        bind(i)
        ctx.step(K, 0)
    ctx.synchronize()
    ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_ITERATE,))
    for i in range(STEPS):
        bind(i)
        ctx.step(K, cmpc.CMPC_APPLY_MOVE)
    ctx.synchronize()
    ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
    ctx.enable_timing(False)
    print(f"{label:10s} iterate {ms / n * 1e3:7.2f} us over {n} launches", flush=True)


# the settled states: init + a few steps without the move, then copy back
dev = [upload(hb) for hb in host]
for b in range(NB):
    ctx.bind_lin(dev[b][0].data_ptr())
    ctx.bind_state(dev[b][1].data_ptr(), dev[b][2].data_ptr(), dev[b][3].data_ptr())
    ctx.build()
    ctx.init_warmstart()
for i in range(8):
    d = dev[i % NB]
    ctx.bind_lin(d[0].data_ptr())
    ctx.bind_state(d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr())
    ctx.step(K, 0)
ctx.synchronize()
settled = [[t.cpu().numpy() for t in d] for d in dev]
for rnd in range(2):
    for order in ("drawn", "grouped"):
        hb_all = []
        for b in range(NB):
            lin, u, du, w = (a.copy() for a in settled[b])
            if order == "grouped":
                act = (w.view(np.uint32).reshape(B, S) != 0).sum(axis=1)  # active QPs of the scenario
                perm = np.argsort(-act, kind="stable")
                qp = (perm[:, None] * S + np.arange(S)[None, :]).reshape(-1)
                lin, u, du, w = lin[qp], u[qp], du[qp], w[qp]
            hb_all.append([lin, u, du, w])
        if rnd == 0 and order == "grouped":
            act = (hb_all[0][3].view(np.uint32).reshape(B, S) != 0).any(axis=1)
            print(f"scenarios with an active QP: {act.mean():.3f}; 32-scenario waves with one: drawn "
                  f"{(settled[0][3].view(np.uint32).reshape(-1, 64) != 0).any(axis=1).mean():.3f}, grouped "
                  f"{act.reshape(-1, 32).any(axis=1).mean():.3f}", flush=True)
        run([upload(hb) for hb in hb_all], order)
ctx.close()
