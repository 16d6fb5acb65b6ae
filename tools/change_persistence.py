"""How persistent are the headline's working-set changes across a batch's
visits?  The bench's step loop (NB resident batches, step i on batch i % NB,
build + K iterations with the move applied), traced: per scenario, whether
any of its QPs changed its working set in Jacobi iteration 0, at every step.
Reports, per pair of consecutive visits of one batch, the overlap of the
changing scenarios and the fraction of 32-scenario waves (64 QPs) with a
change in the natural order and with the scenarios ordered by the previous
visit's flags (a placement that packs likely-changing scenarios together).
GPU only.  usage: python tools/change_persistence.py [B] [steps]"""
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
recs, sts = [], []
for b in range(NB):
    lin, u, du, w = synthetic_batch(cfg, B, seed=1002 + b, n_distinct=min(B, 2048))
    recs.append(torch.from_numpy(lin).cuda())
    sts.append(tuple(torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (u, du, w.view(np.int32))))
ctx = cmpc.Context(cfg, B)
ctx.configure(arr)


def bind(i):
    st = sts[i % NB]
    ctx.bind_lin(recs[i % NB].data_ptr())
    ctx.bind_state(st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr())


for b in range(NB):
    bind(b)
    ctx.build()
    ctx.init_warmstart()
for i in range(8):  # the bench's warm-up / settle steps (no move)
    bind(i)
    ctx.step(K, 0)
flags = []
for i in range(STEPS):
    bind(i)
    ctx.step(K, cmpc.CMPC_APPLY_MOVE | cmpc.CMPC_TRACE)
    _, ntr = ctx.download_trace(K)
    flags.append(ntr[:, 0].reshape(B, cfg.S).max(axis=1) > 0)  # scenario changed in iteration 0
W = 32  # scenarios per wave (64 QPs)
for i in range(NB, STEPS):
    prev, cur = flags[i - NB], flags[i]
    both = int((prev & cur).sum())
    nat = float(cur.reshape(-1, W).any(axis=1).mean())
    order = np.argsort(~prev, kind="stable")  # previous visit's changers first
    srt = float(cur[order].reshape(-1, W).any(axis=1).mean())
    print(f"step {i:3d} batch {i % NB}: changed {int(cur.sum()):6d} (prev {int(prev.sum()):6d}, both {both:6d}, "
          f"{both / max(1, cur.sum()):.2f} of now)  waves with a change: natural {nat:.3f}, "
          f"ordered by the previous visit {srt:.3f}", flush=True)
ctx.close()
