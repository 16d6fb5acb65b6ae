"""The iterate kernel inside the bench's step loop (NB resident batches, each
with its own state, step i on batch i % NB, build + iterate), by event
timing, against the same kernel re-run on one bound batch (tools/time_small
style): K = 1 and 9, with and without CMPC_APPLY_MOVE.  GPU only.
usage: python tools/time_iterate_bench.py [B]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
NB = 4
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
snap = [tuple(a.clone() for a in st) for st in sts]


def restore():
    for st, sn in zip(sts, snap):
        for a, a0 in zip(st, sn):
            a.copy_(a0)
    torch.cuda.synchronize()
    t = time.perf_counter()
    while time.perf_counter() - t < 0.25:
        for k in range(8):
            bind(k)
            ctx.build()
        ctx.synchronize()


for K in (1, 9):
    for flags, fname in ((0, "no move"), (cmpc.CMPC_APPLY_MOVE, "move")):
        restore()
        ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_ITERATE,))
        for i in range(40):
            bind(i)
            ctx.step(K, flags)
        ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
        ctx.enable_timing(False)
        print(f"step loop    K={K} {fname:8s}: iterate {ms / n * 1e3:7.2f} us", flush=True)
    restore()
    bind(0)
    ctx.build()
    ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_ITERATE,))
    for i in range(40):
        ctx.iterate(K)
    ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
    ctx.enable_timing(False)
    print(f"one batch    K={K}          : iterate {ms / n * 1e3:7.2f} us", flush=True)
    restore()
    ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_ITERATE,))
    for i in range(40):
        bind(i)
        ctx.build()
        ctx.iterate(K)
    ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
    ctx.enable_timing(False)
    print(f"build+iterate K={K} no move: iterate {ms / n * 1e3:7.2f} us", flush=True)
ctx.close()

# working-set changes per step over the timed step loop (CMPC_TRACE), per
# step from the snapshot: the drift of u_old under the applied moves
ctx = cmpc.Context(cfg, B)
ctx.configure(arr)
restore()
tot, per_it, waves_it = [], np.zeros(9, np.int64), np.zeros(9, np.int64)
for i in range(40):
    bind(i)
    ctx.step(9, cmpc.CMPC_APPLY_MOVE | cmpc.CMPC_TRACE)
    _, ntr = ctx.download_trace(9)
    tot.append((int(ntr.sum()), int((ntr.sum(axis=1) > 0).sum()),
                int((ntr.reshape(-1, 32, 9).sum(axis=(1, 2)) > 0).sum())))
    if i >= 8:  # past the restored snapshot's first visit of each batch
        per_it += ntr.sum(axis=0)
        waves_it += (ntr.reshape(-1, 64, 9).sum(axis=1) > 0).sum(axis=0)
print("changes per step (total, QPs with a change, 32-QP groups with a change):", tot, flush=True)
print("steps 8-39, per Jacobi iteration: changes", per_it.tolist(), "waves with a change", waves_it.tolist(),
      "(of", 32 * ntr.shape[0] // 64, "wave-steps)", flush=True)
ctx.close()
