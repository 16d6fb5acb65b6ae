"""Lane-per-QP against row-per-QP iterate (CMPC_SOLVE_LANE / CMPC_SOLVE_ROWS)
in the bench's step loop (NB resident batches, step i on batch i % NB, build
+ K iterations with the move applied), by the iterate's events, alternating
from the same snapshot; and the two solvers' plans, statuses and working sets
compared bit for bit after the loop.  GPU only.
usage: python tools/solver_variant_ab.py [p=50] [plant=par] [c=coop] [K=9] [B ...]"""
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

NB, STEPS = 4, 40
args = sys.argv[1:]
opt = {"p": "50", "plant": "par", "c": "coop", "K": "9"}
while args and "=" in args[0]:
    k, v = args.pop(0).split("=", 1)
    opt[k] = v
P, K = int(opt["p"]), int(opt["K"])
cfg = cmpc.reference_config(opt["plant"], opt["c"], p=P)
arr = cmpc.controller_arrays(cfg, reference_setup(opt["plant"], opt["c"]))
for B in [int(a) for a in args] or [65536]:
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
    for i in range(8):
        bind(i)
        ctx.step(K, 0)
    ctx.synchronize()
    snap = [tuple(a.clone() for a in st) for st in sts]
    finals = {}
    for rnd in range(3):
        for sv, name in ((cmpc.CMPC_SOLVE_LANE, "lane"), (cmpc.CMPC_SOLVE_ROWS, "rows")):
            for st, sn in zip(sts, snap):
                for a, a0 in zip(st, sn):
                    a.copy_(a0)
            ctx.set_solve_variant(sv)
            torch.cuda.synchronize()
            t = time.perf_counter()
            while time.perf_counter() - t < 0.25:  # hold the clock
                for k in range(8):
                    bind(k)
                    ctx.build()
                ctx.synchronize()
            ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_ITERATE,))
            for i in range(STEPS):
                bind(i)
                ctx.step(K, cmpc.CMPC_APPLY_MOVE)
            ctx.synchronize()
            ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
            ctx.enable_timing(False)
            used = ctx.last_solve_kernel()
            print(f"{opt['plant']}-{opt['c']} p {P} K {K} B {B:6d} round {rnd} {name}: iterate {ms / n * 1e3:7.2f} us (kernel {used})", flush=True)
            finals[name] = [a.cpu().numpy().copy() for st in sts for a in st]
    same = all(np.array_equal(a.view(np.uint8), b.view(np.uint8)) for a, b in zip(finals["lane"], finals["rows"]))
    print(f"B {B:6d}: states after {STEPS} steps bit-identical between the solvers: {same}", flush=True)
    ctx.close()
