"""cmpc_step fused (one launch) against split (build + iterate, two launches)
in a back-to-back step loop (NB resident batches, step i on batch i % NB,
the move applied), alternating from the same snapshot, wall time per step
and the results compared bit for bit.  GPU only.
usage: python tools/step_variant_ab.py plant ctype p K B [B ...]"""
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

plant, ctype, p, K = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
cfg = cmpc.reference_config(plant, ctype, p=p)
arr = cmpc.controller_arrays(cfg, reference_setup(plant, ctype))
NB, STEPS = 4, 200
names = {cmpc.CMPC_STEP_SPLIT: "split", cmpc.CMPC_STEP_FUSED: "fused", cmpc.CMPC_STEP_AUTO: "auto"}
for B in [int(a) for a in sys.argv[5:]]:
    recs, sts = [], []
    for b in range(NB):
        lin, u, du, w = synthetic_batch(cfg, B, seed=40 + b, n_distinct=min(B, 256))
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
    ctx.synchronize()
    snap = [tuple(a.clone() for a in st) for st in sts]
    finals = {}
    for rnd in range(3):
        for v in (cmpc.CMPC_STEP_AUTO, cmpc.CMPC_STEP_SPLIT, cmpc.CMPC_STEP_FUSED):
            for st, sn in zip(sts, snap):
                for a, a0 in zip(st, sn):
                    a.copy_(a0)
            try:
                ctx.set_step_variant(v)
                t = time.perf_counter()
                while time.perf_counter() - t < 0.2:  # hold the clock (no move)
                    for i in range(8):
                        bind(i)
                        ctx.build()
                    ctx.synchronize()
                for st, sn in zip(sts, snap):
                    for a, a0 in zip(st, sn):
                        a.copy_(a0)
                torch.cuda.synchronize()
                t = time.perf_counter()
                for i in range(STEPS):
                    bind(i)
                    ctx.step(K, cmpc.CMPC_APPLY_MOVE)
                ctx.synchronize()
                us = (time.perf_counter() - t) / STEPS * 1e6
                fused = ctx.last_step_fused()
                print(f"{plant}-{ctype} p={p} K={K} B={B} round {rnd} {names[v]:5s} (fused {int(fused)}): "
                      f"{us:7.2f} us per step", flush=True)
                finals[names[v]] = [a.cpu().numpy().copy() for st in sts for a in st]
            except Exception as e:
                print(f"{names[v]} n/a: {str(e)[:60]}", flush=True)
    same = all(np.array_equal(a.view(np.uint8), b.view(np.uint8))
               for a, b in zip(finals.get("split", []), finals.get("fused", [])))
    print(f"B={B}: split and fused states bit-identical after {STEPS} steps: {same}", flush=True)
    ctx.close()
