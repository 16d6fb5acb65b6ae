"""cmpc_control_step as one launch (AUTO) against its three calls
(CMPC_STEP_SPLIT: observe_step + step + observe_apply) in a back-to-back loop
of T control steps on device arrays, alternating, wall time per step; the
plans compared bit for bit.  GPU only.
usage: python tools/control_step_ab.py plant ctype p K B [B ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import cmpc  # noqa: E402
from test_observer import setup  # noqa: E402  (the observer tests' operating points)

plant, ctype, p, K = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
T = 100
for B in [int(a) for a in sys.argv[5:]]:
    cfg, arr, dims, L, rng, x, u, y, M = setup(plant, ctype, p, B, 29, xs=1e-4, us=1e-3, ms=0.01)
    nq = B * cfg.S
    ys = [torch.from_numpy(np.ascontiguousarray(y * (1 + 3e-4 * rng.normal(size=y.shape)))).cuda()
          for _ in range(8)]
    tu = torch.from_numpy(np.ascontiguousarray(u)).cuda()
    res = {}
    for rnd in range(3):
        for variant, name in ((cmpc.CMPC_STEP_AUTO, "one launch"), (cmpc.CMPC_STEP_SPLIT, "three calls")):
            with cmpc.Context(cfg, B, device=0) as ctx:
                ctx.configure(arr)
                ctx.set_state(np.zeros((nq, cfg.nu_tot)), np.zeros((nq, cfg.nV)), np.zeros(nq, np.uint32))
                for s_ in range(cfg.S):
                    ctx.set_observer(s_, M[s_])
                ctx.observer_init(torch.from_numpy(np.ascontiguousarray(x)).cuda().data_ptr(), tu.data_ptr(),
                                  torch.from_numpy(np.ascontiguousarray(y)).cuda().data_ptr())
                ctx.build()
                ctx.init_warmstart()
                ctx.set_step_variant(variant)
                for i in range(20):  # warm
                    ctx.control_step(tu.data_ptr(), ys[i % 8].data_ptr(), K)
                ctx.synchronize()
                t = time.perf_counter()
                for i in range(T):
                    ctx.control_step(tu.data_ptr(), ys[i % 8].data_ptr(), K)
                ctx.synchronize()
                us = (time.perf_counter() - t) / T * 1e6
                fused = ctx.last_step_fused()
                res[name] = ctx.download()[0].copy()
                print(f"{plant}-{ctype} p={p} K={K} B={B} ({nq} QPs) round {rnd} {name:11s} (fused {int(fused)}): "
                      f"{us:8.2f} us per step", flush=True)
    print(f"B={B}: plans bit-identical: {np.array_equal(res['one launch'], res['three calls'])}", flush=True)
