"""Build-kernel time on device-produced records: the build repeated on one
produced batch vs the build right after each producer launch (closed-loop
pattern), and on host-made records bound from torch (the bench pattern).
usage: python tools/time_produce_build.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch, synthetic_operating_points, synthetic_u_old  # noqa: E402

B, K = 65536, 9
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
xs, us, ys = synthetic_operating_points(cfg, B, seed=77, n_distinct=2048)
tx, tu, ty = (torch.from_numpy(a).cuda() for a in (xs, us, ys))
lin, u, du, ws = synthetic_batch(cfg, B, seed=1002, n_distinct=2048)
tl = torch.from_numpy(lin).cuda()
S = cfg.S
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr)
    ctx.set_state(synthetic_u_old(cfg, B, np.random.default_rng(78)), np.zeros((B * S, cfg.nV)),
                  np.zeros(B * S, np.uint32))
    ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
    ctx.build(); ctx.init_warmstart()
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        for _ in range(8):
            ctx.build()
        ctx.synchronize()

    def timed(fn, n=30):
        ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_BUILD,))
        for _ in range(n):
            fn()
        ctx.synchronize()
        ms, k = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
        ctx.enable_timing(False)
        return ms / k

    for rep in range(2):
        ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
        a = timed(lambda: ctx.build())
        b = timed(lambda: (ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr()), ctx.build()))
        def c_():
            ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
            ctx.synchronize(); time.sleep(0.0005)
            ctx.build()
        c = timed(c_)
        ctx.bind_lin(tl.data_ptr())
        d = timed(lambda: ctx.build())
        ctx.bind_lin(0)
        print(f"build on produced records, repeated {a:.4f} ms; right after the producer {b:.4f} ms; "
              f"after the producer + 0.5 ms idle {c:.4f} ms; host records bound {d:.4f} ms", flush=True)
