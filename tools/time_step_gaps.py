"""Per-step wall time of the bench step (coop-par p=50, K=9, B=65536) with
and without the HIP timing events, against the sum of the kernel times:
what the launch gaps and the events cost.
usage: python tools/time_step_gaps.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

B, K, STEPS = 65536, 9, 100
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
lin, u, du, ws = synthetic_batch(cfg, B, seed=3, n_distinct=2048)
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr)
    ctx.set_state(u, du, ws)
    ctx.upload_lin(lin)
    ctx.build()
    ctx.init_warmstart()
    for _ in range(10):
        ctx.step(K, 0)
    ctx.synchronize()
    for timing in (False, True, "build", False, True, "build"):
        if timing == "build":
            ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_BUILD,))
        else:
            ctx.enable_timing(timing)
        t0 = time.perf_counter()
        for _ in range(STEPS):
            ctx.step(K, 0)
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / STEPS * 1e3
        line = f"timing events {'off' if not timing else 'on ' if timing is True else timing}: {dt:.4f} ms per step"
        if timing is True:
            bms, nb = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
            ims, ni = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
            ks = bms / nb + ims / ni
            line += f"  kernels {ks:.4f} ms (build {bms / nb:.4f}, iterate {ims / ni:.4f}), gap {dt - ks:.4f} ms"
        if timing == "build":
            bms, nb = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
            line += f"  build {bms / nb:.4f} ms"
        print(line, flush=True)
