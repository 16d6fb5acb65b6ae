"""Time series of the bench step (coop-par p=50, K=9, B=65536, four resident
input batches) from a cold start: per-block mean step time and build-kernel
time, to size the untimed settle phase of bench.py (the clock the chip holds
under this load ramps up over the first ~second).
usage: python tools/time_clock_ramp.py [seconds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import torch  # noqa: E402
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

T = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
B, K = 65536, 9
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
batches, st = [], None
for b in range(4):
    lin, u, du, ws = synthetic_batch(cfg, B, seed=1002 + b, n_distinct=2048)
    if st is None:
        st = (u, du, ws)
    batches.append(torch.from_numpy(lin).to("cuda:0"))
torch.cuda.synchronize()
with cmpc.Context(cfg, B, device=0) as ctx:
    ctx.configure(arr)
    ctx.set_state(*st)
    ctx.bind_lin(batches[0].data_ptr())
    ctx.build()
    ctx.init_warmstart()
    ctx.synchronize()
    t_start = time.perf_counter()
    i = 0
    while time.perf_counter() - t_start < T:
        ctx.enable_timing(True)
        t0 = time.perf_counter()
        for _ in range(25):
            ctx.bind_lin(batches[i % 4].data_ptr())
            ctx.step(K, 0)
            i += 1
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / 25 * 1e3
        ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
        ctx.enable_timing(False)
        print(f"t={time.perf_counter() - t_start:6.3f} s  step {dt:.4f} ms  build {ms / n:.4f} ms", flush=True)
