"""Iterate-kernel time by phase: K = 0 (loads, H^-1, stores), K = 1 and K = 9,
on a repeated batch (warm start from the same QP's last solve) and in the
bench's rotation (4 input batches, build before every iterate, so the warm
start comes from another QP).  usage: python tools/time_iterate_phases.py"""
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

B = int(os.environ.get("CMPC_TI_B", "65536"))
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
batches = []
for b in range(4):
    lin, u, du, ws = synthetic_batch(cfg, B, seed=1002 + b, n_distinct=2048)
    if b == 0:
        u0, du0, ws0 = u, du, ws
    batches.append(torch.from_numpy(lin).cuda())
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr)
    ctx.set_state(u0, du0, ws0)
    ctx.bind_lin(batches[0].data_ptr())
    ctx.build()
    ctx.init_warmstart()
    t_end = time.perf_counter() + 0.3
    i = 0
    while time.perf_counter() < t_end:
        for _ in range(8):
            ctx.bind_lin(batches[i % 4].data_ptr()); i += 1
            ctx.step(9, 0)
        ctx.synchronize()
    for K in (0, 1, 9):
        ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_ITERATE,))
        for r in range(40):
            ctx.bind_lin(batches[(i + r) % 4].data_ptr())
            ctx.step(K, 0)
        i += 40
        ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
        rot = ms / n
        ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_ITERATE,))
        for r in range(40):
            ctx.iterate(K)
        ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
        ctx.enable_timing(False)
        _, _, nw = ctx.download()
        print(f"K={K}: rotation {rot:.4f} ms   repeated batch {ms / n:.4f} ms", flush=True)
