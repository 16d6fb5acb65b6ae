"""Build-kernel time against the kind and place of its input records, same
context and state: host-made records (random observer tail) bound from a
torch tensor or uploaded into the context's buffer, the same with the tail
zeroed, and device-produced records.  usage: python tools/time_build_inputs.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import cmpc  # noqa: E402
from cmpc._abi import CmpcDims  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch, synthetic_operating_points  # noqa: E402

B = 65536
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
L = cmpc.layout_of(CmpcDims.from_config(cfg, B))
lin, u, du, ws = synthetic_batch(cfg, B, seed=1002, n_distinct=2048)
lin0 = lin.copy()
lin0[:, L.off_x:L.off_x + L.naug] = 0.0
t_rand, t_zero = torch.from_numpy(lin).cuda(), torch.from_numpy(lin0).cuda()
xs, us, ys = synthetic_operating_points(cfg, B, seed=77, n_distinct=2048)
tx, tu, ty = (torch.from_numpy(a).cuda() for a in (xs, us, ys))
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr)
    ctx.set_state(u, du, ws)
    ctx.bind_lin(t_rand.data_ptr())
    ctx.build()
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        for _ in range(8):
            ctx.build()
        ctx.synchronize()

    def timed(n=40):
        ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_BUILD,))
        for _ in range(n):
            ctx.build()
        ctx.synchronize()
        ms, k = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
        ctx.enable_timing(False)
        return ms / k

    t_late = torch.empty_like(t_rand)
    t_late.copy_(t_rand)
    torch.cuda.synchronize()
    print("addresses: bound %x, late %x, own %x" % (t_rand.data_ptr(), t_late.data_ptr(), ctx.lin_device_ptr()),
          flush=True)
    ctx2 = cmpc.Context(cfg, B)  # a second context: its own record buffer, bound into the first
    ctx2.upload_lin(lin)
    for rep in range(2):
        r = {}
        ctx.bind_lin(ctx2.lin_device_ptr()); r["host random tail, another context's buffer"] = timed()
        ctx.bind_lin(t_late.data_ptr()); r["host random tail, torch tensor made after the context"] = timed()
        ctx.bind_lin(t_rand.data_ptr()); r["host random tail, bound"] = timed()
        ctx.bind_lin(0); ctx.upload_lin(lin); r["host random tail, uploaded"] = timed()
        ctx.bind_lin(t_zero.data_ptr()); r["host zero tail, bound"] = timed()
        ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr()); r["device-produced (zero tail)"] = timed()
        print("  ".join(f"{k}: {v:.4f}" for k, v in r.items()), flush=True)
    ctx2.close()
