"""Build-kernel time vs the number of distinct resident input batches the
steps rotate through (1: the same 327 MB of records every step; 4: the bench).
Separates a cache effect (MALL 256 MB) from the kernel's own cost.
usage: python tools/time_rotation.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import torch  # noqa: E402
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

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
    for nb in (1, 4, 2, 1, 4):
        for i in range(5):
            ctx.bind_lin(batches[i % nb].data_ptr())
            ctx.step(K, 0)
        ctx.synchronize()
        ctx.enable_timing(True)
        for i in range(40):
            ctx.bind_lin(batches[i % nb].data_ptr())
            ctx.build()
        ctx.synchronize()
        ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
        ctx.enable_timing(False)
        print(f"{nb} distinct batches: build {ms / n:.4f} ms", flush=True)
