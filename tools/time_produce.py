"""Time the device record producer (cmpc_produce_lin, scenario mode) alone at
the bench size, by the library's event timing; for PRODUCE_EXP ablation
builds (CMPC_LIBRARY=ab/<name>/libcmpc.so; results invalid, timing only).
GPU only.  usage: python tools/time_produce.py [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_operating_points  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
xs, us, ys = synthetic_operating_points(cfg, B, seed=77, n_distinct=min(B, 2048))
tx, tu, ty = (torch.from_numpy(a).to("cuda:0") for a in (xs, us, ys))
with cmpc.Context(cfg, B, device=0) as ctx:
    ctx.configure(arr)
    for _ in range(20):
        ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
    ctx.synchronize()
    ctx.enable_timing(True)
    for _ in range(50):
        ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
    ctx.synchronize()
    t, n = ctx.kernel_time(cmpc.CMPC_KERNEL_PRODUCE)
    ctx.enable_timing(False)
    print(f"produce B={B}: {t / max(n, 1) * 1e3:.2f} us per launch ({n} launches)"
          f" = {B * cfg.S * 312 * 8 / (t / max(n, 1)) / 1e9:.2f} TB/s of records written")
