"""Time the device record producer (cmpc_produce_lin) alone."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np
import torch
import cmpc
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
cfg = cmpc.reference_config("par", "coop", p=50)
rng = np.random.default_rng(3)
x0, u0 = cmpc.plant_default(cfg.plant)
xs = x0[None, :] * (1 + 0.01 * rng.normal(size=(B, len(x0))))
us = np.tile(u0, (B, 1)); us[:, [0, 3, 4, 7]] += rng.uniform(-0.02, 0.02, (B, 4))
ys = np.tile(cmpc.plant_output(cfg.plant, x0), (B, 1))
tx, tu, ty = (torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (xs, us, ys))
with cmpc.Context(cfg, B) as ctx:
    for _ in range(3): ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(20): ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
    ctx.synchronize()
    print(f"produce B={B}: {(time.perf_counter() - t0) / 20 * 1e3:.4f} ms", flush=True)
