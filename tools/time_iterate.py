"""Time cmpc_iterate (K Jacobi iterations of warm-started solves) alone."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import cmpc
from cmpc.configs import reference_setup
from cmpc.synthetic import synthetic_batch
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
K = int(sys.argv[2]) if len(sys.argv) > 2 else 9
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
lin, u, du, ws = synthetic_batch(cfg, B, seed=7, n_distinct=2048)
if os.environ.get("CMPC_TI_UNCONSTRAINED"):  # diagnostic: bounds far away, no active set
    import numpy as np
    for s_ in range(cfg.S):
        arr.lower[s_][:] = -1e6; arr.upper[s_][:] = 1e6
        arr.rate_lower[s_][:] = -1e6; arr.rate_upper[s_][:] = 1e6
    ws = np.zeros_like(ws)
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr); ctx.set_state(u, du, ws); ctx.upload_lin(lin)
    ctx.build(); ctx.init_warmstart()
    import time
    t_end = time.perf_counter() + float(os.environ.get("CMPC_TB_SETTLE", "0.3"))  # clock settle
    while time.perf_counter() < t_end:
        for _ in range(8): ctx.iterate(K)
        ctx.synchronize()
    ctx.enable_timing(True)
    for _ in range(40): ctx.iterate(K)
    ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
    _, _, ws_now = ctx.get_state()
    scen = (ws_now.reshape(B, cfg.S) != 0).any(axis=1).mean()
    print(f"iterate K={K}: {ms/n:.4f} ms  active fraction {(ws_now != 0).mean():.3f} "
          f"(scenarios {scen:.3f})", flush=True)
