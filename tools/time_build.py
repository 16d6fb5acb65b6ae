"""Time cmpc_build alone at several horizons (per-step vs fixed per-QP cost).
CMPC_TB_CASE=plant-ctype selects the configuration (default par-coop);
CMPC_TB_VARIANT=wave|rows|both selects the build kernel (default both)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np
import cmpc
from cmpc.configs import reference_setup
from cmpc.synthetic import synthetic_batch
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
PS = [int(a) for a in sys.argv[2:]] or [2, 10, 25, 50, 100]
PLANT, CTYPE = os.environ.get("CMPC_TB_CASE", "par-coop").split("-")
VAR = {"wave": [cmpc.CMPC_BUILD_WAVE], "rows": [cmpc.CMPC_BUILD_ROWS],
       "both": [cmpc.CMPC_BUILD_WAVE, cmpc.CMPC_BUILD_ROWS]}[os.environ.get("CMPC_TB_VARIANT", "both")]
for p in PS:
    cfg = cmpc.reference_config(PLANT, CTYPE, p=p)
    arr = cmpc.controller_arrays(cfg, reference_setup(PLANT, CTYPE))
    lin, u, du, ws = synthetic_batch(cfg, B, seed=7, n_distinct=256)
    if os.environ.get("CMPC_TB_ZERO"):  # diagnostic: zero-filled records (power/clock test)
        lin = np.zeros_like(lin); u = np.zeros_like(u)
    for v in VAR:
        with cmpc.Context(cfg, B) as ctx:
            ctx.configure(arr); ctx.set_state(u, du, ws); ctx.upload_lin(lin)
            ctx.set_build_variant(v)
            # settle: the clock ramps over the first ~40 ms of load (tools/time_clock_ramp.py)
            t_end = time.perf_counter() + float(os.environ.get("CMPC_TB_SETTLE", "0.3"))
            while time.perf_counter() < t_end:
                for _ in range(8): ctx.build()
                ctx.synchronize()
            ctx.enable_timing(True)
            for _ in range(int(os.environ.get("CMPC_TB_N", "40"))): ctx.build()
            ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
            name = "wave" if v == cmpc.CMPC_BUILD_WAVE else "rows"
            print(f"p={p:4d}  {name} build {ms/n:.4f} ms  per QP-step {ms/n*1e6/(B*cfg.S*p):.3f} ns"
                  f"  ({PLANT}-{CTYPE})", flush=True)
