"""Per-step time and QP solves/s of SURVEY.md §8(d)'s single-GPU configurations
(build + K Jacobi iterations, warm-started, inputs resident in HBM), on one GPU.
Config 4 (64 sub-controllers over 8 GPUs) is tools/bench_coupled.py.
usage: python tools/time_survey_configs.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

CONFIGS = [  # (name, plant, controller, p, B scenarios, K)
    ("1 cent-ser p=100 (reference's own)", "ser", "cent", 100, 65536, 1),
    ("2 coop-par p=20", "par", "coop", 20, 4096, 9),
    ("2' coop-par p=20, 65536 scenarios", "par", "coop", 20, 65536, 9),
    ("3 ncoop-par p=50, K=1", "par", "ncoop", 50, 65536, 1),
    ("headline coop-par p=50", "par", "coop", 50, 65536, 9),
    ("5 cent-par p=200", "par", "cent", 200, 1024, 1),
    ("5' cent-par p=200, 65536 scenarios", "par", "cent", 200, 65536, 1),
]
REPS = 20
for name, plant, ctype, p, B, K in CONFIGS:
    cfg = cmpc.reference_config(plant, ctype, p=p)
    arr = cmpc.controller_arrays(cfg, reference_setup(plant, ctype))
    lin, u, du, ws = synthetic_batch(cfg, B, seed=11, n_distinct=min(B, 2048))
    with cmpc.Context(cfg, B) as ctx:
        ctx.configure(arr)
        ctx.set_state(u, du, ws)
        ctx.upload_lin(lin)
        ctx.build()
        ctx.init_warmstart()
        # settle: the clock ramps over the first ~40 ms of load (tools/time_clock_ramp.py)
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            for _ in range(4):
                ctx.build()
                ctx.iterate(K)
            ctx.synchronize()
        ctx.enable_timing(True)
        for _ in range(REPS):
            ctx.build()
            ctx.iterate(K)
        ctx.synchronize()
        bms, nb = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
        ims, ni = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
        kern = "rows" if ctx.last_build_kernel() == cmpc.CMPC_BUILD_ROWS else "wave"
    step = bms / nb + ims / ni
    solves = B * cfg.S * K / (step / 1e3)
    print(f"{name:38s} QPs {B * cfg.S:7d}  build {bms / nb:.4f} ms ({kern})  iterate(K={K}) "
          f"{ims / ni:.4f} ms  -> {solves:.3e} QP solves/s", flush=True)
