"""A short, repeatable launch sequence of one small-batch kernel for rocprofv3
--pmc passes: CONFIG (tools/time_small.py names), WHAT = iterate-lane |
iterate-rows | build | step, N launches after a warm-up.
usage: python tools/pmc_small.py CONFIG WHAT [N [K]]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402
from time_small import CONFIGS  # noqa: E402

name, what = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
plant, ctype, p, B, K = CONFIGS[name]
if len(sys.argv) > 4:
    K = int(sys.argv[4])
cfg = cmpc.reference_config(plant, ctype, p=p)
arr = cmpc.controller_arrays(cfg, reference_setup(plant, ctype))
lin, u, du, ws = synthetic_batch(cfg, B, seed=11, n_distinct=min(B, 2048))
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr)
    ctx.set_state(u, du, ws)
    ctx.upload_lin(lin)
    ctx.build()
    ctx.init_warmstart()
    if what == "iterate-rows":
        ctx.set_solve_variant(cmpc.CMPC_SOLVE_ROWS)
    elif what == "iterate-lane":
        ctx.set_solve_variant(cmpc.CMPC_SOLVE_LANE)
    for i in range(n + 5):
        if what.startswith("iterate"):
            ctx.iterate(K)
        elif what == "build":
            ctx.build()
        else:
            ctx.step(K)
    ctx.synchronize()
print("done", name, what, n)
