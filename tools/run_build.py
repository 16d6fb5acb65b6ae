"""Launch cmpc_build a few times at one horizon (for rocprofv3 PMC passes).
CMPC_BUILD_VARIANT=wave|rows|auto selects the build kernel (default auto)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import cmpc
from cmpc.configs import reference_setup
from cmpc.synthetic import synthetic_batch
p = int(sys.argv[1]) if len(sys.argv) > 1 else 50
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
cfg = cmpc.reference_config("par", "coop", p=p)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
lin, u, du, ws = synthetic_batch(cfg, B, seed=7, n_distinct=256)
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr); ctx.set_state(u, du, ws); ctx.upload_lin(lin)
    ctx.set_build_variant({"auto": cmpc.CMPC_BUILD_AUTO, "wave": cmpc.CMPC_BUILD_WAVE,
                           "rows": cmpc.CMPC_BUILD_ROWS}[os.environ.get("CMPC_BUILD_VARIANT", "auto")])
    for _ in range(4): ctx.build()
    ctx.synchronize()
print("ok")
