"""Build-kernel time by variant (CMPC_BUILD_ROWS / SPLIT / WAVE) for one
configuration over batch sizes, by the build's events after a clock settle;
AUTO's pick is printed beside.  GPU only.
usage: python tools/build_variant_sweep.py plant ctype p B1 [B2 ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

plant, ctype, p = sys.argv[1], sys.argv[2], int(sys.argv[3])
cfg = cmpc.reference_config(plant, ctype, p=p)
arr = cmpc.controller_arrays(cfg, reference_setup(plant, ctype))
names = {cmpc.CMPC_BUILD_ROWS: "rows", cmpc.CMPC_BUILD_SPLIT: "split", cmpc.CMPC_BUILD_WAVE: "wave",
         cmpc.CMPC_BUILD_AUTO: "auto"}
for B in [int(a) for a in sys.argv[4:]]:
    lin, u, du, ws = synthetic_batch(cfg, B, seed=5, n_distinct=min(B, 256))
    with cmpc.Context(cfg, B) as ctx:
        ctx.configure(arr)
        ctx.set_state(u, du, ws)
        ctx.upload_lin(lin)
        line = []
        for v in (cmpc.CMPC_BUILD_AUTO, cmpc.CMPC_BUILD_ROWS, cmpc.CMPC_BUILD_SPLIT, cmpc.CMPC_BUILD_WAVE):
            try:
                ctx.set_build_variant(v)
                t = time.perf_counter()
                while time.perf_counter() - t < 0.2:
                    for _ in range(16):
                        ctx.build()
                    ctx.synchronize()
                ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_BUILD,))
                for _ in range(50):
                    ctx.build()
                ctx.synchronize()
                ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
                ctx.enable_timing(False)
                used = names.get(ctx.last_build_kernel(), "?")
                line.append(f"{names[v]}({used}) {ms / n * 1e3:7.2f}")
            except Exception as e:  # a variant not available at these dimensions
                line.append(f"{names[v]} n/a ({str(e)[:40]})")
        print(f"{plant}-{ctype} p={p} B={B} QPs={B * cfg.S}: " + "  ".join(line), flush=True)
