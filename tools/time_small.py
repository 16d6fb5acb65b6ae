"""Small-batch timing (BASELINE configs 2 and 5, B = 1): build kernel per
variant, iterate at K = 0 / 1 / K, and the step's wall time (back-to-back
steps, and one synchronised step at a time).  Library: CMPC_LIBRARY.
usage: python tools/time_small.py [config ...]   (config names below)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

CONFIGS = {  # name: (plant, controller, p, B scenarios, K)
    "c5": ("par", "cent", 200, 1024, 1),
    "c2": ("par", "coop", 20, 4096, 9),
    "c2q256": ("par", "coop", 20, 128, 9),
    "c2q1k": ("par", "coop", 20, 512, 9),
    "b1": ("par", "coop", 50, 1, 9),
    "c1b1": ("ser", "cent", 100, 1, 1),
    "c3": ("par", "ncoop", 50, 65536, 1),
    "c1": ("ser", "cent", 100, 65536, 1),
    "head": ("par", "coop", 50, 65536, 9),
}
REPS = int(os.environ.get("CMPC_TS_REPS", "50"))
VARS = [("wave", cmpc.CMPC_BUILD_WAVE), ("split", getattr(cmpc, "CMPC_BUILD_SPLIT", -1)),
        ("rows", cmpc.CMPC_BUILD_ROWS), ("auto", cmpc.CMPC_BUILD_AUTO)]


def settle(ctx, K, sec=0.3):
    t_end = time.perf_counter() + sec
    while time.perf_counter() < t_end:
        for _ in range(8):
            ctx.build()
            ctx.iterate(K)
        ctx.synchronize()


def main():
  for name in (sys.argv[1:] or ["c5", "c2", "b1"]):
      plant, ctype, p, B, K = CONFIGS[name]
      cfg = cmpc.reference_config(plant, ctype, p=p)
      arr = cmpc.controller_arrays(cfg, reference_setup(plant, ctype))
      lin, u, du, ws = synthetic_batch(cfg, B, seed=11, n_distinct=min(B, 2048))
      with cmpc.Context(cfg, B) as ctx:
          ctx.configure(arr)
          ctx.set_state(u, du, ws)
          ctx.upload_lin(lin)
          ctx.build()
          ctx.init_warmstart()
          settle(ctx, K)
          res = []
          for vn, v in VARS:
              try:
                  ctx.set_build_variant(v)
                  ctx.build()
              except Exception as e:  # noqa: BLE001
                  res.append(f"{vn} n/a")
                  continue
              ctx.synchronize()
              ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_BUILD,))
              for _ in range(REPS):
                  ctx.build()
              ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
              ctx.enable_timing(False)
              res.append(f"{vn} {ms / n * 1e3:7.2f}")
          ctx.set_build_variant(cmpc.CMPC_BUILD_AUTO)
          its = []
          for sv, sn in ((getattr(cmpc, "CMPC_SOLVE_LANE", None), "lane"), (getattr(cmpc, "CMPC_SOLVE_ROWS", None), "rows")):
              if sv is None:
                  continue
              ctx.set_solve_variant(sv)
              for k in (0, 1, K):
                  ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_ITERATE,))
                  for _ in range(REPS):
                      ctx.iterate(k)
                  ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
                  ctx.enable_timing(False)
                  its.append(f"{sn} K={k} {ms / n * 1e3:6.2f}")
          if hasattr(cmpc, "CMPC_SOLVE_AUTO"):
              ctx.set_solve_variant(cmpc.CMPC_SOLVE_AUTO)
          steps = []
          variants = [("split", getattr(cmpc, "CMPC_STEP_SPLIT", None)), ("fused", getattr(cmpc, "CMPC_STEP_FUSED", None)),
                      ("auto", getattr(cmpc, "CMPC_STEP_AUTO", None))]
          for vn, v in variants:
              if v is None and vn != "auto":
                  continue
              try:
                  if v is not None:
                      ctx.set_step_variant(v)
                  ctx.step(K)
                  ctx.synchronize()
              except Exception:  # noqa: BLE001
                  steps.append(f"{vn} n/a")
                  continue
              settle(ctx, K, 0.1)
              t0 = time.perf_counter()
              for _ in range(REPS):
                  ctx.step(K)
              ctx.synchronize()
              t_bb = (time.perf_counter() - t0) / REPS
              t0 = time.perf_counter()
              for _ in range(REPS):
                  ctx.step(K)
                  ctx.synchronize()
              t_sync = (time.perf_counter() - t0) / REPS
              kern = ""
              if vn == "fused":
                  ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_STEP,))
                  for _ in range(REPS):
                      ctx.step(K)
                  ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_STEP)
                  ctx.enable_timing(False)
                  kern = f" kernel {ms / n * 1e3:.2f}"
              steps.append(f"{vn} {t_bb * 1e6:.1f}/{t_sync * 1e6:.1f}{kern}")
      print(f"{name:5s} {plant}-{ctype} p={p} B={B} K={K}  build us: {', '.join(res)} | iterate us: "
            f"{', '.join(its)} | step us back-to-back/synchronised: {'; '.join(steps)}", flush=True)


if __name__ == "__main__":
    main()
