"""Per-phase cycle attribution of the row build kernel, or with KERNEL=wave of
the one-QP-per-wave kernel (diagnostic library built with -DCMPC_ROWS_TIMING=1
-DCMPC_WAVE_TIMING=1: tools/build_variant.sh timing "...").  For the wave
kernel slot 1 is the fused solve (0 here) and a "group" is one QP.
usage: CMPC_LIBRARY=ab/timing/libcmpc.so python tools/rows_timing.py [p] [B] [plant-ctype] [rows|wave]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np
import cmpc
from cmpc.configs import reference_setup
from cmpc.synthetic import synthetic_batch
p = int(sys.argv[1]) if len(sys.argv) > 1 else 50
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
PLANT, CTYPE = (sys.argv[3] if len(sys.argv) > 3 else "par-coop").split("-")
KERNEL = sys.argv[4] if len(sys.argv) > 4 else "rows"
cfg = cmpc.reference_config(PLANT, CTYPE, p=p)
arr = cmpc.controller_arrays(cfg, reference_setup(PLANT, CTYPE))
lin, u, du, ws = synthetic_batch(cfg, B, seed=7, n_distinct=min(B, 256))
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr); ctx.set_state(u, du, ws); ctx.upload_lin(lin)
    ctx.set_build_variant(cmpc.CMPC_BUILD_ROWS if KERNEL == "rows" else cmpc.CMPC_BUILD_WAVE)
    import time
    t_end = time.perf_counter() + 0.3  # settle at the steady clock
    while time.perf_counter() < t_end:
        for _ in range(16):
            ctx.build()
        ctx.synchronize()
    ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_BUILD,))
    ctx.build()
    ctx.synchronize()
    kms, _ = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
    print(f"build kernel (events): {kms * 1e3:.2f} us")
    H, f, G = ctx.download_qp()
raw = np.concatenate([H.reshape(H.shape[0], -1), f, G.reshape(G.shape[0], -1)], axis=1).reshape(-1)
d = raw[: (raw.size // 16) * 16].reshape(-1, 16)
d = d[d[:, 7] == 1.0]
ng = d[:, 6].sum()
names = ["tail/back-edge", "staging issue", "staging wait", "prologue compute", "horizon loop", "epilogue"]
order = [5, 0, 1, 2, 3, 4]
tot = d[:, :6].sum()
print(f"{KERNEL} kernel, {PLANT}-{CTYPE} p={p}: {len(d)} waves, {ng:.0f} groups; s_memtime cycles per group:")
for i in order:
    print(f"  {names[order.index(i)] if False else ['staging issue','staging wait','prologue compute','horizon loop','epilogue','tail/back-edge'][i]:18s} {d[:, i].sum() / ng:10.0f}  ({d[:, i].sum() / tot * 100:5.1f} %)")
clk = d[:, 8] / (d[:, 9] / 100e6) / 1e9
print(f"  in-kernel shader clock: median {np.median(clk):.3f} GHz (min {clk.min():.3f}, max {clk.max():.3f})")
st, en = d[:, 10], d[:, 11]
span = (en.max() - st.min()) / 100e6 * 1e3
print(f"  kernel span (first wave start -> last wave end): {span:.4f} ms; wave lifetime ms: "
      f"min {d[:, 9].min() / 1e5:.4f} median {np.median(d[:, 9]) / 1e5:.4f} max {d[:, 9].max() / 1e5:.4f}; "
      f"start skew max {(st.max() - st.min()) / 1e5:.4f} ms")

# placement (HW_ID, XCC_ID): per-SIMD group counts against wave end times
hw = d[:, 12].astype(np.int64)
xcc = d[:, 13].astype(np.int64) & 0xF
simd = (hw >> 4) & 3
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
simd_key = key * 4 + simd
t0 = st.min()
end_us = (en - t0) / 100.0
print(f"  XCDs {len(np.unique(xcc))}, CUs {len(np.unique(key))}, SIMDs {len(np.unique(simd_key))}")
grp = {}
for k_, n_, e_ in zip(simd_key, d[:, 6], end_us):
    g_ = grp.setdefault(k_, [0, 0, 0.0])
    g_[0] += n_; g_[1] += 1; g_[2] = max(g_[2], e_)
tot_g = np.array([v[0] for v in grp.values()]); nw = np.array([v[1] for v in grp.values()])
last = np.array([v[2] for v in grp.values()])
for n_ in np.unique(tot_g):
    m_ = tot_g == n_
    print(f"  SIMDs with {n_:.0f} groups: {m_.sum():4d} (waves/SIMD {np.unique(nw[m_])}); last wave end "
          f"us: median {np.median(last[m_]):.1f} max {last[m_].max():.1f}")
for x_ in np.unique(xcc):
    m_ = xcc == x_
    print(f"  XCC {x_}: waves {m_.sum()}, clock median {np.median(clk[m_]):.3f} GHz, wave end us median "
          f"{np.median(end_us[m_]):.1f} max {end_us[m_].max():.1f}")
for n_ in np.unique(d[:, 6]):
    m_ = d[:, 6] == n_
    print(f"  waves with {n_:.0f} groups: {m_.sum()}, end us median {np.median(end_us[m_]):.1f} "
          f"max {end_us[m_].max():.1f}")
