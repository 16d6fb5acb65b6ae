"""Could the iterate skip Jacobi iterations once a scenario's pair of
sub-controllers has reached a bitwise fixed point (the next iteration's inputs
equal this one's, so every later iteration repeats it exactly)?  The oracle's
step from the same settled states with K = 1 .. 15: per K, the fraction of
QPs, of scenario pairs and of 32-scenario waves (64 QPs) whose plans equal
those after K - 1 iterations bit for bit.  CPU only (oracle/liboracle.so).
usage: python tools/jacobi_fixed_point.py [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _oracle as O  # noqa: E402
import cmpc  # noqa: E402
from cmpc._abi import CmpcDims  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
dims = CmpcDims.from_config(cfg, B)
lin, u, du, ws = synthetic_batch(cfg, B, seed=1002, n_distinct=256)
O.step(dims, arr, lin, 9, u, du, ws, init=True, threads=8)
for _ in range(6):  # settle with the move applied, as the bench does
    O.step(dims, arr, lin, 9, u, du, ws, flags=cmpc.CMPC_APPLY_MOVE, threads=8)
plans = {}
for K in range(1, 16):
    x, _, _, _, _ = O.step(dims, arr, lin, K, u.copy(), du.copy(), ws.copy(), threads=8)
    plans[K] = x
for K in range(2, 16):
    same = (plans[K] == plans[K - 1]).all(axis=1)
    pair = same.reshape(B, cfg.S).all(axis=1)
    wave = pair.reshape(-1, 32).all(axis=1)
    print(f"K {K:2d}: QPs fixed {same.mean():.3f}, pairs {pair.mean():.3f}, waves {wave.mean():.3f}")
