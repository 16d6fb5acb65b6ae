"""Seeded synthetic batches of the reference workload.

Per scenario b (seed = 1000 + config_id unless given):
  x_b = x_def * (1 + 0.01 N(0,1))          x_def: include/parallel_compressors.h:74-78
  u_b = u_def + U(-0.02, 0.02) on the control entries  (:81-86)
  linearise + discretise at (x_b, u_b), Ts = 0.05, on the host (untimed);
  an operating point whose discrete A has spectral radius > 1 is redrawn
  (about 9% of parallel-plant draws: a 1% pressure perturbation can bring a
  compressor's discharge pressure to the tank pressure, where the valve
  derivative ~ 1/sqrt|dp| explodes; the nominal radius is 0.995)
Per QP slot (scenario b, sub-controller s):
  dx_aug tail ~ N(0, 1e-3)
  u_old: torque inputs ~ U(-0.098, 0.074), recycle inputs 0 (closed, at its
         lower bound) with probability 0.1, else U(0, 0.066) — calibrated to
         the reference's closed-loop records (results/parallel/run1/coop9.dat:
         torque in [-0.0977, 0.0739], recycle in [0, 0.0656], recycle == 0 in
         10.0% of the 10 000 steps); the survey recipe (U(-0.05,0.05), U(0,0.05))
         leaves only ~5% of QPs with an active constraint
  y_prev = plant output at x_b (controlled entries)
  du_old = 0, ws = 0
"""
import numpy as np

from ._abi import CmpcDims
from .configs import REF_TS, ControllerConfig
from . import plant_default, plant_lin_record, plant_output, layout_of

CONTROL_ENTRIES = (0, 3, 4, 7)   # ControlInputIndex <0,3,4,7> of both plants


def _stable_point(cfg, dims, L, rng, x_def, u_def, out):
    """One operating point whose discrete A has spectral radius <= 1; fills
    out[s] with the S host-produced records and returns (x, u_full)."""
    ns = cfg.ns
    while True:
        x = x_def * (1.0 + 0.01 * rng.standard_normal(x_def.shape))
        u = u_def.copy()
        u[list(CONTROL_ENTRIES)] += rng.uniform(-0.02, 0.02, len(CONTROL_ENTRIES))
        for s in range(cfg.S):
            plant_lin_record(cfg, dims, s, x, u, Ts=REF_TS, out=out[s])
        A = out[0, L.off_A:L.off_A + ns * ns].reshape(ns, ns)
        if np.all(np.isfinite(out)) and np.abs(np.linalg.eigvals(A)).max() <= 1.0:
            return x, u


def synthetic_operating_points(cfg: ControllerConfig, B: int, seed: int = 1002,
                               n_distinct: int = None):
    """Plant states of B scenarios (for the device producer, cmpc_produce_lin):
    (x [B, ns], u_full [B, n_inputs], y [B, n_outputs]), drawn and filtered as
    in synthetic_batch, n_distinct distinct points tiled over the batch."""
    rng = np.random.default_rng(seed)
    dims = CmpcDims.from_config(cfg, 1)
    L = layout_of(dims)
    nd = n_distinct or B
    x_def, u_def = plant_default(cfg.plant)
    xs, us, ys = [], [], []
    scratch = np.zeros((cfg.S, L.rec_len))
    for _ in range(nd):
        x, u = _stable_point(cfg, dims, L, rng, x_def, u_def, scratch)
        xs.append(x); us.append(u); ys.append(plant_output(cfg.plant, x))
    idx = np.arange(B) % nd
    return (np.ascontiguousarray(np.stack(xs)[idx]), np.ascontiguousarray(np.stack(us)[idx]),
            np.ascontiguousarray(np.stack(ys)[idx]))


def synthetic_u_old(cfg: ControllerConfig, B: int, rng) -> np.ndarray:
    """u_old per QP slot, calibrated to the reference's closed-loop records."""
    S = cfg.S
    u_old = np.zeros((B, S, cfg.nu_tot))
    for s in range(S):
        for c, plant_c in enumerate(cfg.input_order[s]):
            torque = plant_c in (0, 2)     # control inputs: torque1, rec1, torque2, rec2
            if torque:
                u_old[:, s, c] = rng.uniform(-0.098, 0.074, B)
            else:
                u_old[:, s, c] = np.where(rng.random(B) < 0.1, 0.0, rng.uniform(0.0, 0.066, B))
    return np.ascontiguousarray(u_old.reshape(B * S, cfg.nu_tot))


def synthetic_batch(cfg: ControllerConfig, B: int, seed: int = 1002, n_distinct: int = None):
    """Returns (lin [B*S, rec_len], u_old [B*S, nu_tot], du_old, ws).

    n_distinct: number of distinct linearisations to compute (the rest of the
    batch cycles through them with fresh dx_aug / u_old draws) — the host-side
    producer is not what is measured, this only bounds set-up time."""
    rng = np.random.default_rng(seed)
    dims = CmpcDims.from_config(cfg, B)
    L = layout_of(dims)
    S = cfg.S
    nq = B * S
    nd = n_distinct or B
    x_def, u_def = plant_default(cfg.plant)
    base = np.zeros((nd, S, L.rec_len))
    ys = np.zeros((nd, 4))
    for i in range(nd):
        x, _ = _stable_point(cfg, dims, L, rng, x_def, u_def, base[i])
        ys[i] = plant_output(cfg.plant, x)
    lin = np.ascontiguousarray(np.tile(base, ((B + nd - 1) // nd, 1, 1))[:B])
    idx = np.arange(B) % nd
    for s in range(S):
        lin[:, s, L.off_x:L.off_x + L.naug] = 1e-3 * rng.standard_normal((B, L.naug))
        lin[:, s, L.off_y:L.off_y + cfg.ny] = ys[idx][:, cfg.out_idx[s]]
    lin = lin.reshape(nq, L.rec_len)
    u_old = synthetic_u_old(cfg, B, rng)
    du_old = np.zeros((nq, cfg.nV))
    ws = np.zeros(nq, np.uint32)
    return np.ascontiguousarray(lin), u_old, du_old, ws
