"""Host-side problem assembly (numpy), mirroring the reference's per-controller
configuration plumbing:

  NerveCenter::SetWeightsSubHelper  include/nerve_center.h:222-231
      uwt_sub = uwt[own, own] (ControlInputIndexType::GetSubMatrix,
      include/constexpr_array.h:114-139); ywt_sub = the sub-controller's block
  NerveCenter::SetOutputReferenceHelper include/nerve_center.h:234-249
      y_ref_sub[i] = y_ref[i][ControlledOutputIndices] for i < p
  InputConstraints<nu> per sub-controller (include/input_constraints.h:12-26)
"""
from dataclasses import dataclass

import numpy as np

from .configs import ControllerConfig, SetupFile


@dataclass
class ControllerArrays:
    y_ref: np.ndarray       # S x (p*ny)
    ywt: np.ndarray         # S x ny x ny
    uwt: np.ndarray         # S x nu x nu
    lower: np.ndarray       # S x nu
    upper: np.ndarray
    rate_lower: np.ndarray
    rate_upper: np.ndarray


def controller_arrays(cfg: ControllerConfig, setup: SetupFile, n_outputs: int = 4) -> ControllerArrays:
    S, ny, nu, p = cfg.S, cfg.ny, cfg.nu, cfg.p
    yref = np.asarray(setup.yref, dtype=np.float64)
    if yref.size == n_outputs:
        yref_full = np.tile(yref, (p, 1))            # reference replicated over p
    else:
        yref_full = yref.reshape(-1, n_outputs)[:p]
    y_ref = np.stack([yref_full[:, cfg.out_idx[s]].reshape(p * ny) for s in range(S)])
    ywt = np.stack([np.asarray(setup.ywt[s], dtype=np.float64).reshape(ny, ny) for s in range(S)])
    uwt_full = np.asarray(setup.uwt, dtype=np.float64).reshape(cfg.nu_tot, cfg.nu_tot)
    uwt = np.stack([uwt_full[np.ix_(cfg.own_inputs(s), cfg.own_inputs(s))] for s in range(S)])

    def per_sub(v):
        v = np.asarray(v, dtype=np.float64)
        if v.size == nu:
            return np.tile(v, (S, 1))
        if v.size == cfg.nu_tot:
            return np.stack([v[cfg.own_inputs(s)] for s in range(S)])
        raise ValueError(f"constraint vector of {v.size} entries for nu={nu}")

    return ControllerArrays(
        y_ref=np.ascontiguousarray(y_ref), ywt=np.ascontiguousarray(ywt),
        uwt=np.ascontiguousarray(uwt),
        lower=per_sub(setup.constraints_lower), upper=per_sub(setup.constraints_upper),
        rate_lower=per_sub(setup.rate_lower), rate_upper=per_sub(setup.rate_upper))


def plant_input_from_plans(cfg: ControllerConfig, du: np.ndarray) -> np.ndarray:
    """First move of every sub-controller scattered to plant control-input
    order (NerveCenter::UpdateUOld, include/nerve_center.h:313-319).
    du: (..., S, nV) -> (..., nu_tot)."""
    out = np.zeros(du.shape[:-2] + (cfg.nu_tot,))
    for s in range(cfg.S):
        out[..., cfg.own_inputs(s)] = du[..., s, : cfg.nu]
    return out
