"""Optimality of the solver specification, independent of its algorithm.

The GPU solve kernel equals the oracle solver (oracle/or_qp.c) bit for bit
(test_gpu_parity.py, test_solver_host.py), so pinning the oracle's answers to
the QP optimum pins the product.  The reference solves with qpOASES 3.2.0
(libs/mpc_qp_solver.cc:62-72), absent here; for SPD H the optimum of

    min 1/2 x'Hx + g'x   s.t.  lb <= x <= ub,  lbA <= A x <= ubA,
    A = [I_nu 0 ...; -I_nu I_nu ...]            (include/mpc_qp_solver.h:108-123)

is unique, so any correct solver returns the same x up to rounding.  Two
checks on every QP the oracle reports as solved (status OK):
  * KKT certificate from the reported working set: primal feasibility,
    stationarity H x + g = sum_j mu_j s_j a_j with mu >= 0, and the active
    rows tight;
  * for nV = 4, brute-force enumeration of every active set (up to four of
    the eight rows, either side): the unique KKT point equals the oracle's x,
    and a QP the oracle calls infeasible has no KKT point.
Inputs: random MPC-shaped QPs (cold and warm started) and the real condensed
QPs of the coop / cent parallel-plant controllers on synthetic operating
points.
Tolerances: relative 1e-9 of the problem scale (the oracle's own decision
tolerances are 1e-12 relative)."""
import itertools

import numpy as np
import pytest

import _oracle as O
import cmpc
import golden_cases as GC
from cmpc._abi import CmpcDims
from cmpc.synthetic import synthetic_batch
from test_solver_host import random_qp

OK = 0


def rows(n, nu):
    """The 2n constraint rows: bounds (j < n), then the rate rows."""
    A = np.eye(n)
    for i in range(nu, n):
        A[i, i - nu] = -1.0
    return np.vstack([np.eye(n), A])


def kkt_certificate(H, g, lo, hi, C, x, ws):
    n = len(g)
    scale = np.abs(H).max() * max(1.0, np.abs(x).max()) + np.abs(g).max() + 1.0
    cx = C @ x
    bscale = 1.0 + np.maximum(np.abs(lo), np.abs(hi))
    assert np.all(cx >= lo - 1e-9 * bscale), "lower row violated"
    assert np.all(cx <= hi + 1e-9 * bscale), "upper row violated"
    act = [j for j in range(2 * n) if (ws >> j) & 1]
    side = [(ws >> (16 + j)) & 1 for j in act]
    for j, s in zip(act, side):
        target = hi[j] if s else lo[j]
        assert abs(cx[j] - target) <= 1e-9 * bscale[j], ("active row not tight", j, s)
    grad = H @ x + g
    if act:
        N = np.stack([C[j] * (-1.0 if s else 1.0) for j, s in zip(act, side)], axis=1)
        mu, *_ = np.linalg.lstsq(N, grad, rcond=None)
        resid = grad - N @ mu
        assert np.all(mu >= -1e-9 * scale), ("negative multiplier", mu)
    else:
        resid = grad
    assert np.abs(resid).max() <= 1e-9 * scale, ("stationarity", np.abs(resid).max(), scale)


def kkt_certificate_batch(H, g, lo, hi, C, x, ws, tol=1e-9):
    """kkt_certificate over a batch (Q QPs, rows C shared): boolean per QP.
    Multipliers by batched pseudo-inverse of the signed active rows."""
    Q, n = g.shape
    bits = np.arange(C.shape[0], dtype=np.uint32)
    ws = ws.astype(np.uint32)
    act = ((ws[:, None] >> bits) & 1).astype(bool)
    side = ((ws[:, None] >> (bits + 16)) & 1).astype(bool)
    cx = x @ C.T
    bscale = 1.0 + np.maximum(np.abs(lo), np.abs(hi))
    ok = np.all((cx >= lo - tol * bscale) & (cx <= hi + tol * bscale), axis=1)
    target = np.where(side, hi, lo)
    ok &= np.all(~act | (np.abs(cx - target) <= tol * bscale), axis=1)
    grad = np.einsum("qij,qj->qi", H, x) + g
    N = C.T[None, :, :] * (np.where(side, -1.0, 1.0) * act)[:, None, :]
    mu = np.einsum("qri,qi->qr", np.linalg.pinv(N), grad)
    resid = grad - np.einsum("qir,qr->qi", N, mu)
    scale = np.abs(H).max(axis=(1, 2)) * np.maximum(1.0, np.abs(x).max(axis=1)) + np.abs(g).max(axis=1) + 1.0
    ok &= np.all(~act | (mu >= -tol * scale[:, None]), axis=1)
    ok &= np.abs(resid).max(axis=1) <= tol * scale
    return ok


def enumerate_optimum(H, g, lo, hi, C):
    """The unique KKT point by enumeration (n <= 4)."""
    n = len(g)
    scale = np.abs(H).max() + np.abs(g).max() + 1.0
    bscale = 1.0 + np.maximum(np.abs(lo), np.abs(hi))
    found = []
    for k in range(n + 1):
        for act in itertools.combinations(range(2 * n), k):
            for sides in itertools.product((0, 1), repeat=k):
                N = np.array([C[j] * (-1.0 if s else 1.0) for j, s in zip(act, sides)]).reshape(k, n)
                if k and np.linalg.matrix_rank(N) < k:  # e.g. bound j and rate row j < nu coincide
                    continue
                b = np.array([-hi[j] if s else lo[j] for j, s in zip(act, sides)])
                K = np.block([[H, -N.T], [N, np.zeros((k, k))]])
                try:
                    sol = np.linalg.solve(K, np.concatenate([-g, b]))
                except np.linalg.LinAlgError:
                    continue
                x, mu = sol[:n], sol[n:]
                cx = C @ x
                if np.all(mu >= -1e-9 * scale) and np.all(cx >= lo - 1e-9 * bscale) \
                        and np.all(cx <= hi + 1e-9 * bscale):
                    found.append(x)
    assert found, "no KKT point: infeasible QP"
    return found[0], found


def random_ws(rng, n):
    ws = 0
    for j in rng.choice(2 * n, size=rng.integers(0, n + 1), replace=False):
        ws |= (1 << int(j)) | ((int(rng.integers(0, 2)) << (16 + int(j))))
    return ws


def check(H, g, lb, ub, lbA, ubA, nu, ws_in, enumerate_n4):
    n = len(g)
    x, info = O.qp_solve(H, g, lb, ub, lbA, ubA, nu, ws_in)
    C = rows(n, nu)
    lo = np.concatenate([lb, lbA])
    hi = np.concatenate([ub, ubA])
    if info.status == cmpc.CMPC_QP_INFEASIBLE and enumerate_n4 and n == 4:
        with pytest.raises(AssertionError, match="infeasible"):
            enumerate_optimum(H, g, lo, hi, C)
    if info.status != OK:
        return info.status
    kkt_certificate(H, g, lo, hi, C, x, info.ws)
    if enumerate_n4 and n == 4:
        xs, allx = enumerate_optimum(H, g, lo, hi, C)
        xscale = 1e-9 * (1.0 + np.abs(xs).max())
        for xo in allx:  # every KKT point is the same point (strict convexity)
            assert np.abs(xo - xs).max() <= xscale
        assert np.abs(x - xs).max() <= xscale, (x, xs)
    return info.status


@pytest.mark.parametrize("n,nu", [(4, 2), (8, 4)])
def test_oracle_solver_kkt_random(n, nu):
    rng = np.random.default_rng(77 + n)
    ok = active = 0
    trials = 300 if n == 4 else 600
    for t in range(trials):
        H, g, lb, ub, lbA, ubA = random_qp(rng, n, nu)
        ws_in = random_ws(rng, n) if t % 2 else 0
        st = check(H, g, lb, ub, lbA, ubA, nu, ws_in, enumerate_n4=(t % 3 == 0))
        ok += st == OK
        _, info = O.qp_solve(H, g, lb, ub, lbA, ubA, nu, ws_in)
        active += st == OK and info.ws != 0
    # the rest are infeasible (checked for nV = 4) or hit the nWSR cap
    assert ok > 0.5 * trials and active > 0.3 * trials, (ok, active)


@pytest.mark.parametrize("ctype", ["coop", "cent"])
def test_oracle_solver_kkt_condensed_qps(ctype):
    """The real condensed QPs (parallel plant, p = 50) with the Jacobi term
    G du_other of a random neighbour plan, cold and warm started."""
    _, setup, _, _ = GC.case(f"{ctype}-par")
    cfg = cmpc.reference_config("par", ctype, p=50)
    arr = cmpc.controller_arrays(cfg, setup)
    B = 40 if ctype == "coop" else 100  # enumeration (nV = 4) is the slow part
    lin, u_old, _, _ = synthetic_batch(cfg, B, seed=5)
    dims = CmpcDims.from_config(cfg, 1)
    rng = np.random.default_rng(6)
    nu, m = cfg.nu, cfg.m
    ok = active = 0
    batch = []
    for q in range(B * cfg.S):
        s = q % cfg.S
        H, f, _, _, G = O.build_qp(dims, lin[q], u_old[q], arr.y_ref[s], arr.ywt[s], arr.uwt[s])
        g = f + (G @ rng.uniform(-0.05, 0.05, G.shape[1]) if G.shape[1] else 0.0)
        uo = u_old[q][:nu]
        lb = np.tile(np.asarray(arr.lower[s]) - uo, m)
        ub = np.tile(np.asarray(arr.upper[s]) - uo, m)
        lbA = np.tile(np.asarray(arr.rate_lower[s]), m)
        ubA = np.tile(np.asarray(arr.rate_upper[s]), m)
        for ws_in in (0, random_ws(rng, len(g))):
            st = check(H, g, lb, ub, lbA, ubA, nu, ws_in, enumerate_n4=True)
            ok += st == OK
            x, info = O.qp_solve(H, g, lb, ub, lbA, ubA, nu, ws_in)
            active += st == OK and info.ws != 0
            if st == OK:
                batch.append((H, g, np.concatenate([lb, lbA]), np.concatenate([ub, ubA]), x, info.ws))
    assert ok >= 0.9 * 2 * B * cfg.S and active > 0, (ok, active)
    # the batched certificate (used on the GPU's full-size output) agrees
    H, g, lo, hi, x, ws = (np.array(a) for a in zip(*batch))
    C = rows(len(g[0]), nu)
    assert kkt_certificate_batch(H, g, lo, hi, C, x, ws).all()
    # ... and rejects a perturbed solution and a wrong working set
    x2 = x.copy()
    x2[:, 0] += 1e-3 * (1.0 + np.abs(x).max(axis=1))
    assert not kkt_certificate_batch(H, g, lo, hi, C, x2, ws).any()
    flip = ws ^ np.uint32(1 << 16)  # flip the side bit of row 0
    has0 = (ws & 1) == 1
    if has0.any():
        assert not kkt_certificate_batch(H, g, lo, hi, C, x, flip)[has0].any()
