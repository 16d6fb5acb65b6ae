"""Decision margins of the oracle solver (oracle/or_qp.c header): the
checker's near-tie flag that the GPU parity tests use to tell a rounding-level
near-tie from an active-set bug.

Every branch or index choice of the dual active-set solver records the
relative distance between its two sides; a QP slot's margin is the smallest
over its solves.  The GPU build forms H, f, G in a different summation order
than the oracle (agreement ~1e-13 relative), so the solvers see inputs that
differ at that level.  These tests pin what the margin means:
- a decision tie gives margin 0, a well-separated QP a large margin;
- under a relative input perturbation delta, every scenario whose
  working-set change sequence differs has a margin below ~delta: the margin
  predicts where sequences can diverge (checked at delta = 1e-4 and 1e-3,
  where some do);
- at delta = 1e-13 (the reassociation level) no unflagged scenario
  (margin >= 1e-9) differs.
"""
import numpy as np
import pytest

import _oracle as O
import cmpc
from cmpc._abi import CmpcDims
from cmpc.configs import reference_setup
from cmpc.synthetic import synthetic_batch

FLAG = 1e-9


def test_margin_of_a_tie_is_zero_and_of_a_clear_qp_large():
    n, nu = 4, 2
    H = np.diag([2.0, 2.0, 3.0, 4.0])
    lb, ub = np.full(n, -1.0), np.full(n, 1.0)
    lbA, ubA = np.full(n, -0.1), np.full(n, 0.1)
    # unconstrained optimum strictly inside everything
    x, info = O.qp_solve(H, np.array([0.01, -0.02, 0.0, 0.03]), lb, ub, lbA, ubA, nu)
    assert info.status == 0 and info.ws == 0
    assert info.margin > 1e-3
    # x_u = (0.2, 0.2, 0, 0): rate rows 0 and 1 are violated by exactly the
    # same amount -> the most-violated choice is a tie (lowest index wins)
    x, info = O.qp_solve(H, np.array([-0.4, -0.4, 0.0, 0.0]), lb, ub, lbA, ubA, nu)
    assert info.status == 0
    assert info.margin == 0.0
    assert info.trace[0] == 0x80 | 0x40 | 4     # added: rate row 0 (j = n + 0), upper side


def _run(cfg, arr, B, lin, state, K, init, threads=8):
    dims = CmpcDims.from_config(cfg, B)
    m = np.zeros(B * cfg.S)
    du, st, nw, tr, ntr = O.step(dims, arr, lin, K, *state, flags=cmpc.CMPC_APPLY_MOVE, init=init,
                                 threads=threads, want_trace=True, margin=m)
    return du, st, nw, tr, ntr, state[2].copy(), m


def _diverged(a, b, B):
    du1, s1, n1, t1, nt1, w1, _ = a
    du2, s2, n2, t2, nt2, w2, _ = b
    d = (s1 != s2) | (w1 != w2) | (n1 != n2) | np.any(nt1 != nt2, axis=1) | np.any(t1 != t2, axis=(1, 2))
    return d.reshape(B, -1).any(1)


@pytest.mark.parametrize("plant,ctype,p,K", [("par", "coop", 50, 9), ("ser", "coop", 50, 9),
                                             ("par", "cent", 50, 1)])
def test_margin_predicts_divergence(plant, ctype, p, K):
    cfg = cmpc.reference_config(plant, ctype, p=p)
    arr = cmpc.controller_arrays(cfg, reference_setup(plant, ctype))
    B = 2048
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=100 + p)
    base = _run(cfg, arr, B, lin, [u_old.copy(), du_old.copy(), ws.copy()], K, True)
    m0 = base[-1].reshape(B, -1).min(1)
    total = 0
    for delta in (1e-13, 1e-4, 1e-3):
        rng = np.random.default_rng(7)
        lin2 = lin * (1 + delta * rng.normal(size=lin.shape))
        pert = _run(cfg, arr, B, lin2, [u_old.copy(), du_old.copy(), ws.copy()], K, True)
        div = _diverged(base, pert, B)
        m = np.minimum(m0, pert[-1].reshape(B, -1).min(1))
        bound = FLAG if delta < 1e-9 else 10 * delta
        print(plant, ctype, "delta", delta, "diverged", div.sum(), "flagged", (m < bound).sum(),
              "largest margin among diverged", m[div].max() if div.any() else None)
        assert not np.any(div & (m >= bound)), np.flatnonzero(div & (m >= bound))[:5]
        # the oracle's own margin alone (what the GPU tests use) at the
        # reassociation level
        if delta < 1e-9:
            assert not np.any(div & (m0 >= FLAG))
        total += div.sum()
    # the perturbed runs do diverge somewhere, so the bound above is exercised
    assert total > 0
