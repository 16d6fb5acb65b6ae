"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden records.  Marked gpu; runs on an MI355X.

Tolerances:
  H, f, G   : |gpu - oracle| <= 1e-11 * max|.| of the same matrix (FP64
              reassociation: the kernel folds W = L_W L_W' into the
              propagation and never forms Su; the oracle follows the
              reference's O(p^2) order)
  du        : abs 1e-10 + rel 1e-9
  active-set: statuses, nWSR, working sets and working-set change sequences
              bit-exact, except scenarios whose oracle solves take a
              decision within 1e-9 (relative) of a tie (the oracle's decision
              margin, oracle/or_qp.c; tests/test_solver_margins.py shows it
              predicts where sequences can diverge); flagged scenarios are
              counted, printed and bounded (at most 1/32 of the scenarios of
              a step, 1/1000 at the headline size), nothing else is excused
  solver    : on identical (H, g, bounds, ws) the device solver is bit-exact
              with the oracle solver (same arithmetic order, no contraction)
"""
import numpy as np
import pytest

import _oracle as O
import cmpc
import golden_cases as GC
from cmpc._abi import CmpcDims
from cmpc.synthetic import synthetic_batch

pytestmark = pytest.mark.gpu


def make_ctx(cfg, arr, B, lin, u_old, du_old, ws):
    ctx = cmpc.Context(cfg, B)
    ctx.configure(arr)
    ctx.set_state(u_old, du_old, ws)
    ctx.upload_lin(lin)
    return ctx


GPU_GOLDEN = ("cent-par", "coop-par", "ncoop-par", "cent-ser", "coop-ser", "ncoop-ser")


@pytest.mark.parametrize("name", GPU_GOLDEN)
def test_gpu_step0_matches_reference(name):
    cfg, setup, arr, g = GC.case(name)
    dims = CmpcDims.from_config(cfg, 1)
    L = cmpc.layout_of(dims)
    x0, u_full = cmpc.plant_default(cfg.plant)
    y = cmpc.plant_output(cfg.plant, x0)
    lin = GC.step0_records(cfg, dims, L, cmpc.plant_lin_record, x0, u_full, y)
    with make_ctx(cfg, arr, 1, lin, np.zeros((cfg.S, cfg.nu_tot)), np.zeros((cfg.S, cfg.nV)),
                  np.zeros(cfg.S, np.uint32)) as ctx:
        ctx.build()
        ctx.init_warmstart()
        ctx.iterate(g["n_iterations"])
        du, status, nwsr = ctx.download()
    assert (status == 0).all()
    u = cmpc.plant_input_from_plans(cfg, du.reshape(1, cfg.S, cfg.nV))[0]
    GC.assert_six_digits(u, g["u0"])


def oracle_qps(cfg, arr, lin, u_old):
    dims = CmpcDims.from_config(cfg, 1)
    Hs, fs, Gs = [], [], []
    for q in range(lin.shape[0]):
        s = q % cfg.S
        H, f, _, _, G = O.build_qp(dims, lin[q], u_old[q], arr.y_ref[s], arr.ywt[s], arr.uwt[s])
        Hs.append(H); fs.append(f); Gs.append(G)
    return np.stack(Hs), np.stack(fs), np.stack(Gs)


# p = 100 and 200 run the row kernel's ring lines (one wrap at p = 100, three
# per line at p = 200: rows_layout.cpp)
BUILD_CASES = [("par", "coop", 20), ("par", "coop", 50), ("par", "ncoop", 50),
               ("par", "cent", 50), ("par", "coop", 100), ("ser", "ncoop", 50),
               ("ser", "coop", 50), ("ser", "cent", 50), ("ser", "coop", 100),
               ("ser", "cent", 100), ("par", "cent", 200)]


def setup_for(plant, ctype):
    name = f"{ctype}-{plant}"
    return GC.case(name)


@pytest.mark.parametrize("variant", [cmpc.CMPC_BUILD_WAVE, cmpc.CMPC_BUILD_ROWS])
@pytest.mark.parametrize("plant,ctype,p", BUILD_CASES)
def test_gpu_build_matches_oracle(plant, ctype, p, variant):
    """Both build kernels (one QP per wave / four QPs per wave, one per DPP
    row) against the oracle; B*S = 94 QPs, not a multiple of four, so the
    row kernel's last group is partial."""
    _, setup, _, _ = setup_for(plant, ctype)
    cfg = cmpc.reference_config(plant, ctype, p=p)
    arr = cmpc.controller_arrays(cfg, setup)
    B = 47
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=11 + p)
    with make_ctx(cfg, arr, B, lin, u_old, du_old, ws) as ctx:
        ctx.set_build_variant(variant)
        ctx.build()
        H, f, G = ctx.download_qp()
    Ho, fo, Go = oracle_qps(cfg, arr, lin, u_old)
    assert np.all(np.abs(H - np.transpose(H, (0, 2, 1))) == 0), "H must be exactly symmetric"
    for q in range(B * cfg.S):
        sH = np.abs(Ho[q]).max()
        np.testing.assert_allclose(H[q], Ho[q], rtol=0, atol=1e-11 * sH)
        sf = max(np.abs(fo[q]).max(), 1e-300)
        np.testing.assert_allclose(f[q], fo[q], rtol=0, atol=1e-10 * max(sf, 1e-6 * sH))
        if cfg.nVo:
            sG = max(np.abs(Go[q]).max(), 1e-300)
            np.testing.assert_allclose(G[q], Go[q], rtol=0, atol=1e-11 * max(sG, 1e-6 * sH))


# delays other than the reference plants' (0, 40, 0, 40): other segment
# bounds, rings with other wrap steps, two-step delays and one of p - 1 (a
# one-step delay with two delayed inputs is rejected: test_abi.py)
OTHER_DELAYS = [("par", "coop", 50, (0, 10, 0, 25)), ("par", "coop", 100, (0, 30, 0, 60)),
                ("par", "cent", 120, (0, 45, 0, 45)), ("ser", "coop", 80, (0, 15, 0, 50)),
                ("par", "ncoop", 64, (0, 2, 0, 63)), ("par", "coop", 50, (0, 40, 0, 2)),
                # short horizons: delays beyond p, a one-step remainder block
                ("par", "coop", 7, (0, 40, 0, 40)), ("par", "coop", 3, (0, 2, 0, 2)),
                ("ser", "cent", 11, (0, 4, 0, 9))]


@pytest.mark.parametrize("variant", [cmpc.CMPC_BUILD_WAVE, cmpc.CMPC_BUILD_ROWS])
@pytest.mark.parametrize("plant,ctype,p,delays", OTHER_DELAYS)
def test_gpu_build_other_delays_match_oracle(plant, ctype, p, delays, variant):
    """Both build kernels against the oracle for input delays the reference
    plants do not use (the delay lines, segment bounds and ring wraps of the
    row kernel are runtime parameters)."""
    import dataclasses
    _, setup, _, _ = setup_for(plant, ctype)
    cfg = dataclasses.replace(cmpc.reference_config(plant, ctype, p=p), delays=tuple(delays))
    arr = cmpc.controller_arrays(cfg, setup)
    B = 47
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=23 + p)
    with make_ctx(cfg, arr, B, lin, u_old, du_old, ws) as ctx:
        ctx.set_build_variant(variant)
        ctx.build()
        assert ctx.last_build_kernel() == variant
        H, f, G = ctx.download_qp()
    Ho, fo, Go = oracle_qps(cfg, arr, lin, u_old)
    assert np.all(np.abs(H - np.transpose(H, (0, 2, 1))) == 0)
    for q in range(B * cfg.S):
        sH = np.abs(Ho[q]).max()
        np.testing.assert_allclose(H[q], Ho[q], rtol=0, atol=1e-11 * sH)
        sf = max(np.abs(fo[q]).max(), 1e-300)
        np.testing.assert_allclose(f[q], fo[q], rtol=0, atol=1e-10 * max(sf, 1e-6 * sH))
        if cfg.nVo:
            sG = max(np.abs(Go[q]).max(), 1e-300)
            np.testing.assert_allclose(G[q], Go[q], rtol=0, atol=1e-11 * max(sG, 1e-6 * sH))


@pytest.mark.parametrize("plant,ctype,p", [("par", "coop", 50), ("par", "cent", 50),
                                           ("ser", "coop", 100), ("par", "coop", 20),
                                           ("par", "coop", 100), ("par", "cent", 200),
                                           ("ser", "cent", 100)])
def test_gpu_build_variants_agree_large(plant, ctype, p):
    """Row-layout vs one-QP-per-wave build on a large batch (persistent grid,
    several groups per wave): H, f, G agree to FP64 reassociation.  par-coop
    p = 100 runs the row kernel in 2-wave workgroups."""
    _, setup, _, _ = setup_for(plant, ctype)
    cfg = cmpc.reference_config(plant, ctype, p=p)
    arr = cmpc.controller_arrays(cfg, setup)
    B = 20001
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=101 + p, n_distinct=512)
    out = {}
    with make_ctx(cfg, arr, B, lin, u_old, du_old, ws) as ctx:
        for v in (cmpc.CMPC_BUILD_WAVE, cmpc.CMPC_BUILD_ROWS):
            ctx.set_build_variant(v)
            ctx.build()
            out[v] = ctx.download_qp()
    (Hw, fw, Gw), (Hr, fr, Gr) = out[cmpc.CMPC_BUILD_WAVE], out[cmpc.CMPC_BUILD_ROWS]
    assert np.isfinite(Hr).all() and np.isfinite(fr).all() and np.isfinite(Gr).all()
    sH = np.abs(Hw).max(axis=(1, 2))
    assert (np.abs(Hr - Hw).max(axis=(1, 2)) <= 1e-11 * sH).all()
    assert (np.abs(fr - fw).max(axis=1) <= 1e-10 * np.maximum(np.abs(fw).max(axis=1), 1e-6 * sH)).all()
    if cfg.nVo:
        assert (np.abs(Gr - Gw).max(axis=(1, 2)) <= 1e-11 * np.maximum(np.abs(Gw).max(axis=(1, 2)), 1e-6 * sH)).all()


def test_gpu_solver_bitexact_on_identical_inputs():
    """Device solver == oracle solver bit for bit (x, status, changes, ws,
    trace) on the oracle's QPs, warm-started from assorted working sets."""
    _, setup, _, _ = setup_for("par", "coop")
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, setup)
    B = 64
    lin, u_old, _, _ = synthetic_batch(cfg, B, seed=5)
    Ho, fo, Go = oracle_qps(cfg, arr, lin, u_old)
    rng = np.random.default_rng(3)
    n, nu = cfg.nV, cfg.nu
    nq = B * cfg.S
    lb = np.zeros((nq, n)); ub = np.zeros((nq, n)); lbA = np.zeros((nq, n)); ubA = np.zeros((nq, n))
    g = fo + np.einsum("qac,qc->qa", Go, rng.normal(0, 0.05, (nq, cfg.nVo)))
    for q in range(nq):
        s = q % cfg.S
        for mv in range(cfg.m):
            lb[q, mv * nu:(mv + 1) * nu] = arr.lower[s] - u_old[q, :nu]
            ub[q, mv * nu:(mv + 1) * nu] = arr.upper[s] - u_old[q, :nu]
            lbA[q, mv * nu:(mv + 1) * nu] = arr.rate_lower[s]
            ubA[q, mv * nu:(mv + 1) * nu] = arr.rate_upper[s]
    # also stress: tighter boxes and random warm starts
    g2 = g * rng.uniform(1, 40, (nq, 1))
    ws_in = np.zeros(nq, np.uint32)
    for q in range(nq):
        bits = rng.choice(2 * n, size=rng.integers(0, 3), replace=False)
        for j in bits:
            ws_in[q] |= np.uint32(1 << int(j))
            if rng.random() < 0.5:
                ws_in[q] |= np.uint32(1 << (16 + int(j)))
    for gg, wsi in ((g, np.zeros(nq, np.uint32)), (g2, ws_in)):
        x, st, nchg, wso, tr, ntr = cmpc.qp_solve_batch(Ho, gg, lb, ub, lbA, ubA, nu, wsi)
        for q in range(nq):
            xo, info = O.qp_solve(Ho[q], gg[q], lb[q], ub[q], lbA[q], ubA[q], nu, int(wsi[q]))
            assert st[q] == info.status
            assert nchg[q] == info.nchg
            assert wso[q] == info.ws
            assert ntr[q] == info.ntrace
            assert bytes(tr[q][:ntr[q]]) == bytes(info.trace[:info.ntrace])
            assert np.array_equal(x[q], xo), (q, x[q], xo)


def test_gpu_map_form_solver_bitexact_on_identical_inputs():
    """The Jacobi iteration's solve (map form, g = f + G d;
    cmpc_qp_solve_batch_map, the solve of DistributedSolver::UpdateAndSolveQP)
    == the oracle's or_qp_solve_map bit for bit, on the oracle's QPs with
    plans d of several sizes and assorted warm starts (phase-A drops from the
    map's multipliers, phase-B adds)."""
    _, setup, _, _ = setup_for("par", "coop")
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, setup)
    B = 64
    lin, u_old, _, _ = synthetic_batch(cfg, B, seed=6)
    Ho, fo, Go = oracle_qps(cfg, arr, lin, u_old)
    rng = np.random.default_rng(4)
    n, nu = cfg.nV, cfg.nu
    nq = B * cfg.S
    lb = np.zeros((nq, n)); ub = np.zeros((nq, n)); lbA = np.zeros((nq, n)); ubA = np.zeros((nq, n))
    for q in range(nq):
        s = q % cfg.S
        for mv in range(cfg.m):
            lb[q, mv * nu:(mv + 1) * nu] = arr.lower[s] - u_old[q, :nu]
            ub[q, mv * nu:(mv + 1) * nu] = arr.upper[s] - u_old[q, :nu]
            lbA[q, mv * nu:(mv + 1) * nu] = arr.rate_lower[s]
            ubA[q, mv * nu:(mv + 1) * nu] = arr.rate_upper[s]
    total = 0
    for scale in (0.01, 0.2, 2.0):
        d = rng.normal(0, scale, (nq, cfg.nVo))
        ws_in = np.zeros(nq, np.uint32)
        for q in range(nq):
            for j in rng.choice(2 * n, size=rng.integers(0, 3), replace=False):
                ws_in[q] |= np.uint32(1 << int(j))
                if rng.random() < 0.5:
                    ws_in[q] |= np.uint32(1 << (16 + int(j)))
        x, st, nchg, wso, tr, ntr = cmpc.qp_solve_batch_map(Ho, fo, Go, d, lb, ub, lbA, ubA, nu, ws_in)
        for q in range(nq):
            xo, info = O.qp_solve_map(Ho[q], fo[q], Go[q], d[q], lb[q], ub[q], lbA[q], ubA[q], nu, int(ws_in[q]))
            assert st[q] == info.status and nchg[q] == info.nchg and wso[q] == info.ws, q
            assert bytes(tr[q][:ntr[q]]) == bytes(info.trace[:info.ntrace]), q
            assert np.array_equal(x[q], xo), (q, x[q], xo)
        total += int(ntr.sum())
    assert total > 50


def test_gpu_solver_status_paths():
    """Zero move on every non-success (libs/mpc_qp_solver.cc:66-69)."""
    n, nu = 4, 2
    H = np.tile(np.diag([2.0, 3.0, 4.0, 5.0]), (3, 1, 1))
    H[2] = -H[2]                                           # not positive definite
    g = np.array([[1.0, -1.0, 0.5, 0.2]] * 3)
    lb = np.full((3, n), -1.0); ub = np.full((3, n), 1.0)
    lbA = np.full((3, n), -0.1); ubA = np.full((3, n), 0.1)
    lb[1, 0] = 0.5; ub[1, 0] = 0.6                         # bound beyond the rate limit: infeasible
    x, st, nchg, _, _, _ = cmpc.qp_solve_batch(H, g, lb, ub, lbA, ubA, nu)
    assert st[0] == cmpc.CMPC_QP_OK and st[1] == cmpc.CMPC_QP_INFEASIBLE
    assert st[2] == cmpc.CMPC_QP_NOT_PD
    # non-finite gradients (a NaN, an infinite entry) and a NaN Hessian: zero
    # move with a failure status, as the oracle
    H2 = np.tile(np.diag([2.0, 3.0, 4.0, 5.0]), (3, 1, 1))
    H2[2, 1, 1] = np.nan
    g2 = np.array([[1.0, np.nan, 0.5, 0.2], [np.inf, -1.0, 0.5, 0.2], [1.0, -1.0, 0.5, 0.2]])
    lb2 = np.full((3, n), -1.0); ub2 = np.full((3, n), 1.0)
    lbA2 = np.full((3, n), -0.1); ubA2 = np.full((3, n), 0.1)
    x2, st2, _, _, _, _ = cmpc.qp_solve_batch(H2, g2, lb2, ub2, lbA2, ubA2, nu)
    for q in range(3):
        xo, info = O.qp_solve(H2[q], g2[q], lb2[q], ub2[q], lbA2[q], ubA2[q], nu, 0)
        assert st2[q] == info.status and st2[q] != cmpc.CMPC_QP_OK, (q, st2[q], info.status)
        assert np.all(x2[q] == 0.0) and np.all(xo == 0.0)
    assert np.all(x[1] == 0) and np.all(x[2] == 0)
    # n_wsr cap: the unconstrained optimum violates several rate rows
    g3 = np.array([[-50.0, 60.0, 80.0, -90.0]])
    x, st, nchg, _, _, _ = cmpc.qp_solve_batch(H[:1], g3, lb[:1] * 0 - 1, ub[:1] * 0 + 1,
                                               lbA[:1], ubA[:1], nu, max_chg=1)
    assert st[0] == cmpc.CMPC_QP_MAX_NWSR and np.all(x[0] == 0)
    for q in range(1):
        xo, info = O.qp_solve(H[0], g3[0], lb[0] * 0 - 1, ub[0] * 0 + 1, lbA[0], ubA[0], nu,
                              0, max_chg=1)
        assert info.status == st[0]


STEP_CASES = [("par", "coop", 20, 9), ("par", "coop", 50, 9), ("par", "ncoop", 50, 9),
              ("par", "cent", 50, 1), ("ser", "ncoop", 50, 9),
              ("ser", "coop", 50, 9), ("ser", "cent", 50, 1)]

NEAR_TIE = 1e-9   # oracle decision margin below which a sequence may differ (or_qp.c)


def compare_step(B, S, K, dev, orc, margin, excused):
    """One step's device results against the oracle's, per scenario.  dev /
    orc = (du, status, nwsr, ws, trace, ntrace).  Returns (unflagged,
    flagged) scenario masks of differing working-set sequences; a scenario
    may differ only when the oracle flags one of its solves as a near-tie
    (margin < NEAR_TIE) in this step, or it already diverged at a flagged
    near-tie earlier (its warm starts then differ)."""
    du, st, nw, ws, tr, ntr = dev
    odu, ost, onw, ows, otr, ontr = orc
    seq = np.zeros(B * S, bool)
    for k in range(K):
        n_ = ntr[:, k]
        seq |= n_ != ontr[:, k]
        for c in range(16):
            live = c < np.minimum(n_, ontr[:, k])
            seq |= live & (tr[:, k, c] != otr[:, k, c])
    diff = ((st != ost) | (nw != onw) | (ws != ows) | seq).reshape(B, S).any(1)
    flag = (margin < NEAR_TIE).reshape(B, S).any(1)
    return diff & ~flag & ~excused, diff & (flag | excused)


def _step_parity(cfg, setup, K, B=96, seed=100, expect_fused=None, threads=1, step_variant=None):
    """Three closed-loop steps (state persists: ws, du_old, u_old with the
    first move applied), device and oracle each on their own state: plans
    within tolerance, statuses, nWSR, working sets and the working-set change
    sequences of every Jacobi iteration bit-exact, except scenarios the
    oracle flags as near-ties (decision margin < 1e-9, or_qp.c), which are
    counted and printed."""
    arr = cmpc.controller_arrays(cfg, setup)
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=seed)
    o_u, o_du, o_ws = u_old.copy(), du_old.copy(), ws.copy()
    dims = CmpcDims.from_config(cfg, B)
    nq = B * cfg.S
    excused = np.zeros(B, bool)
    with make_ctx(cfg, arr, B, lin, u_old, du_old, ws) as ctx:
        if step_variant is not None:
            ctx.set_step_variant(step_variant)
        for step in range(3):
            flags = cmpc.CMPC_APPLY_MOVE | cmpc.CMPC_TRACE
            if step == 0:
                ctx.build()
                ctx.init_warmstart()
                ctx.iterate(K, flags)
            else:
                ctx.step(K, flags)
                if expect_fused is not None:
                    assert ctx.last_step_fused() == expect_fused, step
            du, st, nw = ctx.download()
            tr, ntr = ctx.download_trace(K)
            u_g, du_g, ws_g = ctx.get_state()
            margin = np.zeros(nq)
            odu, ost, onw, otr, ontr = O.step(dims, arr, lin, K, o_u, o_du, o_ws,
                                              flags=cmpc.CMPC_APPLY_MOVE, init=(step == 0),
                                              want_trace=True, margin=margin, threads=threads)
            bad, flagged = compare_step(B, cfg.S, K, (du, st, nw, ws_g, tr, ntr),
                                        (odu, ost, onw, o_ws, otr, ontr), margin, excused)
            print(f"step {step}: scenarios differing at a flagged near-tie {flagged.sum()}, "
                  f"unflagged {bad.sum()}, smallest oracle margin {margin.min():.3g}")
            assert not bad.any(), np.flatnonzero(bad)[:10]
            # the near-tie allowance is bounded: a regression that changes
            # near-tie decisions wholesale fails here
            assert flagged.sum() <= max(3, B // 32), flagged.sum()
            excused |= flagged
            keep = np.repeat(~excused, cfg.S)
            np.testing.assert_allclose(du[keep], odu[keep], rtol=1e-9, atol=1e-10)
            np.testing.assert_allclose(u_g[keep], o_u[keep], rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("plant,ctype,p,K", STEP_CASES)
def test_gpu_step_matches_oracle(plant, ctype, p, K):
    """_step_parity on the reference plants' configurations."""
    _, setup, _, _ = setup_for(plant, ctype)
    _step_parity(cmpc.reference_config(plant, ctype, p=p), setup, K, seed=100 + p)


@pytest.mark.parametrize("plant,ctype,p,K,B", [("par", "cent", 200, 1, 1024),   # SURVEY config 5
                                              ("par", "coop", 50, 9, 1)])      # the B = 1 call
def test_gpu_fused_step_matches_oracle(plant, ctype, p, K, B):
    """_step_parity through the fused one-launch steps at these sizes
    (config 5: the one-QP-per-wave build with the row solver in the same
    kernel; B = 1 coop-par: the fused step with the lane solver; pinned with
    CMPC_STEP_FUSED; AUTO runs the split build and the iterate kernel at B = 1),
    each step after the first checked to have run fused, directly against the
    oracle over three steps with the move applied; then the same through AUTO."""
    _, setup, _, _ = setup_for(plant, ctype)
    cfg = cmpc.reference_config(plant, ctype, p=p)
    _step_parity(cfg, setup, K, B=B, seed=300 + p, expect_fused=1, threads=8, step_variant=cmpc.CMPC_STEP_FUSED)
    _step_parity(cfg, setup, K, B=B, seed=300 + p, expect_fused=int(B > 1), threads=8)


# other delays and move counts: m = 1 (nV = nu) and m = 3 (the one-QP-per-wave
# build kernel, nV = 6 solves)
OTHER_STEP_CASES = [("par", "coop", 50, 2, (0, 10, 0, 25), 9), ("par", "coop", 120, 2, (0, 45, 0, 45), 9),
                    ("ser", "coop", 80, 2, (0, 15, 0, 50), 5), ("par", "coop", 50, 1, (0, 40, 0, 40), 9),
                    ("par", "coop", 30, 3, (0, 40, 0, 40), 9), ("par", "ncoop", 64, 2, (0, 2, 0, 63), 1)]


@pytest.mark.parametrize("plant,ctype,p,m,delays,K", OTHER_STEP_CASES)
def test_gpu_step_other_dims_matches_oracle(plant, ctype, p, m, delays, K):
    """_step_parity for input delays and move counts the reference plants do
    not use."""
    import dataclasses
    _, setup, _, _ = setup_for(plant, ctype)
    cfg = dataclasses.replace(cmpc.reference_config(plant, ctype, p=p, m=m), delays=tuple(delays))
    _step_parity(cfg, setup, K, seed=300 + p + m)


def test_gpu_step_matches_oracle_headline_size():
    """The bench workload (coop-par p = 50, 65 536 scenarios = 131 072 QPs,
    K = 9): cold solves, then two steps with the first move applied, every
    QP's status, nWSR, working set and change sequence of every Jacobi
    iteration against the oracle, each side on its own state."""
    import os
    _, setup, _, _ = setup_for("par", "coop")
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, setup)
    B, K = 65536, 9
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=1002, n_distinct=2048)
    o_u, o_du, o_ws = u_old.copy(), du_old.copy(), ws.copy()
    dims = CmpcDims.from_config(cfg, B)
    nq = B * cfg.S
    threads = min(16, os.cpu_count() or 1)
    excused = np.zeros(B, bool)
    active = 0.0
    with make_ctx(cfg, arr, B, lin, u_old, du_old, ws) as ctx:
        for step in range(2):
            flags = cmpc.CMPC_APPLY_MOVE | cmpc.CMPC_TRACE
            if step == 0:
                ctx.build()
                ctx.init_warmstart()
                ctx.iterate(K, flags)
            else:
                ctx.step(K, flags)
            du, st, nw = ctx.download()
            tr, ntr = ctx.download_trace(K)
            u_g, du_g, ws_g = ctx.get_state()
            margin = np.zeros(nq)
            odu, ost, onw, otr, ontr = O.step(dims, arr, lin, K, o_u, o_du, o_ws,
                                              flags=cmpc.CMPC_APPLY_MOVE, init=(step == 0),
                                              threads=threads, want_trace=True, margin=margin)
            bad, flagged = compare_step(B, cfg.S, K, (du, st, nw, ws_g, tr, ntr),
                                        (odu, ost, onw, o_ws, otr, ontr), margin, excused)
            active = (ws_g != 0).mean()
            print(f"step {step}: {nq} QPs x {K} iterations, changes {int(ntr.sum())}, active "
                  f"{active:.3f}; differing at a flagged near-tie {flagged.sum()}, unflagged "
                  f"{bad.sum()}, QPs flagged {(margin < NEAR_TIE).sum()}")
            assert not bad.any(), np.flatnonzero(bad)[:10]
            assert flagged.sum() <= B // 1000, flagged.sum()  # bounded near-tie allowance
            excused |= flagged
            keep = np.repeat(~excused, cfg.S)
            np.testing.assert_allclose(du[keep], odu[keep], rtol=1e-9, atol=1e-10)
    assert active > 0.05


def test_gpu_large_batch_properties():
    """BASELINE-size batch (coop-par p=50, B=65536): every QP solved, every
    plan feasible, plans of a sample equal to the oracle's."""
    _, setup, _, _ = setup_for("par", "coop")
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, setup)
    B = 65536
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=1002, n_distinct=512)
    with make_ctx(cfg, arr, B, lin, u_old, du_old, ws) as ctx:
        ctx.build()
        ctx.init_warmstart()
        ctx.iterate(9)
        du, st, nw = ctx.download()
        ctx_state = ctx.get_state()
    assert (st == 0).mean() > 0.999
    nu, n = cfg.nu, cfg.nV
    tol = 1e-9
    for mv in range(cfg.m):
        blk = du[:, mv * nu:(mv + 1) * nu]
        s = np.arange(B * cfg.S) % cfg.S
        assert np.all(blk >= arr.lower[s] - u_old[:, :nu] - tol)
        assert np.all(blk <= arr.upper[s] - u_old[:, :nu] + tol)
        rate = blk if mv == 0 else blk - du[:, (mv - 1) * nu:mv * nu]
        assert np.all(rate >= arr.rate_lower[s] - tol) and np.all(rate <= arr.rate_upper[s] + tol)
    _, _, ws_out = ctx_state
    active = ws_out != 0  # at least one active constraint (bound or rate row)
    print("fraction of QPs with an active constraint:", active.mean())
    assert active.mean() > 0.05
    sample = np.arange(0, B, B // 64)
    qs = np.concatenate([sample * 2, sample * 2 + 1])
    sub = CmpcDims.from_config(cfg, len(sample))
    lin_s = np.ascontiguousarray(lin.reshape(B, 2, -1)[sample].reshape(len(sample) * 2, -1))
    u_s = np.ascontiguousarray(u_old.reshape(B, 2, -1)[sample].reshape(len(sample) * 2, -1))
    odu, ost, *_ = O.step(sub, arr, lin_s, 9, u_s, np.zeros((len(qs), n)),
                          np.zeros(len(qs), np.uint32), init=True)
    np.testing.assert_allclose(du.reshape(B, 2, n)[sample].reshape(-1, n), odu, rtol=1e-9,
                               atol=1e-10)


def test_gpu_max_batch_64bit_offsets():
    """Maximum-size case: 2^20 scenarios (2 097 152 QPs; 5.2 GB of lin records
    on the device, so byte offsets pass 2^32 and QP indices 2^21), records made
    by the device producer from 1 024 distinct operating points and u_old
    rows tiled with the same period.  Every QP must equal its first copy bit
    for bit (H, f, G, the plans, status and working sets: an index or offset
    overflow anywhere in the batch breaks that), and the last scenarios must
    match the oracle."""
    import torch
    from cmpc.synthetic import synthetic_operating_points, synthetic_u_old
    _, setup, _, _ = setup_for("par", "coop")
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, setup)
    B, nd, S, n = 1 << 20, 1024, cfg.S, cfg.nV
    xs, us, ys = synthetic_operating_points(cfg, B, seed=2024, n_distinct=nd)
    u_nd = synthetic_u_old(cfg, nd, np.random.default_rng(2025))
    u_old = np.ascontiguousarray(np.tile(u_nd, (B // nd, 1)))
    tx, tu, ty = (torch.from_numpy(a).cuda() for a in (xs, us, ys))
    with cmpc.Context(cfg, B) as ctx:
        ctx.configure(arr)
        ctx.set_state(u_old, np.zeros((B * S, n)), np.zeros(B * S, np.uint32))
        ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
        ctx.build()
        assert ctx.last_build_kernel() == cmpc.CMPC_BUILD_ROWS
        H, f, G = ctx.download_qp()
        ctx.init_warmstart()
        ctx.iterate(9)
        du, st, nw = ctx.download()
        _, _, ws = ctx.get_state()
    per = nd * S  # QPs per period
    for a in (H, f, G, du, st, nw, ws):
        v = a.reshape(B * S // per, per, -1)
        assert np.array_equal(v, np.broadcast_to(v[:1], v.shape)), "copies differ"
    assert (st == 0).all()
    # the last eight scenarios against the oracle (records from the host producer)
    last = np.arange(B - 8, B)
    dims1 = CmpcDims.from_config(cfg, 1)
    L = cmpc.layout_of(dims1)
    lin_s = np.zeros((len(last) * S, L.rec_len))
    for i, b in enumerate(last):
        for s_ in range(S):
            r = lin_s[i * S + s_]
            cmpc.plant_lin_record(cfg, dims1, s_, xs[b], us[b], out=r)
            r[L.off_y:L.off_y + cfg.ny] = ys[b][cfg.out_idx[s_]]
    qs = (last[:, None] * S + np.arange(S)[None, :]).reshape(-1)
    u_s = np.ascontiguousarray(u_old[qs])
    Ho, fo, Go = oracle_qps(cfg, arr, lin_s, u_s)
    for i, q in enumerate(qs):
        sH = np.abs(Ho[i]).max()
        np.testing.assert_allclose(H[q], Ho[i], rtol=0, atol=1e-11 * sH)
        np.testing.assert_allclose(f[q], fo[i], rtol=0, atol=1e-10 * max(np.abs(fo[i]).max(), 1e-6 * sH))
    sub = CmpcDims.from_config(cfg, len(last))
    odu, ost, *_ = O.step(sub, arr, lin_s, 9, u_s.copy(), np.zeros((len(qs), n)),
                          np.zeros(len(qs), np.uint32), init=True)
    np.testing.assert_allclose(du[qs], odu, rtol=1e-9, atol=1e-10)


def test_gpu_full_batch_kkt():
    """At the bench size (coop-par p=50, B=65536, 131 072 QPs) every QP the
    device solves is the QP optimum: a KKT certificate (feasibility, tight
    active rows, multipliers >= 0, stationarity; relative 1e-9) from the
    working set the kernel reports.  One Jacobi iteration from a random
    neighbour plan, so g = f + G du_other is known on the host."""
    from test_solver_kkt import kkt_certificate_batch, rows
    _, setup, _, _ = setup_for("par", "coop")
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, setup)
    B, S, nu, m = 65536, cfg.S, cfg.nu, cfg.m
    lin, u_old, _, ws = synthetic_batch(cfg, B, seed=1003, n_distinct=2048)
    du_prev = np.random.default_rng(4).uniform(-0.05, 0.05, (B * S, cfg.nV))
    with make_ctx(cfg, arr, B, lin, u_old, du_prev, ws) as ctx:
        ctx.build()
        ctx.init_warmstart()           # cold solves: sets the working sets only
        H, f, G = ctx.download_qp()
        ctx.iterate(1)
        du, st, _ = ctx.download()
        _, _, ws_out = ctx.get_state()
    other = np.arange(B * S) ^ 1       # S = 2: the neighbour sub-controller
    g = f + np.einsum("qij,qj->qi", G, du_prev[other])
    s = np.arange(B * S) % S
    uo = u_old[:, :nu]
    lo = np.concatenate([np.tile(arr.lower[s] - uo, m), np.tile(arr.rate_lower[s], m)], axis=1)
    hi = np.concatenate([np.tile(arr.upper[s] - uo, m), np.tile(arr.rate_upper[s], m)], axis=1)
    okq = st == 0
    assert okq.mean() > 0.999
    cert = kkt_certificate_batch(H[okq], g[okq], lo[okq], hi[okq], rows(cfg.nV, nu), du[okq], ws_out[okq])
    print("QPs solved:", okq.sum(), "with active constraints:", (ws_out[okq] != 0).mean())
    assert cert.all(), np.flatnonzero(~cert)[:10]
    assert (ws_out[okq] != 0).mean() > 0.05


# SURVEY.md §8(d) configs restated as parity cases (the bench line is config
# "coop p=50"; these run at their own sizes): (1) cent-ser at the reference's
# p=100 (its CPU timing case, here batched B=4096), (2) coop-par p=20 B=4096
# K=9, (3) ncoop-par p=50 B=65536 K=1, (5) cent-par p=200 B=1024 K=1.
SURVEY_CONFIGS = [("ser", "cent", 100, 4096, 1), ("par", "coop", 20, 4096, 9),
                  ("par", "ncoop", 50, 65536, 1), ("par", "cent", 200, 1024, 1)]


@pytest.mark.parametrize("plant,ctype,p,B,K", SURVEY_CONFIGS)
def test_gpu_survey_config(plant, ctype, p, B, K):
    _, setup, _, _ = setup_for(plant, ctype)
    cfg = cmpc.reference_config(plant, ctype, p=p)
    arr = cmpc.controller_arrays(cfg, setup)
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=300 + p, n_distinct=min(B, 1024))
    with make_ctx(cfg, arr, B, lin, u_old, du_old, ws) as ctx:
        ctx.build()
        H, f, G = ctx.download_qp()
        ctx.init_warmstart()
        ctx.iterate(K)
        du, st, _ = ctx.download()
    assert (st == 0).mean() > 0.999
    assert np.all(H == np.transpose(H, (0, 2, 1)))
    # a sample of whole scenarios against the oracle: QP data and plans
    S, n = cfg.S, cfg.nV
    sample = np.arange(0, B, max(1, B // 24))
    qs = (sample[:, None] * S + np.arange(S)[None, :]).reshape(-1)
    lin_s, u_s = np.ascontiguousarray(lin[qs]), np.ascontiguousarray(u_old[qs])
    Ho, fo, Go = oracle_qps(cfg, arr, lin_s, u_s)
    for i, q in enumerate(qs):
        sH = np.abs(Ho[i]).max()
        np.testing.assert_allclose(H[q], Ho[i], rtol=0, atol=1e-11 * sH)
        np.testing.assert_allclose(f[q], fo[i], rtol=0, atol=1e-10 * max(np.abs(fo[i]).max(), 1e-6 * sH))
    sub = CmpcDims.from_config(cfg, len(sample))
    odu, ost, *_ = O.step(sub, arr, lin_s, K, u_s.copy(), np.zeros((len(qs), n)),
                          np.zeros(len(qs), np.uint32), init=True)
    np.testing.assert_allclose(du[qs], odu, rtol=1e-9, atol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("plant,ctype,p,B,expect", [("par", "coop", 50, 4096, "rows"),
                                                    ("par", "coop", 100, 4096, "rows"),
                                                    ("par", "cent", 200, 8192, "rows"),
                                                    ("par", "coop", 50, 64, "split"),
                                                    ("par", "cent", 200, 1024, "split"),
                                                    ("ser", "cent", 100, 64, "split"),
                                                    ("ser", "cent", 100, 2048, "wave")])
def test_gpu_build_auto_selects_kernel(plant, ctype, p, B, expect):
    """CMPC_BUILD_AUTO runs the four-QPs-per-wave kernel wherever its LDS fits
    and the batch gives it a wave per SIMD; below that the role-split kernel
    up to one QP per SIMD (SURVEY config 5: cent p = 200, 1 024 QPs), the
    one-QP-per-wave kernel between that and one row group per SIMD;
    DESIGN.md §3.0."""
    _, setup, _, _ = setup_for(plant, ctype)
    cfg = cmpc.reference_config(plant, ctype, p=p)
    arr = cmpc.controller_arrays(cfg, setup)
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=5, n_distinct=min(B, 256))
    with make_ctx(cfg, arr, B, lin, u_old, du_old, ws) as ctx:
        ctx.build()
        got = ctx.last_build_kernel()
    assert got == {"rows": cmpc.CMPC_BUILD_ROWS, "wave": cmpc.CMPC_BUILD_WAVE, "split": cmpc.CMPC_BUILD_SPLIT}[expect]


SPLIT_CASES = [("par", "cent", 200, None), ("par", "coop", 50, None), ("par", "ncoop", 20, None),
               ("ser", "ncoop", 80, None), ("par", "coop", 50, (0, 10, 0, 25)), ("par", "cent", 60, (0, 45, 0, 45)),
               ("ser", "cent", 100, None), ("ser", "coop", 50, None), ("ser", "cent", 40, (0, 4, 0, 9))]


@pytest.mark.gpu
@pytest.mark.parametrize("plant,ctype,p,delays", SPLIT_CASES)
def test_gpu_build_split_equals_wave_bitwise(plant, ctype, p, delays):
    """The role-split build (chain wave + gather wave, one barrier per block,
    z through a two-block ring) gives the one-QP-per-wave kernel's H, f and G
    bit for bit: the same FMAs in the same order per lane."""
    import dataclasses
    _, setup, _, _ = setup_for(plant, ctype)
    cfg = cmpc.reference_config(plant, ctype, p=p)
    if delays is not None:
        cfg = dataclasses.replace(cfg, delays=tuple(delays))
    arr = cmpc.controller_arrays(cfg, setup)
    B = 97
    lin, u_old, du_old, ws = synthetic_batch(cfg, B, seed=41 + p, n_distinct=B)
    out = {}
    with make_ctx(cfg, arr, B, lin, u_old, du_old, ws) as ctx:
        for v in (cmpc.CMPC_BUILD_WAVE, cmpc.CMPC_BUILD_SPLIT):
            ctx.set_build_variant(v)
            ctx.build()
            assert ctx.last_build_kernel() == v
            out[v] = ctx.download_qp()
    for a, b in zip(out[cmpc.CMPC_BUILD_WAVE], out[cmpc.CMPC_BUILD_SPLIT]):
        assert np.array_equal(a, b)
        assert np.isfinite(a).all()


def test_gpu_bound_state_rotation():
    """cmpc_bind_state: one context serving two sets of scenarios in rotation
    (records by cmpc_bind_lin, state by cmpc_bind_state, as bench.py does)
    gives bit for bit what two contexts with their own state give; NULL
    re-binds the context's own, untouched state."""
    import torch
    _, setup, _, _ = setup_for("par", "coop")
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, setup)
    B, K = 512, 9
    sets = [synthetic_batch(cfg, B, seed=4100 + i, n_distinct=128) for i in range(2)]
    # reference: one context per set, each with its own state
    ref = []
    for lin, u, du0, w in sets:
        with make_ctx(cfg, arr, B, lin, u, du0, w) as ctx:
            ctx.build()
            ctx.init_warmstart()
            outs = []
            for _ in range(3):
                ctx.step(K, cmpc.CMPC_APPLY_MOVE)
                outs.append(ctx.download())
            ref.append((outs, ctx.get_state()))
    # one context, the two sets bound in rotation
    dev = "cuda:0"
    lins = [torch.from_numpy(s[0]).to(dev) for s in sets]
    states = [tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                    for a in (s[1], s[2], s[3].view(np.int32))) for s in sets]
    u_own = np.full_like(sets[0][1], 0.25)
    with cmpc.Context(cfg, B) as ctx:
        ctx.configure(arr)
        ctx.set_state(u_own, None, None)

        def bind(i):
            ctx.bind_lin(lins[i].data_ptr())
            ctx.bind_state(*(a.data_ptr() for a in states[i]))

        for i in range(2):
            bind(i)
            ctx.build()
            ctx.init_warmstart()
        got = [[], []]
        for r in range(3):
            for i in range(2):
                bind(i)
                ctx.step(K, cmpc.CMPC_APPLY_MOVE)
                got[i].append(ctx.download())
        for i in range(2):
            for (du, st, nw), (rdu, rst, rnw) in zip(got[i], ref[i][0]):
                assert np.array_equal(du, rdu) and np.array_equal(st, rst) and np.array_equal(nw, rnw)
            ru, rdu_old, rws = ref[i][1]
            u_b, du_b, ws_b = (a.cpu().numpy() for a in states[i])
            assert np.array_equal(u_b, ru) and np.array_equal(du_b, rdu_old)
            assert np.array_equal(ws_b.view(np.uint32), rws)
        assert not np.array_equal(ref[0][1][0], sets[0][1])  # the moves were applied
        ctx.bind_state()
        u_back, _, _ = ctx.get_state()
        assert np.array_equal(u_back, u_own)
        with pytest.raises(RuntimeError):
            ctx.bind_state(states[0][0].data_ptr(), 0, 0)


def test_gpu_timing_stride_samples_every_nth_launch():
    """cmpc_set_timing_stride(n): only every n-th launch of a timed kernel
    carries events (the bench samples its timed builds this way); the
    results do not depend on it; a stride below 1 is refused."""
    _, setup, _, _ = setup_for("par", "coop")
    cfg = cmpc.reference_config("par", "coop", p=20)
    arr = cmpc.controller_arrays(cfg, setup)
    lin, u_old, du_old, ws = synthetic_batch(cfg, 256, seed=3, n_distinct=64)
    with make_ctx(cfg, arr, 256, lin, u_old, du_old, ws) as ctx:
        ctx.build()
        _, _, G0 = ctx.download_qp()
        for stride, launches in ((1, 9), (3, 3), (4, 3), (10, 1)):
            ctx.set_timing_stride(stride)
            ctx.enable_timing(True, only=(cmpc.CMPC_KERNEL_BUILD,))
            for _ in range(9):
                ctx.build()
            ms, n = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD)
            assert n == launches and ms > 0, (stride, n, ms)
        ctx.enable_timing(False)
        ctx.set_timing_stride(1)
        _, _, G1 = ctx.download_qp()
        assert np.array_equal(G0, G1)
        with pytest.raises(RuntimeError):
            ctx.set_timing_stride(0)
