"""Small-batch kernels (SURVEY configs 2 and 5, B = 1): the row-layout solve
kernel (one QP per 16-lane DPP row, csrc/solve_rows.hip) against the
one-QP-per-lane kernel, bit for bit, on the same QPs and states: plans,
statuses, working-set change counts, working sets and the change sequence of
every Jacobi iteration, over init + several closed-loop steps with the first
move applied.  (The step-parity tests of test_gpu_parity.py, B = 96, run the
row kernel against the oracle through CMPC_SOLVE_AUTO.)"""
import dataclasses

import numpy as np
import pytest

import cmpc
from cmpc.configs import reference_setup
from cmpc.synthetic import synthetic_batch

pytestmark = pytest.mark.gpu

CASES = [  # plant, controller, p, m, K, B scenarios
    ("par", "coop", 20, 2, 9, 512),
    ("par", "coop", 20, 2, 9, 13),
    ("par", "coop", 50, 2, 9, 4096),
    ("par", "ncoop", 50, 2, 9, 512),
    ("par", "cent", 200, 2, 1, 1024),
    ("ser", "cent", 100, 2, 3, 256),
    ("ser", "coop", 50, 2, 9, 256),
    ("par", "coop", 50, 1, 9, 256),
    ("par", "coop", 30, 3, 9, 256),
]


def _tight(arr, f):
    """Tighter input and rate bounds: more active constraints per QP."""
    return dataclasses.replace(arr, lower=arr.lower * f, upper=arr.upper * f,
                               rate_lower=arr.rate_lower * f, rate_upper=arr.rate_upper * f)


def _run(cfg, arr, lin, u, du, ws, K, variant, steps=3):
    out = []
    with cmpc.Context(cfg, lin.shape[0] // cfg.S) as ctx:
        ctx.configure(arr)
        ctx.set_state(u, du, ws)
        ctx.upload_lin(lin)
        ctx.set_solve_variant(variant)
        for step in range(steps):
            flags = cmpc.CMPC_APPLY_MOVE | cmpc.CMPC_TRACE
            ctx.build()
            if step == 0:
                ctx.init_warmstart()
            ctx.iterate(K, flags)
            assert ctx.last_solve_kernel() == variant
            d, st, nw = ctx.download()
            tr, ntr = ctx.download_trace(K)
            out.append((d, st, nw, *ctx.get_state(), tr, ntr))
    return out


@pytest.mark.parametrize("plant,ctype,p,m,K,B", CASES)
@pytest.mark.parametrize("tight", [1.0, 0.3])
def test_gpu_row_solver_equals_lane_solver(plant, ctype, p, m, K, B, tight):
    cfg = cmpc.reference_config(plant, ctype, p=p, m=m)
    arr = _tight(cmpc.controller_arrays(cfg, reference_setup(plant, ctype)), tight)
    lin, u, du, ws = synthetic_batch(cfg, B, seed=40 + p + m, n_distinct=min(B, 512))
    lane = _run(cfg, arr, lin, u, du, ws, K, cmpc.CMPC_SOLVE_LANE)
    rows = _run(cfg, arr, lin, u, du, ws, K, cmpc.CMPC_SOLVE_ROWS)
    names = ("du", "status", "nwsr", "u_old", "du_old", "ws", "trace", "ntrace")
    for step, (a, b) in enumerate(zip(lane, rows)):
        for name, x, y in zip(names, a, b):
            assert np.array_equal(x, y), (step, name, np.flatnonzero((x != y).reshape(len(x), -1).any(1))[:8])
    st, ntr = lane[-1][1], lane[-1][-1]
    print(f"{plant}-{ctype} p={p} m={m} tight={tight}: ok {np.mean(st == 0):.3f}, "
          f"active {np.mean(lane[-1][5] != 0):.3f}, changes/QP {ntr.sum() / len(st):.3f}")


def test_gpu_row_solver_failure_statuses_equal_lane_solver():
    """Non-finite records (a NaN gradient -> NONFINITE, a NaN Hessian ->
    NOT_PD): the same status and the zero move from both kernels."""
    cfg = cmpc.reference_config("par", "coop", p=20)
    arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
    B = 64
    lin, u, du, ws = synthetic_batch(cfg, B, seed=9, n_distinct=64)
    L = cmpc.layout_of(cmpc.CmpcDims.from_config(cfg, B))
    lin = lin.copy()
    lin[3, L.off_y] = np.nan          # y_prev: f only
    lin[10, L.off_A] = np.nan         # A: H and f
    lin[21, L.off_x + 5] = np.inf     # a delay state: f only
    res = [_run(cfg, arr, lin, u, du, ws, 9, v, steps=2) for v in (cmpc.CMPC_SOLVE_LANE, cmpc.CMPC_SOLVE_ROWS)]
    for a, b in zip(*res):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    st = res[0][-1][1]
    assert st[3] != cmpc.CMPC_QP_OK and st[10] != cmpc.CMPC_QP_OK and st[21] != cmpc.CMPC_QP_OK
    assert (st == cmpc.CMPC_QP_OK).mean() > 0.9


@pytest.mark.parametrize("ctype,B,solve,fused,p", [
    ("cent", 16, cmpc.CMPC_SOLVE_ROWS, False, 20), ("cent", 1024, cmpc.CMPC_SOLVE_ROWS, False, 20),
    ("cent", 1024, cmpc.CMPC_SOLVE_ROWS, True, 50), ("cent", 2048, cmpc.CMPC_SOLVE_ROWS, False, 50),
    ("cent", 65536, cmpc.CMPC_SOLVE_LANE, False, 20),
    ("coop", 1, cmpc.CMPC_SOLVE_ROWS, False, 20), ("coop", 512, cmpc.CMPC_SOLVE_ROWS, False, 20),
    ("coop", 2048, cmpc.CMPC_SOLVE_ROWS, False, 20),   # 4 096 QPs: four per SIMD
    ("coop", 4096, cmpc.CMPC_SOLVE_LANE, False, 20),
    ("coop", 65536, cmpc.CMPC_SOLVE_LANE, False, 20)])
def test_gpu_auto_kernel_selection(ctype, B, solve, fused, p):
    """CMPC_SOLVE_AUTO: the row solve kernel for nV = 8 batches below 16 384
    QPs and nV = 4 batches up to four QPs per SIMD; CMPC_STEP_AUTO: nV = 8
    steps fused from one to four QPs per CU at p >= 50 (the one-QP-per-wave
    kernel with its row solver), every other step the build and the iterate
    kernel (two launches)."""
    cfg = cmpc.reference_config("par", ctype, p=p)
    arr = cmpc.controller_arrays(cfg, reference_setup("par", ctype))
    lin, u, du, ws = synthetic_batch(cfg, B, seed=3, n_distinct=16)
    with cmpc.Context(cfg, B) as ctx:
        ctx.configure(arr)
        ctx.set_state(u, du, ws)
        ctx.upload_lin(lin)
        ctx.build()
        ctx.init_warmstart()
        ctx.iterate(1)
        assert ctx.last_solve_kernel() == solve
        ctx.step(2)
        assert ctx.last_step_fused() == fused
        if fused:  # the fused kernel reports the solver it ran
            assert ctx.last_solve_kernel() == solve


FUSED_CASES = [  # plant, controller, p, K, B scenarios (pinned to the fused kernels; AUTO fuses config 5)
    ("par", "coop", 20, 9, 4096),     # SURVEY config 2: the row build kernel, lane solver
    ("par", "cent", 20, 1, 8192),     # the row build kernel, row solver per group
    ("par", "coop", 20, 9, 13),       # one-QP-per-wave kernel, lane solver of wave 0
    ("par", "coop", 50, 9, 1),        # B = 1, the reference's own call pattern
    ("par", "ncoop", 50, 9, 64),
    ("par", "cent", 200, 1, 1024),    # SURVEY config 5: the one-QP-per-wave kernel
    ("ser", "cent", 100, 1, 1),       # SURVEY config 1 at B = 1
    ("ser", "cent", 100, 3, 512),
    ("ser", "coop", 50, 9, 64),
]


def _run_step(cfg, arr, lin, u, du, ws, K, variant, build=None, steps=3):
    """three steps; returns the per-step results and the build kernel used
    (a split run pins `build`: the two build kernels differ in rounding)"""
    out = []
    with cmpc.Context(cfg, lin.shape[0] // cfg.S) as ctx:
        ctx.configure(arr)
        ctx.set_state(u, du, ws)
        ctx.upload_lin(lin)
        if build is not None:
            ctx.set_build_variant(build)
        ctx.build()
        ctx.init_warmstart()
        ctx.set_step_variant(variant)
        if variant == cmpc.CMPC_STEP_SPLIT:
            ctx.set_solve_variant(cmpc.CMPC_SOLVE_ROWS)
        for step in range(steps):
            ctx.step(K, cmpc.CMPC_APPLY_MOVE | cmpc.CMPC_TRACE)
            assert ctx.last_step_fused() == (variant == cmpc.CMPC_STEP_FUSED)
            kind = ctx.last_build_kernel()
            d, st, nw = ctx.download()
            tr, ntr = ctx.download_trace(K)
            out.append((d, st, nw, *ctx.get_state(), tr, ntr, *ctx.download_qp()))
    return out, kind


@pytest.mark.parametrize("plant,ctype,p,K,B", FUSED_CASES)
def test_gpu_fused_step_equals_split_step(plant, ctype, p, K, B):
    """cmpc_step as one launch (the build kernel solves its own QPs) against
    cmpc_build + cmpc_iterate: the QPs (H, f, G), plans, statuses, working
    sets, states and change sequences of three steps, bit for bit."""
    cfg = cmpc.reference_config(plant, ctype, p=p)
    arr = _tight(cmpc.controller_arrays(cfg, reference_setup(plant, ctype)), 0.5)
    lin, u, du, ws = synthetic_batch(cfg, B, seed=70 + p, n_distinct=min(B, 512))
    fused, kind = _run_step(cfg, arr, lin, u, du, ws, K, cmpc.CMPC_STEP_FUSED)
    split, _ = _run_step(cfg, arr, lin, u, du, ws, K, cmpc.CMPC_STEP_SPLIT, build=kind)
    names = ("du", "status", "nwsr", "u_old", "du_old", "ws", "trace", "ntrace", "H", "f", "G")
    for step, (a, b) in enumerate(zip(split, fused)):
        for name, x, y in zip(names, a, b):
            if x is None:
                continue
            assert np.array_equal(x, y), (step, name)
    print(f"{plant}-{ctype} p={p} B={B}: ok {np.mean(split[-1][1] == 0):.3f}, "
          f"changes/QP {split[-1][7].sum() / len(split[-1][1]):.3f}")


def _oracle_jacobi(cfg, arr, H, f, G, u_old, du_old, ws, K):
    """The Jacobi loop of one step on the device's own (H, f, G) with the
    oracle's map-form solve (or_qp.c step A, version 3): per iteration each
    sub-controller solves with d = the other sub-controllers' previous plans
    in G's column order (controller-major inside each move,
    include/nerve_center.h:283-285)."""
    import _oracle as O
    S, nu, m = cfg.S, cfg.nu, cfg.m
    nV = nu * m
    nqp = H.shape[0]
    dprev = du_old.reshape(nqp, nV).copy()
    ws = ws.copy()
    st = np.zeros(nqp, np.int32); nw = np.zeros(nqp, np.int32)
    tr = np.full((nqp, K, 16), 0xFF, np.uint8); ntr = np.zeros((nqp, K), np.int32)
    for k in range(K):
        dnew = np.zeros_like(dprev)
        for q in range(nqp):
            b, s = divmod(q, S)
            d = np.zeros((S - 1) * nV)
            for rk in range(S - 1):
                s2 = rk + (rk >= s)
                for mv in range(m):
                    d[mv * (S - 1) * nu + rk * nu: mv * (S - 1) * nu + rk * nu + nu] = \
                        dprev[b * S + s2, mv * nu:(mv + 1) * nu]
            lo = np.tile(arr.lower[s] - u_old[q, :nu], m); hi = np.tile(arr.upper[s] - u_old[q, :nu], m)
            rlo = np.tile(arr.rate_lower[s], m); rhi = np.tile(arr.rate_upper[s], m)
            x, info = O.qp_solve_map(H[q], f[q], G[q], d, lo, hi, rlo, rhi, nu, int(ws[q]))
            dnew[q] = x
            ws[q] = info.ws
            st[q] = info.status; nw[q] = info.nchg
            tr[q, k] = np.frombuffer(bytes(info.trace), np.uint8); ntr[q, k] = info.ntrace
        dprev = dnew
    return dprev, st, nw, ws, tr, ntr


JCASES = [  # plant, controller, p, m, K, B scenarios
    ("par", "coop", 20, 2, 9, 96),
    ("par", "ncoop", 50, 2, 9, 48),
    ("ser", "coop", 50, 2, 9, 48),
    ("par", "coop", 30, 3, 9, 48),
    ("par", "cent", 50, 2, 3, 64),
    ("ser", "cent", 100, 2, 3, 48),
]


@pytest.mark.parametrize("plant,ctype,p,m,K,B", JCASES)
@pytest.mark.parametrize("tight", [1.0, 0.3])
@pytest.mark.parametrize("variant", ["lane", "rows"])
def test_gpu_jacobi_map_form_bitexact_vs_oracle(plant, ctype, p, m, K, B, tight, variant):
    """The iterate kernels' Jacobi solves against the oracle's map form on
    the device's own QPs (identical inputs): every iteration's change
    sequence, and the step's plans, statuses, change counts and working
    sets, bit for bit, over three closed-loop steps with the first move
    applied (the map of a working set kept and rebuilt across iterations on
    the device, rebuilt per solve by the oracle)."""
    cfg = cmpc.reference_config(plant, ctype, p=p, m=m)
    arr = _tight(cmpc.controller_arrays(cfg, reference_setup(plant, ctype)), tight)
    lin, u, du, ws = synthetic_batch(cfg, B, seed=70 + p + m, n_distinct=min(B, 512))
    sv = cmpc.CMPC_SOLVE_LANE if variant == "lane" else cmpc.CMPC_SOLVE_ROWS
    changes = 0
    with cmpc.Context(cfg, B) as ctx:
        ctx.configure(arr)
        ctx.set_state(u, du, ws)
        ctx.upload_lin(lin)
        ctx.set_solve_variant(sv)
        for step in range(3):
            ctx.build()
            if step == 0:
                ctx.init_warmstart()
            H, f, G = ctx.download_qp()
            u0, du0, ws0 = (a.copy() for a in ctx.get_state())
            ctx.iterate(K, cmpc.CMPC_APPLY_MOVE | cmpc.CMPC_TRACE)
            assert ctx.last_solve_kernel() == sv
            d, st, nw = ctx.download()
            tr, ntr = ctx.download_trace(K)
            _, _, ws1 = ctx.get_state()
            od, ost, onw, ows, otr, ontr = _oracle_jacobi(cfg, arr, H, f, G, u0, du0, ws0, K)
            assert np.array_equal(ntr, ontr), (step, np.flatnonzero((ntr != ontr).any(1))[:8])
            for q in range(len(st)):
                for k in range(K):
                    n = ntr[q, k]
                    assert np.array_equal(tr[q, k, :n], otr[q, k, :n]), (step, q, k)
            assert np.array_equal(st, ost) and np.array_equal(nw, onw), step
            assert np.array_equal(ws1.view(np.uint32), ows.astype(np.uint32)), step
            assert np.array_equal(d.reshape(od.shape), od), (step, np.abs(d.reshape(od.shape) - od).max())
            changes += int(ntr.sum())
    print(f"{plant}-{ctype} p={p} m={m} tight={tight} {variant}: {changes} working-set changes")
