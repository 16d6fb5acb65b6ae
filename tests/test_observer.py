"""Observer + receding-horizon update.

The reference's observer gain M comes from its missing harness include
(common-simulation.inc), so later closed-loop steps have no recorded output to
compare with.  Parity is therefore pinned three ways:
  CPU  the oracle restatement (oracle/or_observer.c) equals an independent
       dense formulation of the same equations: explicit augmented A, B, C
       matrices built from AComposite / BComposite's definitions
       (libs/aug_lin_sys.cc:27-57, :182-199, :20-21), rtol 1e-12;
  GPU  the product kernels equal the oracle bit for bit on identical inputs
       (same arithmetic order, no contraction); a three-step device-resident
       closed loop (observe, linearise per QP, build, iterate, apply) equals
       the oracle chain to the build's tolerance (du rtol 1e-9);
       all six reference step-0 goldens come out of the observer path
       (at t = 0 the a-posteriori update is the identity).
"""
import dataclasses

import numpy as np
import pytest

import _oracle as O
import cmpc
import golden_cases as GC
from cmpc._abi import CmpcDims
from cmpc.configs import reference_setup

CTRL = [0, 3, 4, 7]  # ControlInputIndex of both plants


def delayed(cfg):
    return [i for i in range(cfg.nu_tot) if cfg.delays[i]]


def dense_prior(cfg, L, rec, du_own, u_old, dx):
    """UpdateU with explicit augmented matrices (independent of or_observer.c)."""
    ns, nut, nobs, ntot = cfg.ns, cfg.nu_tot, L.nobs, L.ntot
    Aorig = rec[L.off_A:L.off_A + ns * ns].reshape(ns, ns)
    Bin = rec[L.off_B:L.off_B + ns * nut].reshape(ns, nut)
    f = rec[L.off_f:L.off_f + ns]
    A = np.zeros((ntot, ntot))
    Bm = np.zeros((ntot, nut))
    A[:ns, :ns] = Aorig
    for i in range(cfg.ndist):
        A[ns + i, ns + i] = 1.0
    blk, k = nobs + L.nd, 0
    for i in range(nut):
        if cfg.delays[i]:
            size = cfg.delays[i] - 1
            A[:ns, nobs + k] = Bin[:, i]          # Adelay column
            A[nobs + k, blk] = 1.0                # slot <- first state of the block
            for j in range(1, size):
                A[blk + j - 1, blk + j] = 1.0     # shift register
            Bm[blk + size - 1, i] = 1.0           # Baug: input enters at the end
            blk += size
            k += 1
        else:
            Bm[:ns, i] = Bin[:, i]
    du = np.zeros(nut)
    du[:cfg.nu] = du_own
    dup = du.copy()
    dxp = dx.copy()
    dxp[:ns] = 0.0
    for k, i in enumerate(delayed(cfg)):
        dup[i] += u_old[i]
        dxp[nobs + k] -= u_old[i]
    new = Bm @ dup + A @ dxp
    new[:ns] += f
    return new, u_old + du


def dense_post(ns, ndist, Cp, M, y, y_old, dx, x_hat):
    n_out = len(y)
    Caug = np.hstack([Cp, np.eye(n_out, ndist)])
    nobs = ns + ndist
    v = (y - y_old) - Caug @ dx[:nobs]
    dx = dx.copy()
    dx[:nobs] += M @ v
    return dx, y.copy(), x_hat + dx[:ns]


def setup(plant, ctype, p, B, seed, xs=0.005, us=0.01, ms=0.05, delays=None):
    cfg = cmpc.reference_config(plant, ctype, p=p)
    if delays is not None:
        cfg = dataclasses.replace(cfg, delays=tuple(delays))
    arr = cmpc.controller_arrays(cfg, reference_setup(plant, ctype))
    dims = CmpcDims.from_config(cfg, B)
    L = cmpc.layout_of(dims)
    rng = np.random.default_rng(seed)
    x0, u0 = O.plant_default(cfg.plant)
    x = x0[None, :] * (1 + xs * rng.normal(size=(B, len(x0))))
    u = np.tile(u0, (B, 1))
    u[:, CTRL] += rng.uniform(-us, us, (B, 4))
    y = np.stack([O.plant_output(cfg.plant, xb) for xb in x])
    n_out = y.shape[1]
    M = [ms * rng.normal(size=(L.nobs, n_out)) for _ in range(cfg.S)]
    return cfg, arr, dims, L, rng, x, u, y, M


# ---- CPU: the oracle against the dense formulation -------------------------

@pytest.mark.parametrize("plant,ctype", [("par", "coop"), ("ser", "cent"), ("par", "ncoop")])
def test_oracle_prior_matches_dense_augmented_system(plant, ctype):
    cfg, _, dims, L, rng, x, u, _, _ = setup(plant, ctype, 20, 4, 1)
    for trial in range(6):
        s = trial % cfg.S
        rec = O.lin_record(cfg, dims, s, x[trial % 4], u[trial % 4])
        dx = rng.normal(0, 0.01, L.ntot)
        u_old = rng.normal(0, 0.05, cfg.nu_tot)
        du_own = rng.normal(0, 0.02, cfg.nu)
        want_dx, want_u = dense_prior(cfg, L, rec, du_own, u_old, dx)
        got_dx, got_u = dx.copy(), u_old.copy()
        O.observe_prior(dims, rec, du_own, got_u, got_dx)
        np.testing.assert_allclose(got_dx, want_dx, rtol=1e-12, atol=1e-15)
        np.testing.assert_array_equal(got_u, want_u)
        # the first delay block's last state took the applied input du + u_old
        i0 = delayed(cfg)[0]
        assert got_dx[L.nobs + L.nd + cfg.delays[i0] - 2] == du_own[i0] + u_old[i0]


@pytest.mark.parametrize("plant", ["par", "ser"])
def test_oracle_post_matches_dense(plant):
    cfg, _, dims, L, rng, x, u, y, M = setup(plant, "coop", 20, 4, 2)
    _, _, Cp, _ = O.plant_linearize(cfg.plant, x[0], u[0])
    for trial in range(5):
        dx = rng.normal(0, 0.01, L.ntot)
        xh = x[trial % 4].copy()
        yo = y[trial % 4] * (1 + 0.01 * rng.normal(size=y.shape[1]))
        want = dense_post(cfg.ns, cfg.ndist, Cp, M[0], y[0], yo, dx, xh)
        O.observe_post(cfg.ns, cfg.ndist, Cp, M[0], y[0], yo, dx, xh)
        np.testing.assert_allclose(dx, want[0], rtol=1e-12, atol=1e-15)
        np.testing.assert_array_equal(yo, want[1])
        np.testing.assert_allclose(xh, want[2], rtol=1e-14)


def test_oracle_post_is_identity_at_step0():
    """dx_init = 0 and y = y_init: the t = 0 update changes nothing (why the
    step-0 goldens do not depend on the unknown M)."""
    cfg, _, dims, L, rng, x, u, y, M = setup("par", "coop", 20, 1, 3)
    _, _, Cp, _ = O.plant_linearize(cfg.plant, x[0], u[0])
    dx, yo, xh = np.zeros(L.ntot), y[0].copy(), x[0].copy()
    O.observe_post(cfg.ns, cfg.ndist, Cp, M[0], y[0], yo, dx, xh)
    assert not dx.any() and np.array_equal(xh, x[0])


# ---- GPU: the product kernels ----------------------------------------------

def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


@pytest.fixture(autouse=True)
def _torch_first(request):
    """GPU tests: torch's HIP runtime comes up before the library's
    (cmpc.Context does this too once torch is imported)."""
    if request.node.get_closest_marker("gpu"):
        import torch
        torch.cuda.init()
    yield


def split(cfg, L, st, n_out=4):
    """An observer row [x_hat ns][dx_aug ntot][y_old n_out][C n_out x ns]
    (+ padding to the row stride)."""
    ns, ntot = cfg.ns, L.ntot
    xh = st[:, :ns]
    dx = st[:, ns:ns + ntot]
    yo = st[:, ns + ntot:ns + ntot + n_out]
    C = st[:, ns + ntot + n_out:ns + ntot + n_out + n_out * ns].reshape(-1, n_out, ns)
    return xh, dx, yo, C


def lin_records(cfg, dims, L, xh, u_full, dx, y):
    """Oracle records, one linearisation per QP slot at its x_hat."""
    S = cfg.S
    recs = np.zeros((len(xh), L.rec_len))
    for q in range(len(xh)):
        b, s = divmod(q, S)
        recs[q] = O.lin_record(cfg, dims, s, xh[q], u_full[b])
        recs[q, L.off_x:L.off_x + L.naug] = dx[q, cfg.ns:]
        recs[q, L.off_y:L.off_y + cfg.ny] = y[b][cfg.out_idx[s]]
    return recs


@pytest.mark.gpu
@pytest.mark.parametrize("plant,ctype,B,delays", [
    ("par", "coop", 96, None), ("ser", "cent", 96, None),
    # B*S not a multiple of the 16 QPs per a-priori workgroup: the tail groups
    ("par", "coop", 37, None), ("ser", "cent", 37, None),
    # longer delay lines (118 and 138 delay-block states; rings of 59 and 69)
    ("par", "coop", 37, (0, 60, 0, 60)), ("par", "coop", 21, (0, 70, 0, 70)),
    # unequal delays: rings of different lengths, a one-entry ring
    ("par", "coop", 37, (0, 2, 0, 25)), ("ser", "coop", 29, (0, 33, 0, 9))])
def test_gpu_observer_kernels_match_oracle(plant, ctype, B, delays):
    cfg, arr, dims, L, rng, x, u, y, M = setup(plant, ctype, 20, B, 5, delays=delays)
    nq = B * cfg.S
    dx0 = rng.normal(0, 1e-3, (nq, L.ntot))
    with cmpc.Context(cfg, B, device=0) as ctx:
        ctx.configure(arr)
        for s in range(cfg.S):
            ctx.set_observer(s, M[s])
        tx, tu, ty, tdx = dev(x), dev(u), dev(y), dev(dx0)
        ctx.observer_init(tx.data_ptr(), tu.data_ptr(), ty.data_ptr(), tdx.data_ptr())
        st0 = ctx.observer_state()
        rec0 = ctx.download_lin()
        xh0, d0, yo0, C0 = split(cfg, L, st0)
        assert np.array_equal(xh0, np.repeat(x, cfg.S, axis=0))
        assert np.array_equal(d0, dx0) and np.array_equal(yo0, np.repeat(y, cfg.S, axis=0))
        for q in range(nq):
            _, _, Cq, _ = O.plant_linearize(cfg.plant, x[q // cfg.S], u[q // cfg.S])
            np.testing.assert_allclose(C0[q], Cq, rtol=1e-11, atol=1e-14)
        np.testing.assert_allclose(rec0, lin_records(cfg, dims, L, xh0, u, d0, y), rtol=1e-11,
                                   atol=1e-14)

        # a posteriori + per-QP linearisation
        y1 = y * (1 + 0.01 * rng.normal(size=y.shape))
        u1 = u.copy()
        u1[:, CTRL] += rng.uniform(-0.005, 0.005, (B, 4))
        ty1, tu1 = dev(y1), dev(u1)
        ctx.observe_step(tu1.data_ptr(), ty1.data_ptr())
        xh1, d1, yo1, C1 = split(cfg, L, ctx.observer_state())
        rec1 = ctx.download_lin()
        for q in range(nq):
            b, s = divmod(q, cfg.S)
            xh, dd, yo = xh0[q].copy(), d0[q].copy(), yo0[q].copy()
            O.observe_post(cfg.ns, cfg.ndist, C0[q], M[s], y1[b], yo, dd, xh)
            assert np.array_equal(xh1[q], xh) and np.array_equal(d1[q], dd), q
            assert np.array_equal(yo1[q], yo)
            _, _, Cq, _ = O.plant_linearize(cfg.plant, xh, u1[b])
            np.testing.assert_allclose(C1[q], Cq, rtol=1e-11, atol=1e-14)
        np.testing.assert_allclose(rec1, lin_records(cfg, dims, L, xh1, u1, d1, y1), rtol=1e-11,
                                   atol=1e-14)

        # a priori + u_old update with arbitrary plans
        u_old = rng.normal(0, 0.05, (nq, cfg.nu_tot))
        du_old = rng.normal(0, 0.02, (nq, cfg.nV))
        ctx.set_state(u_old, du_old, np.zeros(nq, np.uint32))
        ctx.observe_apply()
        xh2, d2, _, _ = split(cfg, L, ctx.observer_state())
        u2, _, _ = ctx.get_state()
        for q in range(nq):
            dd, uo = d1[q].copy(), u_old[q].copy()
            O.observe_prior(dims, rec1[q], du_old[q, :cfg.nu], uo, dd)
            assert np.array_equal(d2[q], dd), q
            assert np.array_equal(u2[q], uo), q
        assert np.array_equal(xh2, xh1)  # x_hat moves only in the a-posteriori step


@pytest.mark.gpu
@pytest.mark.parametrize("delays,steps", [((0, 5, 0, 7), 30), (None, 83)])
def test_gpu_observer_delay_rings_wrap(delays, steps):
    """The delay blocks live on the device as rings rotated by the a-priori
    step count (cmpc_obs_prior_kernel).  Over enough a-priori steps for every
    ring to wrap (block lengths 4 and 6 thirty times; the reference's 39 over
    83 steps) the state equals the oracle's shifted AugmentedState bit for bit
    at every check, the logical rows survive a get/set round trip, and the
    per-QP producer's records after the last step carry the logical tail."""
    B = 21
    cfg, arr, dims, L, rng, x, u, y, M = setup("par", "coop", 20, B, 11, delays=delays)
    nq = B * cfg.S
    dx0 = rng.normal(0, 1e-3, (nq, L.ntot))
    with cmpc.Context(cfg, B, device=0) as ctx:
        ctx.configure(arr)
        for s in range(cfg.S):
            ctx.set_observer(s, M[s])
        tx, tu, ty, tdx = dev(x), dev(u), dev(y), dev(dx0)
        ctx.observer_init(tx.data_ptr(), tu.data_ptr(), ty.data_ptr(), tdx.data_ptr())
        rec = ctx.download_lin()
        d = dx0.copy()
        for t in range(steps):
            u_old = rng.normal(0, 0.05, (nq, cfg.nu_tot))
            du_old = rng.normal(0, 0.02, (nq, cfg.nV))
            ctx.set_state(u_old, du_old, np.zeros(nq, np.uint32))
            ctx.observe_apply()
            for q in range(nq):
                O.observe_prior(dims, rec[q], du_old[q, :cfg.nu], u_old[q].copy(), d[q])
            if t % 7 == 6 or t == steps - 1:
                st = ctx.observer_state()
                _, g_d, _, _ = split(cfg, L, st)
                assert np.array_equal(g_d, d), t
                ctx.set_observer_state(st)  # logical rows in, the same rings out
                assert np.array_equal(ctx.observer_state(), st), t
        ctx.observe_step(tu.data_ptr(), ty.data_ptr())
        xh1, d1, _, _ = split(cfg, L, ctx.observer_state())
        np.testing.assert_allclose(ctx.download_lin(), lin_records(cfg, dims, L, xh1, u, d1, y),
                                   rtol=1e-11, atol=1e-14)


@pytest.mark.gpu
def test_gpu_closed_loop_observer_matches_oracle():
    """Three device-resident control steps (observe -> linearise per QP ->
    build -> K iterations -> apply) against the oracle chain.  Operating
    points close to the default equilibrium and a small gain keep x_hat where
    the K = 9 Jacobi iteration is well conditioned.  (At 0.5 % state
    perturbations and M ~ 0.05, step 1 had records and u_old equal to 1e-10
    but plans differing by 1e-4 on a few QPs: the iteration amplifies the
    build's rounding differences there.)"""
    B, K, steps = 24, 9, 3
    cfg, arr, dims, L, rng, x, u, y, M = setup("par", "coop", 20, B, 8, xs=1e-4, us=1e-3, ms=0.01)
    nq, S = B * cfg.S, cfg.S
    ys = [y] + [y * (1 + 3e-4 * rng.normal(size=y.shape)) for _ in range(steps - 1)]
    # oracle state
    xh = np.repeat(x, S, axis=0)
    dx = np.zeros((nq, L.ntot))
    yo = np.repeat(y, S, axis=0)
    u_old = np.zeros((nq, cfg.nu_tot))
    du_old = np.zeros((nq, cfg.nV))
    ws = np.zeros(nq, np.uint32)
    Cprev = np.stack([O.plant_linearize(cfg.plant, xh[q], u[q // S])[2] for q in range(nq)])
    o_du, o_rec, o_u, o_dx = [], [], [], []
    for t in range(steps):
        if t > 0:
            for q in range(nq):
                b, s = divmod(q, S)
                O.observe_post(cfg.ns, cfg.ndist, Cprev[q], M[s], ys[t][b], yo[q], dx[q], xh[q])
            Cprev = np.stack([O.plant_linearize(cfg.plant, xh[q], u[q // S])[2] for q in range(nq)])
        recs = lin_records(cfg, dims, L, xh, u, dx, ys[t])
        o_rec.append(recs)
        o_u.append(u_old.copy())
        du, st, *_ = O.step(dims, arr, recs, K, u_old, du_old, ws, init=(t == 0))
        for q in range(nq):
            O.observe_prior(dims, recs[q], du[q, :cfg.nu], u_old[q], dx[q])
        o_du.append((du.copy(), st.copy()))
    # product
    with cmpc.Context(cfg, B, device=0) as ctx:
        ctx.configure(arr)
        ctx.set_state(np.zeros((nq, cfg.nu_tot)), np.zeros((nq, cfg.nV)), np.zeros(nq, np.uint32))
        for s in range(S):
            ctx.set_observer(s, M[s])
        tx, tu = dev(x), dev(u)
        tys = [dev(a) for a in ys]
        ctx.observer_init(tx.data_ptr(), tu.data_ptr(), tys[0].data_ptr())
        for t in range(steps):
            if t > 0:
                ctx.observe_step(tu.data_ptr(), tys[t].data_ptr())
            # the step's inputs first: records (linearisation per QP at x_hat,
            # observer tail, y) and u_old
            np.testing.assert_allclose(ctx.download_lin(), o_rec[t], rtol=1e-10, atol=1e-13,
                                       err_msg=f"records, step {t}")
            np.testing.assert_allclose(ctx.get_state()[0], o_u[t], rtol=1e-10, atol=1e-13,
                                       err_msg=f"u_old, step {t}")
            ctx.build()
            if t == 0:
                ctx.init_warmstart()
            ctx.iterate(K)
            g_du, g_st, _ = ctx.download()
            ctx.observe_apply()
            assert np.array_equal(g_st, o_du[t][1]), t
            np.testing.assert_allclose(g_du, o_du[t][0], rtol=1e-9, atol=1e-10,
                                       err_msg=f"plans, step {t}")
        g_xh, g_dx, _, _ = split(cfg, L, ctx.observer_state())
        g_u, _, _ = ctx.get_state()
    np.testing.assert_allclose(g_xh, xh, rtol=1e-12)
    np.testing.assert_allclose(g_dx, dx, rtol=1e-8, atol=1e-11)
    np.testing.assert_allclose(g_u, u_old, rtol=1e-9, atol=1e-11)


@pytest.mark.gpu
@pytest.mark.parametrize("plant,ctype,p,B,K", [
    ("par", "coop", 50, 1, 9),     # B = 1, the reference's own call pattern
    ("par", "coop", 20, 13, 9),    # a partial last workgroup
    ("par", "ncoop", 50, 3, 9),
    ("par", "cent", 20, 5, 3),     # row solver of each wave
    ("par", "cent", 20, 3, 3),     # one workgroup, waves 1-2 store results (polled path)
    ("ser", "cent", 100, 4, 1),    # one workgroup, waves 1-3 store results (polled path)
    ("ser", "cent", 100, 1, 1),    # SURVEY config 1 at B = 1
    ("ser", "coop", 50, 2, 9)])
def test_gpu_control_step_equals_three_calls(plant, ctype, p, B, K):
    """cmpc_control_step (NerveCenter::GetNextInput as one kernel: a
    posteriori + linearisation, build, K Jacobi iterations, a priori) against
    cmpc_observe_step + cmpc_step(K, 0) + cmpc_observe_apply on the same
    state over four steps: plans, statuses, nWSR, records, QPs, observer rows
    and controller state bit for bit, and the one launch did run."""
    # operating points near the equilibrium and a small gain (as the closed-loop
    # test above): the estimate stays where the linearisation is finite
    cfg, arr, dims, L, rng, x, u, y, M = setup(plant, ctype, p, B, 17, xs=1e-4, us=1e-3, ms=0.01)
    nq = B * cfg.S
    ys = [y * (1 + 3e-4 * rng.normal(size=y.shape)) for _ in range(4)]
    out = []
    for one in (False, True, "poll"):
        with cmpc.Context(cfg, B, device=0) as ctx:
            ctx.configure(arr)
            ctx.set_state(np.zeros((nq, cfg.nu_tot)), np.zeros((nq, cfg.nV)), np.zeros(nq, np.uint32))
            for s_ in range(cfg.S):
                ctx.set_observer(s_, M[s_])
            tx, tu = dev(x), dev(u)
            tys = [dev(a) for a in ys]
            ctx.observer_init(tx.data_ptr(), tu.data_ptr(), dev(y).data_ptr())
            ctx.build()
            ctx.init_warmstart()
            res = []
            for t in range(4):
                if one == "poll":  # host arrays in, results back in one call
                    polled = ctx.control_step_download(u, ys[t], K)
                    assert ctx.last_step_fused() == 1
                    assert all(np.array_equal(a, b) for a, b in zip(polled, ctx.download()))
                elif one:
                    ctx.control_step(tu.data_ptr(), tys[t].data_ptr(), K)
                    assert ctx.last_step_fused() == 1
                else:
                    ctx.observe_step(tu.data_ptr(), tys[t].data_ptr())
                    ctx.step(K, 0)
                    ctx.observe_apply()
                res.append((*ctx.download(), ctx.download_lin(), *ctx.download_qp(), ctx.observer_state(),
                            *ctx.get_state()))
            out.append(res)
    for other in out[1:]:
        for t, (a, b) in enumerate(zip(out[0], other)):
            for i, (va, vb) in enumerate(zip(a, b)):
                if va is None:
                    continue
                assert np.array_equal(va, vb, equal_nan=True), (t, i)
    assert np.isfinite(out[1][-1][3]).all() and (out[1][-1][1] == 0).mean() > 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("plant,ctype,p,B,K", [
    ("par", "coop", 50, 1, 9),     # the reference's own call pattern (polled)
    ("ser", "cent", 100, 1, 1),    # SURVEY config 1 at B = 1 (polled)
    ("par", "coop", 20, 3, 9)])    # two workgroups: the stream-synchronised path
def test_gpu_polled_control_steps_back_to_back(plant, ctype, p, B, K):
    """cmpc_control_step_download called back to back with a new y every call
    and nothing else in between: the polled call frees the page-locked
    staging buffer of its inputs once the kernel's done word is seen (no
    event), so the next call's inputs may overwrite it at once.  Every call's
    plans, statuses and nWSR equal the three-call path's bit for bit."""
    cfg, arr, dims, L, rng, x, u, y, M = setup(plant, ctype, p, B, 23, xs=1e-4, us=1e-3, ms=0.01)
    nq = B * cfg.S
    T = 24
    ys = [y * (1 + 3e-4 * rng.normal(size=y.shape)) for _ in range(T)]
    out = []
    for polled in (False, True):
        with cmpc.Context(cfg, B, device=0) as ctx:
            ctx.configure(arr)
            ctx.set_state(np.zeros((nq, cfg.nu_tot)), np.zeros((nq, cfg.nV)), np.zeros(nq, np.uint32))
            for s_ in range(cfg.S):
                ctx.set_observer(s_, M[s_])
            tx, tu = dev(x), dev(u)
            ctx.observer_init(tx.data_ptr(), tu.data_ptr(), dev(y).data_ptr())
            ctx.build()
            ctx.init_warmstart()
            res = []
            if polled:
                for t in range(T):
                    res.append(tuple(np.array(a, copy=True) for a in ctx.control_step_download(u, ys[t], K)))
                    assert ctx.last_step_fused() == 1
            else:
                tys = [dev(a) for a in ys]
                for t in range(T):
                    ctx.observe_step(tu.data_ptr(), tys[t].data_ptr())
                    ctx.step(K, 0)
                    ctx.observe_apply()
                    res.append(ctx.download())
            out.append(res)
    for t, (a, b) in enumerate(zip(*out)):
        for i, (va, vb) in enumerate(zip(a, b)):
            assert np.array_equal(va, vb), (t, i)
    assert any(not np.array_equal(out[1][t][0], out[1][t + 1][0]) for t in range(T - 1))


@pytest.mark.gpu
@pytest.mark.parametrize("name", GC.NAMES)
def test_gpu_step0_golden_through_observer(name):
    """Initialize + GenerateInitialQP through the observer path reproduce the
    reference's recorded u(t = 0) (the update is the identity at t = 0, so M
    is arbitrary here)."""
    cfg, setup_, arr, g = GC.case(name)
    x0, u_full = cmpc.plant_default(cfg.plant)
    y0 = cmpc.plant_output(cfg.plant, x0)
    n_out = len(y0)
    L = cmpc.layout_of(CmpcDims.from_config(cfg, 1))
    with cmpc.Context(cfg, 1, device=0) as ctx:
        ctx.configure(arr)
        ctx.set_state(np.zeros((cfg.S, cfg.nu_tot)), np.zeros((cfg.S, cfg.nV)),
                      np.zeros(cfg.S, np.uint32))
        for s in range(cfg.S):
            ctx.set_observer(s, np.full((L.nobs, n_out), 0.3))
        tx, tu, ty = dev(x0[None]), dev(u_full[None]), dev(y0[None])
        ctx.observer_init(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
        ctx.observe_step(tu.data_ptr(), ty.data_ptr())
        ctx.build()
        ctx.init_warmstart()
        ctx.iterate(g["n_iterations"])
        du, status, _ = ctx.download()
    assert (status == 0).all()
    u = cmpc.plant_input_from_plans(cfg, du.reshape(1, cfg.S, cfg.nV))[0]
    GC.assert_six_digits(u, g["u0"])
