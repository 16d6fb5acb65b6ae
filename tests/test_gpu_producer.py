"""Device record producer (cmpc_produce_lin) against the
host producer (cmpc_plant_lin_record, itself checked against the oracle's
plant in test_abi.py): the plant linearisation, Taylor-4 discretisation and
record assembly on the GPU give the host's records, and a control step on
them gives the host-record step's plans.

Same source (plant_model.h) and -ffp-contract=off on both sides, so the
records agree to the last bit except where the recycle-valve dead-zone uses
exp() (libm vs OCML, < 1 ulp): tolerance 1e-13 relative there."""
import numpy as np
import pytest

import cmpc
from cmpc._abi import CmpcDims
from cmpc.configs import reference_setup

CASES = [("par", "coop"), ("par", "ncoop"), ("par", "cent"), ("ser", "ncoop"), ("ser", "coop"),
         ("ser", "cent")]
CTRL = [0, 3, 4, 7]  # ControlInputIndex of both plants


def operating_points(cfg, B, seed):
    rng = np.random.default_rng(seed)
    x0, u0 = cmpc.plant_default(cfg.plant)
    x = x0[None, :] * (1 + 0.01 * rng.normal(size=(B, len(x0))))
    u = np.tile(u0, (B, 1))
    u[:, CTRL] += rng.uniform(-0.02, 0.02, (B, 4))
    u[:, [3, 7]] = np.where(rng.uniform(size=(B, 2)) < 0.3, 0.0, np.abs(u[:, [3, 7]]) + 0.03)
    y = np.stack([cmpc.plant_output(cfg.plant, xb) for xb in x])
    return x, u, y


@pytest.mark.gpu
@pytest.mark.parametrize("plant,ctype", CASES)
def test_gpu_producer_matches_host(plant, ctype):
    import torch
    cfg = cmpc.reference_config(plant, ctype, p=50)
    B = 257
    x, u, y = operating_points(cfg, B, seed=9)
    dims = CmpcDims.from_config(cfg, B)
    L = cmpc.layout_of(dims)
    rng = np.random.default_rng(4)
    dx = rng.normal(0, 1e-3, (B * cfg.S, L.naug))
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")
    tx, tu, ty, tdx = dev(x), dev(u), dev(y), dev(dx)
    with cmpc.Context(cfg, B, device=0) as ctx:
        ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr(), tdx.data_ptr())
        got = ctx.download_lin()
    exact = 0
    for b in range(B):
        for s in range(cfg.S):
            q = b * cfg.S + s
            ref = np.zeros(L.rec_len)
            cmpc.plant_lin_record(cfg, dims, s, x[b], u[b], out=ref)
            ref[L.off_x:L.off_x + L.naug] = dx[q]
            ref[L.off_y:L.off_y + cfg.ny] = y[b][cfg.out_idx[s]]
            if np.array_equal(got[q], ref):
                exact += 1
            else:
                np.testing.assert_allclose(got[q], ref, rtol=1e-13, atol=1e-300)
    assert exact >= 0.5 * B * cfg.S, exact


@pytest.mark.gpu
def test_gpu_step_on_produced_records():
    """produce -> build -> InitializeQPProblem -> 9 Jacobi iterations equals
    the same step on host-produced, uploaded records."""
    import torch
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
    B = 1024
    x, u, y = operating_points(cfg, B, seed=21)
    dims = CmpcDims.from_config(cfg, B)
    L = cmpc.layout_of(dims)
    recs = np.zeros((B * cfg.S, L.rec_len))
    for b in range(B):
        for s in range(cfg.S):
            cmpc.plant_lin_record(cfg, dims, s, x[b], u[b], out=recs[b * cfg.S + s])
            recs[b * cfg.S + s, L.off_y:L.off_y + cfg.ny] = y[b][cfg.out_idx[s]]
    z = lambda *sh: np.zeros(sh)

    def run(fill):
        with cmpc.Context(cfg, B, device=0) as ctx:
            ctx.configure(arr)
            ctx.set_state(z(B * cfg.S, cfg.nu_tot), z(B * cfg.S, cfg.nV), np.zeros(B * cfg.S, np.uint32))
            fill(ctx)
            ctx.build()
            ctx.init_warmstart()
            ctx.iterate(9)
            return ctx.download()

    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")
    tx, tu, ty = dev(x), dev(u), dev(y)
    du_d, st_d, _ = run(lambda c: c.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr()))
    du_h, st_h, _ = run(lambda c: c.upload_lin(recs))
    assert np.array_equal(st_d, st_h)
    np.testing.assert_allclose(du_d, du_h, rtol=1e-10, atol=1e-13)


@pytest.mark.gpu
def test_gpu_producer_strided_batch():
    """A batch of several rounds of resident workgroups with a partial last
    group: every record is written (its controlled-output tail is the
    scenario's y, copied exactly) and sampled records, the last ones among
    them, equal the host producer's."""
    import torch
    cfg = cmpc.reference_config("par", "coop", p=50)
    B = 40_003  # 10 001 groups of four scenarios, the last one partial
    x, u, y = operating_points(cfg, B, seed=13)
    dims = CmpcDims.from_config(cfg, B)
    L = cmpc.layout_of(dims)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")
    tx, tu, ty = dev(x), dev(u), dev(y)
    with cmpc.Context(cfg, B, device=0) as ctx:
        ctx.upload_lin(np.full((B * cfg.S, L.rec_len), np.nan))
        ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
        got = ctx.download_lin()
    assert np.isfinite(got).all()
    for s in range(cfg.S):
        np.testing.assert_array_equal(got[s::cfg.S, L.off_y:L.off_y + cfg.ny], y[:, cfg.out_idx[s]])
    rng = np.random.default_rng(5)
    sample = np.concatenate([rng.choice(B, 200, replace=False), np.arange(B - 9, B)])
    for b in sample:
        for s in range(cfg.S):
            ref = np.zeros(L.rec_len)
            cmpc.plant_lin_record(cfg, dims, s, x[b], u[b], out=ref)
            ref[L.off_y:L.off_y + cfg.ny] = y[b][cfg.out_idx[s]]
            np.testing.assert_allclose(got[b * cfg.S + s], ref, rtol=1e-13, atol=1e-300)
