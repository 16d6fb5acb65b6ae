"""Pin the oracle against the reference's own golden records (CPU only).

For each of the six reference configurations, the control input applied at
t = 0 (results/<plant>/run1/<cfg>.dat, record line 3) must be reproduced to
the 6 printed digits by: plant linearisation at the default operating point
-> Taylor-4 discretisation -> GeneratePrediction -> GenerateQP ->
InitializeQPProblem -> n-iterations Jacobi iterations.
Driver assumptions (the reference's common-simulation.inc is missing):
Ts = 0.05, u_offset = GetDefaultInput(), u_init = 0, dx_init = 0,
p_in = p_out = 1 (plant constructor defaults), y_ref replicated over p.
"""
import numpy as np
import pytest

import _oracle as O
import golden_cases as GC
from cmpc._abi import CmpcDims
from cmpc.problem import plant_input_from_plans


@pytest.mark.parametrize("name", GC.NAMES)
def test_plant_output_matches_record(name):
    cfg, setup, arr, g = GC.case(name)
    x0, _ = O.plant_default(cfg.plant)
    np.testing.assert_allclose(x0, g["x0"], rtol=0, atol=0)
    y = O.plant_output(cfg.plant, x0)
    assert [float("%.6g" % v) for v in y] == g["y0"]


@pytest.mark.parametrize("name", GC.NAMES)
def test_oracle_step0_matches_reference(name):
    cfg, setup, arr, g = GC.case(name)
    dims = CmpcDims.from_config(cfg, 1)
    L = O.layout(dims)
    x0, u_full = O.plant_default(cfg.plant)
    y = O.plant_output(cfg.plant, x0)
    lin = GC.step0_records(cfg, dims, L, O.lin_record, x0, u_full, y)
    u_old = np.zeros((cfg.S, cfg.nu_tot))
    du_old = np.zeros((cfg.S, cfg.nV))
    ws = np.zeros(cfg.S, np.uint32)
    du, status, nwsr, _, _ = O.step(dims, arr, lin, g["n_iterations"], u_old, du_old, ws,
                                    init=True)
    assert (status == 0).all()
    u = plant_input_from_plans(cfg, du.reshape(1, cfg.S, cfg.nV))[0]
    GC.assert_six_digits(u, g["u0"])


def test_parallel_recycle_at_lower_bound():
    """Active-set fact of the parallel configs at t=0: both recycle inputs sit
    exactly at their lower bound 0 (setup-*-par constraints-lower ... 0)."""
    for name in ("cent-par", "coop-par", "ncoop-par"):
        cfg, setup, arr, g = GC.case(name)
        dims = CmpcDims.from_config(cfg, 1)
        L = O.layout(dims)
        x0, u_full = O.plant_default(cfg.plant)
        lin = GC.step0_records(cfg, dims, L, O.lin_record, x0, u_full,
                               O.plant_output(cfg.plant, x0))
        du, *_ = O.step(dims, arr, lin, g["n_iterations"], np.zeros((cfg.S, cfg.nu_tot)),
                        np.zeros((cfg.S, cfg.nV)), np.zeros(cfg.S, np.uint32), init=True)
        u = plant_input_from_plans(cfg, du.reshape(1, cfg.S, cfg.nV))[0]
        assert u[1] == 0.0 and u[3] == 0.0


@pytest.mark.parametrize("name", GC.NAMES)
def test_product_reference_setups_match_setup_files(name):
    """cmpc.configs.reference_setup restates setup/setup-<ctrl>-<plant> (fixture)."""
    from cmpc.configs import reference_setup
    cfg, setup, arr, g = GC.case(name)
    ctype, plant = name.split("-")
    mine = reference_setup(plant, ctype)
    assert mine.n_iterations == g["n_iterations"]
    assert mine.yref == g["yref"] and mine.uwt == g["uwt"]
    assert [v for blk in mine.ywt for v in blk][:len(g["ywt"])] == g["ywt"]
    assert mine.constraints_lower == g["constraints_lower"]
    assert mine.constraints_upper == g["constraints_upper"]
    assert mine.rate_lower == g["rate_lower"] and mine.rate_upper == g["rate_upper"]
    assert mine.segments == setup.segments and len(mine.segments) == 2
