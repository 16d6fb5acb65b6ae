"""Plant simulation: the reference harness's
SimulationSystem — controlled Dormand-Prince (Boost odeint semantics, the
reference's 2-norm error), TimeDelay, GetPlantInput — restated in the oracle
(oracle/or_sim.c) and on the GPU (sim.hip).

Pinned by the reference's own recorded closed-loop trajectories
(tests/golden/traj_*.json from results/<plant>/run1/<cfg>.dat, made by
tests/golden/make_traj_golden.py): driven by the recorded controller outputs
u(t_k), the simulated plant state x(t_k+1) and output y(t_k+1) equal the
recorded ones to all 6 printed digits (string equality of %.6g), for 159
sampling intervals (8 s, past the 2 s input-delay onset).  This pin does not
depend on the missing observer gain: the plant sees only the inputs.
"""
import json
import os

import numpy as np
import pytest

import _oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
TRAJ = ["par_centralized", "par_coop9", "par_ncoop9", "ser_centralized", "ser_coop9", "ser_ncoop9"]
TS = 0.05


def load(name):
    return json.load(open(os.path.join(HERE, "golden", f"traj_{name}.json")))["records"]


def six(a):
    return [float("%.6g" % v) for v in a]


def assert_printed_equal(got, want, what):
    g = six(got)
    assert g == [float(w) for w in want], (what, got, want)


@pytest.mark.parametrize("name", TRAJ)
def test_oracle_sim_reproduces_recorded_trajectory(name):
    recs = load(name)
    plant = 0 if name.startswith("par") else 1
    x0, u0 = O.plant_default(plant)
    assert_printed_equal(x0, recs[0]["x"], "x(0)")
    sim = O.PlantSim(plant, x0, u0)
    for k in range(len(recs) - 1):
        sim.set_input(recs[k]["u"])
        t = 0.0 + k * TS                       # integrate_const: t0 + step * dt
        sim.integrate(t, t + TS)
        assert_printed_equal(sim.x, recs[k + 1]["x"], f"x at step {k + 1}")
        assert_printed_equal(O.plant_output(plant, sim.x), recs[k + 1]["y"], f"y at step {k + 1}")


def test_oracle_time_delay_ring():
    """TimeDelay: a delayed input comes out D samples later; others pass."""
    delays = np.array([0, 3, 0, 2], np.int32)
    ring = np.zeros(5)
    cur = np.zeros(4, np.int32)
    L = O._sim_sigs()
    L.or_time_delay_init(4, O.iptr(delays), O.dptr(ring), O.iptr(cur))
    outs = []
    for k in range(8):
        u = np.array([k, 10 + k, 20 + k, 30 + k], dtype=float)
        out = np.zeros(4)
        L.or_time_delay(4, O.iptr(delays), O.dptr(ring), O.iptr(cur), O.dptr(u), O.dptr(out))
        outs.append(out.copy())
    outs = np.array(outs)
    assert np.array_equal(outs[:, 0], np.arange(8)) and np.array_equal(outs[:, 2], 20 + np.arange(8))
    assert np.array_equal(outs[:, 1], [0, 0, 0, 10, 11, 12, 13, 14])
    assert np.array_equal(outs[:, 3], [0, 0, 30, 31, 32, 33, 34, 35])


def _unstable_serial():
    """Serial plant with its input 6 stepped by -0.3 (0.393 -> 0.093), no
    control: the step size collapses within 10 intervals."""
    x0, u0 = O.plant_default(1)
    u = u0.copy()
    u[6] -= 0.3
    return x0, u


def test_oracle_sim_step_bound():
    """odeint's max_step_checker: more than 500 steps between two observer
    calls end the interval (or_sim_interval returns -2) instead of looping
    while the step size collapses."""
    x0, u = _unstable_serial()
    sim = O.PlantSim(1, x0, u)
    rcs = []
    for k in range(12):
        sim.set_input(np.zeros(4))
        rcs.append(sim.L.or_sim_interval(1, 1.0, 1.0, O.dptr(sim.u_full), O.dptr(sim.x), k * TS,
                                         k * TS + TS, O.dptr(sim.dt), 1e-6, 1e-6))
    assert all(0 < r <= 500 for r in rcs[:10]) and rcs[10] == -2, rcs


# ---- GPU ----------------------------------------------------------------------

@pytest.fixture(autouse=True)
def _torch_first(request):
    if request.node.get_closest_marker("gpu"):
        import torch
        torch.cuda.init()
    yield


@pytest.mark.gpu
@pytest.mark.parametrize("plant", [0, 1])
def test_gpu_sim_reproduces_recorded_trajectories(plant):
    """The three recorded trajectories of a plant as one batch of B = 3."""
    import torch
    from cmpc.sim import PlantSimulator
    names = [n for n in TRAJ if n.startswith("par" if plant == 0 else "ser")]
    recs = [load(n) for n in names]
    x0, u0 = O.plant_default(plant)
    B = len(names)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    with PlantSimulator(plant, B) as sim:
        sim.reset(dev(np.tile(x0, (B, 1))), dev(np.tile(u0, (B, 1))), TS)
        for k in range(len(recs[0]) - 1):
            u = dev([r[k]["u"] for r in recs])
            sim.set_input(u)
            t = 0.0 + k * TS
            sim.integrate(t, t + TS)
            y = sim.output().cpu().numpy()
            x, _, _, st = sim.download()
            assert not st.any()
            for j in range(B):
                assert_printed_equal(x[j], recs[j][k + 1]["x"], (names[j], k + 1))
                assert_printed_equal(y[j], recs[j][k + 1]["y"], (names[j], k + 1))


@pytest.mark.gpu
@pytest.mark.parametrize("plant", [0, 1])
def test_gpu_sim_matches_oracle(plant):
    """Perturbed states and random inputs, 30 intervals: states, plant
    inputs and carried step sizes against the oracle simulator."""
    import torch
    from cmpc.sim import PlantSimulator
    B, steps = 96, 30
    rng = np.random.default_rng(3 + plant)
    x0, u0 = O.plant_default(plant)
    xs = x0[None, :] * (1 + 0.002 * rng.normal(size=(B, len(x0))))
    us = np.tile(u0, (B, 1))
    ucs = rng.uniform(-0.01, 0.01, (steps, B, 4))
    ucs[:, :, [1, 3]] = np.abs(ucs[:, :, [1, 3]])
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    sims = [O.PlantSim(plant, xs[b], us[b]) for b in range(B)]
    with PlantSimulator(plant, B) as sim:
        sim.reset(dev(xs), dev(us), TS)
        for k in range(steps):
            sim.set_input(dev(ucs[k]))
            sim.integrate(k * TS, k * TS + TS)
            for b in range(B):
                sims[b].set_input(ucs[k, b])
                sims[b].integrate(k * TS, k * TS + TS)
        x, uf, dt, st = sim.download()
    assert not st.any()
    ox = np.stack([s.x for s in sims])
    np.testing.assert_array_equal(uf, np.stack([s.u_full for s in sims]))
    np.testing.assert_allclose(x, ox, rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(dt, np.array([s.dt[0] for s in sims]), rtol=1e-10)


@pytest.mark.gpu
def test_gpu_sim_step_bound():
    """The device integrator stops a scenario whose step size collapses after
    500 steps in the interval (status 2), like the oracle, and its neighbour
    in the batch is unaffected (status 0, state equal to the oracle's)."""
    import torch
    from cmpc.sim import PlantSimulator
    x0, u_bad = _unstable_serial()
    _, u0 = O.plant_default(1)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    good = O.PlantSim(1, x0, u0)
    with PlantSimulator(1, 2) as sim:
        sim.reset(dev(np.stack([x0, x0])), dev(np.stack([u0, u_bad])), TS)
        for k in range(11):
            sim.set_input(dev(np.zeros((2, 4))))
            sim.integrate(k * TS, k * TS + TS)
            good.set_input(np.zeros(4))
            good.integrate(k * TS, k * TS + TS)
            x, _, _, st = sim.download()
            assert st[0] == 0 and st[1] == (2 if k == 10 else 0), (k, st)
        np.testing.assert_allclose(x[0], good.x, rtol=1e-12)
        # sticky: a later interval — clean or not — neither clears
        # status 2 nor moves the failed scenario on from where it stopped
        x_stop = x[1].copy()
        for k in range(11, 14):
            sim.set_input(dev(np.zeros((2, 4))))
            sim.integrate(k * TS, k * TS + TS)
            good.set_input(np.zeros(4))
            good.integrate(k * TS, k * TS + TS)
        x, _, _, st = sim.download()
        assert st[0] == 0 and st[1] == 2, st
        np.testing.assert_array_equal(x[1], x_stop)
        np.testing.assert_allclose(x[0], good.x, rtol=1e-12)
        # a non-finite state fails with status 3 instead of passing as 0
        xn = np.stack([x0, x0])
        xn[1, 2] = np.nan
        sim.reset(dev(xn), dev(np.stack([u0, u0])), TS)
        x, _, _, st = sim.download()
        assert not st.any(), st                    # reset clears the sticky status
        sim.set_input(dev(np.zeros((2, 4))))
        sim.integrate(0.0, TS)
        x, _, _, st = sim.download()
        assert st[0] == 0 and st[1] == 3, st


# ---- the closed-loop driver (cmpc/driver.py) -----------------------------------

def test_dat_writer_matches_reference_format():
    """The 6-line record text (Eigen's aligned columns, 6 significant digits)
    equals the reference's own first records, byte for byte, given their values."""
    import io
    from cmpc.driver import DatWriter
    for name in TRAJ:
        d = json.load(open(os.path.join(HERE, "golden", f"traj_{name}.json")))
        raw = d["raw_first_records"]
        buf = io.StringIO()
        w = DatWriter(buf)
        for r, ns in zip(d["records"][:2], (int(raw[4]), int(raw[10]))):
            w.record(r["t"], r["x"], r["u"], r["y"], ns)
        assert buf.getvalue().split("\n")[:12] == raw, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cent-par", "coop-par", "ncoop-par", "cent-ser", "coop-ser", "ncoop-ser"])
def test_gpu_closed_loop_driver_first_records(name):
    """Two sampling instants of the device closed loop (plant simulation,
    observer, QP build, Jacobi iterations, delay line) for a batch of 4
    identical scenarios: record 0 (u(0), y(0)) and record 1 (x(0.05),
    y(0.05)) equal the reference's results to 6 digits (both are independent
    of the missing observer gain: record 1's state depends only on u(0))."""
    import cmpc
    import golden_cases as GC
    from cmpc.driver import ClosedLoop
    cfg, setup, arr, g = GC.case(name)
    ctype, plant = name.split("-")
    traj = load(f"{plant}_{'centralized' if ctype == 'cent' else ctype + '9'}")
    x0, u0 = cmpc.plant_default(cfg.plant)
    B = 4
    from cmpc._abi import CmpcDims
    L = cmpc.layout_of(CmpcDims.from_config(cfg, 1))
    M = [np.full((L.nobs, 4), 0.1) for _ in range(cfg.S)]   # arbitrary: no effect on these records
    loop = ClosedLoop(cfg, arr, M, np.tile(x0, (B, 1)), np.tile(u0, (B, 1)), g["n_iterations"])
    try:
        loop.initialize()
        t, y = loop.step()
        u = loop.u_ctrl.cpu().numpy()
        for b in range(B):
            GC.assert_six_digits(u[b], g["u0"])
            assert_printed_equal(y.cpu().numpy()[b], traj[0]["y"], "y(0)")
        x1, _, _, st = loop.sim.download()
        assert not st.any()
        t, y1 = loop.step()
        for b in range(B):
            assert_printed_equal(x1[b], traj[1]["x"], "x(0.05)")
            assert_printed_equal(y1.cpu().numpy()[b], traj[1]["y"], "y(0.05)")
    finally:
        loop.close()
