"""The host-array entry points (cmpc_observer_init_host, cmpc_observe_step_host,
cmpc_download, cmpc_sim_*_host, cmpc_sim_download) stage through page-locked
memory with one DMA per call.  They must give bit for bit what the device-
pointer entry points give, for odd batch sizes (array padding inside the
staging block) and over repeated calls (the staging buffer is reused once its
previous copy is done)."""
import numpy as np
import pytest

import cmpc
from cmpc._abi import dptr, iptr
from cmpc.configs import reference_setup


@pytest.fixture(autouse=True)
def _torch_first(request):
    if request.node.get_closest_marker("gpu"):
        import torch
        torch.cuda.init()
    yield


def _inputs(cfg, B, rng):
    x0, u0 = cmpc.plant_default(cfg.plant)
    x = x0[None, :] * (1 + 1e-3 * rng.normal(size=(B, len(x0))))
    u = np.tile(u0, (B, 1))
    u[:, [0, 3, 4, 7]] += rng.uniform(-0.005, 0.005, (B, 4))
    y = np.stack([cmpc.plant_output(cfg.plant, xb) for xb in x])
    return x, u, y


@pytest.mark.gpu
@pytest.mark.parametrize("plant,ctype,B", [("par", "coop", 37), ("ser", "cent", 5), ("par", "ncoop", 1)])
def test_gpu_host_entry_points_match_device_ones(plant, ctype, B):
    import torch
    cfg = cmpc.reference_config(plant, ctype, p=20)
    arr = cmpc.controller_arrays(cfg, reference_setup(plant, ctype))
    rng = np.random.default_rng(17)
    x, u, y = _inputs(cfg, B, rng)
    nq = B * cfg.S
    M = cmpc.reference_observer_gain(cfg)
    io = np.ascontiguousarray(cfg.input_order, dtype=np.int32)
    oi = np.ascontiguousarray(cfg.out_idx, dtype=np.int32)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    with cmpc.Context(cfg, B, device=0) as cd, cmpc.Context(cfg, B, device=0) as ch:
        for c in (cd, ch):
            c.configure(arr)
            c.set_state(np.zeros((nq, cfg.nu_tot)), np.zeros((nq, cfg.nV)), np.zeros(nq, np.uint32))
            for s in range(cfg.S):
                c.set_observer(s, M)
        dx0 = rng.normal(0, 1e-4, (nq, cd.layout.ntot))
        tx, tu, ty, tdx = dev(x), dev(u), dev(y), dev(dx0)
        cd.observer_init(tx.data_ptr(), tu.data_ptr(), ty.data_ptr(), tdx.data_ptr())
        assert ch.lib.cmpc_observer_init_host(ch._h, cfg.plant, 1.0, 1.0, 0.05, iptr(io), iptr(oi),
                                              dptr(np.ascontiguousarray(x)), dptr(np.ascontiguousarray(u)),
                                              dptr(np.ascontiguousarray(y)), dptr(dx0)) == 0
        assert np.array_equal(cd.observer_state(), ch.observer_state())
        assert np.array_equal(cd.download_lin(), ch.download_lin())
        for c in (cd, ch):
            c.build()
            c.init_warmstart()
        for t in range(4):
            y_t = np.ascontiguousarray(y * (1 + 1e-4 * rng.normal(size=y.shape)))
            u_t = np.ascontiguousarray(u)
            ty_t, tu_t = dev(y_t), dev(u_t)
            cd.observe_step(tu_t.data_ptr(), ty_t.data_ptr())
            assert ch.lib.cmpc_observe_step_host(ch._h, dptr(u_t), dptr(y_t)) == 0
            for c in (cd, ch):
                c.build()
                c.iterate(3)
            a, b = cd.download(), ch.download()
            for p, q in zip(a, b):
                assert np.array_equal(p, q), t
            # partial downloads (the single-block copy is skipped)
            du_only = np.zeros((nq, cfg.nV))
            st_only = np.zeros(nq, np.int32)
            assert ch.lib.cmpc_download(ch._h, dptr(du_only), None, None) == 0
            assert ch.lib.cmpc_download(ch._h, None, iptr(st_only), None) == 0
            assert np.array_equal(du_only, a[0]) and np.array_equal(st_only, a[1])
            for c in (cd, ch):
                c.observe_apply()
        assert np.array_equal(cd.observer_state(), ch.observer_state())


@pytest.mark.gpu
@pytest.mark.parametrize("plant,B", [(0, 3), (1, 37)])
def test_gpu_sim_host_entry_points_match_device_ones(plant, B):
    import torch
    from cmpc.sim import PlantSimulator
    rng = np.random.default_rng(5 + plant)
    x0, u0 = cmpc.plant_default(plant)
    xs = np.ascontiguousarray(x0[None, :] * (1 + 1e-3 * rng.normal(size=(B, len(x0)))))
    us = np.ascontiguousarray(np.tile(u0, (B, 1)))
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()
    with PlantSimulator(plant, B) as sd, PlantSimulator(plant, B) as sh:
        lib = sh.lib
        sd.reset(dev(xs), dev(us), 0.05)
        assert lib.cmpc_sim_reset_host(sh._h, dptr(xs), dptr(us), 0.05) == 0
        for k in range(12):
            uc = np.ascontiguousarray(rng.uniform(-0.01, 0.01, (B, 4)))
            uc[:, [1, 3]] = np.abs(uc[:, [1, 3]])
            sd.set_input(dev(uc))
            assert lib.cmpc_sim_set_input_host(sh._h, dptr(uc)) == 0
            if k == 6:  # a plant-input step, as the setup segments do
                off = np.ascontiguousarray(us + rng.uniform(-0.01, 0.01, us.shape))
                sd.set_offset(dev(off))
                assert lib.cmpc_sim_set_offset_host(sh._h, dptr(off)) == 0
            for s in (sd, sh):
                s.integrate(k * 0.05, k * 0.05 + 0.05)
            yd = sd.output().cpu().numpy()
            yh = np.zeros((B, sh.no))
            assert lib.cmpc_sim_output_host(sh._h, dptr(yh)) == 0
            assert np.array_equal(yd, yh), k
        a, b = sd.download(), sh.download()
        for p, q in zip(a, b):
            assert np.array_equal(p, q)
        assert not a[3].any()


def test_setup_file_text_roundtrip():
    """SetupFile.text() (the writer bench.py uses for the C++ latency harness)
    parses back to the same SetupFile for every reference setup."""
    from cmpc.configs import SetupFile, reference_config, reference_setup
    for plant in ("par", "ser"):
        for ctype in ("cent", "coop", "ncoop"):
            st = reference_setup(plant, ctype)
            assert SetupFile.parse(st.text(), reference_config(plant, ctype)) == st
