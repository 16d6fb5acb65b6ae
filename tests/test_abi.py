"""The C-ABI library loads and exports every symbol include/cmpc.h declares;
host-side (non-GPU) entry points agree with the oracle.  CPU only."""
import ctypes
import os
import re

import numpy as np
import pytest

import _oracle as O
import cmpc
from cmpc._abi import EXPORTS, CmpcDims, load_library
from cmpc.configs import reference_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "cmpc.h")).read()
    return set(re.findall(r"^\s*(?:int|void\*|const char\*|double\*|int32_t\*)\s+(cmpc_\w+)\(", text, re.M))


def test_header_and_binding_agree():
    assert declared_symbols() == set(EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = load_library()
    for name in declared_symbols():
        assert hasattr(lib, name), name


@pytest.mark.parametrize("plant,ctype,p", [("par", "coop", 50), ("par", "ncoop", 50),
                                           ("par", "cent", 200), ("ser", "coop", 100),
                                           ("par", "coop", 20)])
def test_layout_matches_oracle(plant, ctype, p):
    cfg = reference_config(plant, ctype, p=p)
    dims = CmpcDims.from_config(cfg, 7)
    a, b = cmpc.layout_of(dims), O.layout(dims)
    for f, _ in a._fields_:
        assert getattr(a, f) == getattr(b, f), f
    assert a.naug == 84 and a.nd == 2 and a.n_delay_states == 80


def test_layout_rejects_bad_dims():
    cfg = reference_config("par", "coop", p=50)
    d = CmpcDims.from_config(cfg, 1)
    d.m = 60  # m > p
    L = cmpc.CmpcLayout() if hasattr(cmpc, "CmpcLayout") else None
    from cmpc._abi import CmpcLayout
    assert load_library().cmpc_layout_of(ctypes.byref(d), ctypes.byref(CmpcLayout())) != 0
    assert b"invalid" in load_library().cmpc_last_error()


def test_one_step_delay_with_two_delayed_inputs_rejected():
    """The reference's BComposite (aug_lin_sys.cc:189-197) maps a one-step
    delay onto another input's delay state when two inputs are delayed; the
    library refuses such dimensions instead of reproducing that (no GPU is
    touched: the dimensions are checked first)."""
    import dataclasses
    cfg = dataclasses.replace(reference_config("par", "coop", p=50), delays=(0, 1, 0, 40))
    d = CmpcDims.from_config(cfg, 4)
    ctx = ctypes.c_void_p()
    assert load_library().cmpc_create(ctypes.byref(ctx), ctypes.byref(d), 0) != 0
    assert b"one step" in load_library().cmpc_last_error()


def test_empty_batch_rejected_or_noop():
    """Edge cases of the batch size: an empty batch is an invalid dimension
    set (B < 1, like the reference's fixed-size Eigen types, which have no
    empty controller), and the batched solver returns at once for zero QPs
    (no device touched: this runs without a GPU)."""
    cfg = reference_config("par", "coop", p=50)
    d = CmpcDims.from_config(cfg, 1)
    d.B = 0
    from cmpc._abi import CmpcLayout
    assert load_library().cmpc_layout_of(ctypes.byref(d), ctypes.byref(CmpcLayout())) != 0
    assert b"invalid" in load_library().cmpc_last_error()
    z = np.zeros((0, 4))
    x, st, nchg, ws, tr, ntr = cmpc.qp_solve_batch(np.zeros((0, 4, 4)), z, z, z, z, z, nu=2)
    assert x.shape == (0, 4) and st.shape == (0,)


@pytest.mark.parametrize("plant", [0, 1])
def test_plant_producer_matches_oracle(plant):
    """cmpc_plant_lin_record (product, host) == or_lin_record (oracle restatement)."""
    rng = np.random.default_rng(7)
    cfg = reference_config("par" if plant == 0 else "ser", "coop", p=20)
    dims = CmpcDims.from_config(cfg, 1)
    x0, u0 = cmpc.plant_default(plant)
    xo, uo = O.plant_default(plant)
    np.testing.assert_array_equal(x0, xo)
    np.testing.assert_array_equal(u0, uo)
    for trial in range(5):
        x = x0 * (1 + 0.01 * rng.standard_normal(x0.shape))
        u = u0.copy()
        u[[0, 3, 4, 7]] += rng.uniform(-0.02, 0.02, 4)
        np.testing.assert_allclose(cmpc.plant_output(plant, x), O.plant_output(plant, x),
                                   rtol=1e-14, atol=0)
        for s in range(cfg.S):
            a = cmpc.plant_lin_record(cfg, dims, s, x, u)
            b = O.lin_record(cfg, dims, s, x, u)
            np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-14)


def test_library_fails_loudly_without_device():
    """No CPU fallback: creating a context without a HIP device is an error."""
    from tests_util import no_gpu
    if not no_gpu():
        pytest.skip("a GPU is present")
    cfg = reference_config("par", "coop", p=20)
    with pytest.raises(RuntimeError):
        cmpc.Context(cfg, 4)


@pytest.mark.parametrize("plant,ctype,p", [("par", "coop", 50), ("par", "ncoop", 50), ("par", "cent", 50),
                                           ("ser", "coop", 50), ("par", "coop", 20), ("ser", "coop", 100),
                                           ("ser", "cent", 100), ("par", "coop", 100)])
def test_rows_lds_layout_search(plant, ctype, p):
    """The row build kernel's LDS layout (rows_layout.cpp): the bank-conflict
    model of its horizon loop is no worse than regions packed back to back
    (at the bench config, coop p = 50: 28 -> <= 3 extra LDS cycles per
    wave-step), within the LDS budget that keeps the packed layout's
    workgroups per CU."""
    cfg = reference_config(plant, ctype, p=p)
    packed, chosen, nbytes = cmpc.rows_lds_model(CmpcDims.from_config(cfg, 8))
    assert chosen <= packed
    assert 0 < nbytes <= 160 * 1024
    # LDS a workgroup occupies (measured model, rows_layout.cpp): the request
    # rounded up to 512 B, plus 512 B
    alloc = (nbytes + 511) // 512 * 512 + 512
    if (plant, ctype, p) == ("par", "coop", 50):
        assert packed > 20 and chosen <= 3.0
        assert 160 * 1024 // alloc >= 3  # the kernel runs three 4-wave workgroups per CU
    if (plant, ctype, p) == ("ser", "coop", 50):
        assert 160 * 1024 // alloc >= 3  # 54 240 B (two resident) before the model
    if p == 100:
        # the reference horizon: the delayed inputs' lines are rings of D + m
        # entries and the C_hat rows overlay the hand-off areas, so two
        # four-wave workgroups share a CU (ser-coop was 107 584 B, one per CU)
        assert 160 * 1024 // alloc >= 2


def test_rows_lds_model_python_mirror_agrees():
    """tools/lds_rows_sim.py (the model in Python) and the library's model
    (rows_layout.cpp) give the same conflicts and LDS bytes for the packed
    layout of the bench configuration."""
    import sys as _sys
    _sys.path.insert(0, os.path.join(ROOT, "tools"))
    import lds_rows_sim as sim
    cfg = reference_config("par", "coop", p=50)
    dims = CmpcDims.from_config(cfg, 8)
    packed, _, _ = cmpc.rows_lds_model(dims)
    d = dict(sim.PAR_COOP, p=50)
    L = sim.layout(d)
    assert abs(sim.simulate(d, L, 0)[1] - packed) < 1e-9


@pytest.mark.parametrize("p", [20, 50, 81, 82, 83, 100, 163, 200, 250])
def test_row_kernel_ring_protocol(p):
    """The row kernel's delayed-input hand-off (lines, or rings of D + m
    entries with the writer and readers stepping back at every wrap), emulated
    with the kernel's segment bounds and unrolled blocks: every gather read at
    step s returns h_{s-k-D} (zero before the line starts), no access leaves
    the line, and the library's layout agrees on when a ring is used."""
    import sys as _sys
    _sys.path.insert(0, os.path.join(ROOT, "tools"))
    import ring_protocol_check as rp
    errs, ring, nseg = rp.check(p, 40)
    assert errs == 0
    assert (ring > 0) == (p > 2 * 40 + 1)
    assert nseg <= 16


def test_row_kernel_ring_protocol_random_delays():
    """The same emulation over random horizons, delays, move counts and
    unrolls (the kernel's and the others the code supports): every read
    returns the value written for it, with or without rings."""
    import sys as _sys
    _sys.path.insert(0, os.path.join(ROOT, "tools"))
    import ring_protocol_check as rp
    rng = np.random.default_rng(7)
    for _ in range(300):
        p = int(rng.integers(2, 260))
        D = int(rng.integers(1, p + 5))
        M = int(rng.integers(1, 3))
        U = int(rng.choice([rp.KERNEL_U, 4, 5, 10]))
        errs, ring, _ = rp.check(p, D, M=M, U=U)
        assert errs == 0, (p, D, M, U)
        assert (ring > 0) == ((M - 1) + max(0, p - D) > D + M), (p, D, M)


def test_rows_layout_search_under_sanitizers():
    """The row kernel's LDS layout search (rows_layout.cpp, host code) built
    with AddressSanitizer and UndefinedBehaviorSanitizer and run over 40
    random dimension sets (0.6 s each under the sanitizers; the binary takes
    the count as its argument): no memory or UB error, and every layout it returns
    keeps its regions, segments and LDS inside the bounds the kernel assumes
    (tests/cpp/rows_layout_asan.cpp)."""
    import subprocess
    here = os.path.join(ROOT, "tests", "cpp")
    subprocess.check_call(["make", "-s", "-C", here, "rows_layout_asan"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(here, "rows_layout_asan"), "40"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.startswith("ok"), r.stdout
    assert "runtime error" not in r.stderr, r.stderr[-2000:]


def test_timing_stride_refuses_bad_arguments():
    """cmpc_set_timing_stride: a null context and a stride below 1 are
    errors (no device needed for either check)."""
    lib = load_library()
    assert lib.cmpc_set_timing_stride(None, 5) < 0
