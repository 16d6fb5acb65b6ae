"""The C++ adapter (include/cmpc/nerve_center.hpp) — the reference's NerveCenter
API over the C ABI — driven like the reference's tests/*-with-timing.cc
harnesses: a setup file in the reference's format, SetWeights /
SetOutputReference / constraints, Initialize, GetNextInputWithTiming.

CPU: the drivers build and fail loudly (no CPU fallback) without a device.
GPU: u(t = 0) matches the reference's own step-0 records (6 digits); the
closed-loop timing executable (tests/cpp/with_timing.cpp: NerveCenter +
SimulationSystem, the replacement of the missing common-simulation.inc)
writes the reference's recorded runs.
"""
import os
import subprocess

import pytest

import golden_cases as GC

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(HERE, "cpp", "nerve_center_step0")
HARNESS = os.path.join(HERE, "cpp", "with_timing")


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "cpp"), "nerve_center_step0", "with_timing"])
    assert os.path.exists(DRIVER) and os.path.exists(HARNESS)


def _mat(vals, n):
    return "\n".join("\t".join("%g" % v for v in vals[r * n:(r + 1) * n]) for r in range(n))


def write_setup(path, g, ny, S, n_timing=None):
    """setup/setup-<ctrl>-<plant> layout (key line, values, blank line);
    n_timing: n-timing-iterations (run-all-tests.sh sweeps it 1..9)."""
    nci = int(round(len(g["uwt"]) ** 0.5))
    blk = ny * ny
    yw = g["ywt"]
    blocks = [yw[i * blk:(i + 1) * blk] for i in range(len(yw) // blk)]
    n = (9 if g["plant"] == "parallel" else 8) + 1
    sim = g["simulation"]
    segs = [(sim[i:i + n - 1], sim[i + n - 1]) for i in range(0, len(sim), n)]
    parts = [
        ("n-iterations", str(g["n_iterations"])),
        ("n-timing-iterations", str(g["n_iterations"] if n_timing is None else n_timing)),
        ("folder-name", "parallel"),
        ("output-filename", "out.dat"),
        ("yref", " ".join("%g" % v for v in g["yref"])),
        ("uwt", _mat(g["uwt"], nci)),
        ("ywt", "\n\n".join(_mat(b, ny) for b in blocks)),
        ("constraints-lower", "\t".join("%g" % v for v in g["constraints_lower"])),
        ("constraints-upper", "\t".join("%g" % v for v in g["constraints_upper"])),
        ("constraints-rate-lower", "\t".join("%g" % v for v in g["rate_lower"])),
        ("constraints-rate-upper", "\t".join("%g" % v for v in g["rate_upper"])),
        ("simulation", "\n\n".join(" ".join("%g" % v for v in d) + "\n%g" % te for d, te in segs)),
    ]
    with open(path, "w") as fh:
        for k, v in parts:
            fh.write(f"{k}\n{v}\n\n")


def test_driver_builds_and_fails_loudly_without_device(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    _build()
    cfg, _, _, g = GC.case("coop-par")
    setup = tmp_path / "setup-coop-par"
    write_setup(setup, g, cfg.ny, cfg.S)
    r = subprocess.run([DRIVER, str(setup), "par", "coop"], capture_output=True, text=True)
    assert r.returncode == 1
    assert "error: cmpc_create" in r.stderr


def test_harness_builds_and_fails_loudly_without_device(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    _build()
    cfg, _, _, g = GC.case("coop-par")
    setup = tmp_path / "setup-coop-par"
    write_setup(setup, g, cfg.ny, cfg.S)
    r = subprocess.run([HARNESS, str(setup), "par", "coop", str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 1 and "error: cmpc_create" in r.stderr, r.stderr


def test_setup_writer_roundtrip(tmp_path):
    """The written file parses back (Python mirror of read_files.h) to the fixture."""
    from cmpc.configs import SetupFile
    cfg, setup, _, g = GC.case("coop-par")
    path = tmp_path / "s"
    write_setup(path, g, cfg.ny, cfg.S)
    back = SetupFile.parse(path.read_text(), cfg)
    assert back.n_iterations == g["n_iterations"]
    assert back.uwt == g["uwt"]
    assert back.ywt[0] == setup.ywt[0] and back.ywt[1] == setup.ywt[1]
    assert back.rate_upper == g["rate_upper"]
    assert back.segments == setup.segments


@pytest.mark.gpu
@pytest.mark.parametrize("observer", [False, True, "iface"],
                         ids=["external-estimate", "device-observer", "controller-interface"])
@pytest.mark.parametrize("name", ["cent-par", "coop-par", "ncoop-par", "cent-ser", "coop-ser", "ncoop-ser"])
def test_gpu_cpp_adapter_step0_matches_reference(name, observer, tmp_path):
    """The reference's call pattern through cmpc::NerveCenter; with
    SetObserver the reference's own GetNextInputWithTiming(y, n, t), or
    GetNextInput(y) through the ControllerInterface base."""
    _build()
    cfg, _, _, g = GC.case(name)
    ctype, plant = name.split("-")
    setup = tmp_path / f"setup-{name}"
    write_setup(setup, g, cfg.ny, cfg.S)
    mode = {False: [], True: ["observer"], "iface": ["iface"]}[observer]
    args = [DRIVER, str(setup), plant, ctype, "100"] + mode
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    u = [float(t) for t in r.stdout.split()]
    assert "status: " + " ".join(["0"] * cfg.S) in r.stderr, r.stderr
    GC.assert_six_digits(u, g["u0"])


def read_dat(path):
    lines = open(path).read().split("\n")
    recs = []
    for i in range(0, len(lines) - 5, 6):
        recs.append({"t": lines[i], "x": lines[i + 1], "u": lines[i + 2], "y": lines[i + 3]})
    return recs


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cent-par", "coop-par", "ncoop-par", "cent-ser", "coop-ser", "ncoop-ser"])
def test_gpu_cpp_harness_writes_reference_run(name, tmp_path):
    """The whole 500 s run through the C++ adapter: all 10 000 records equal
    the reference's (u, y to every printed digit, |v| < 1e-12 as 0; the
    record times; the plant states of the first 160 records)."""
    import json
    import numpy as np
    _build()
    cfg, _, _, g = GC.case(name)
    ctype, plant = name.split("-")
    setup = tmp_path / f"setup-{name}"
    write_setup(setup, g, cfg.ny, cfg.S)
    r = subprocess.run([HARNESS, str(setup), plant, ctype, str(tmp_path)], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr
    recs = read_dat(tmp_path / "parallel" / "out.dat")
    key = {"cent": "centralized", "coop": "coop9", "ncoop": "ncoop9"}[ctype]
    gold = np.load(os.path.join(HERE, "golden", "traj_long.npz"))
    ur, yr = gold[f"{plant}_{key}_u"], gold[f"{plant}_{key}_y"]
    assert len(recs) == len(ur) == 10000
    first = json.load(open(os.path.join(HERE, "golden", f"traj_{plant}_{key}.json")))["records"]
    full = GC.read_full(str(tmp_path / "parallel" / "out.dat") + ".full")
    assert len(full) == len(recs)
    ties = 0
    for k, rec in enumerate(recs):
        assert float(rec["t"]) == float("%g" % (k * 0.05)), (k, rec["t"])
        for i, (key_, ref) in enumerate((("u", ur[k]), ("y", yr[k]))):
            eq, tie = GC.six_digit_strings_ok(rec[key_].split(), ref, full[k][i])
            assert eq or tie, (k, key_, rec[key_], ref)
            ties += tie
        if k < len(first):
            assert [float(v) for v in rec["x"].split()] == first[k]["x"], k
    assert ties <= 2, ties  # rounding-boundary ties (golden_cases.six_digit_rows)


@pytest.mark.gpu
@pytest.mark.parametrize("n_timing", [1, 4])
def test_gpu_cpp_harness_timed_prefix_keeps_trajectory(n_timing, tmp_path):
    """setup/run-all-tests.sh runs coop with n-timing-iterations 1..9 and the
    reference's coop1..coop9 files hold one trajectory: the
    timed prefix splits the K Jacobi iterations into two launches without
    changing a record (first 1 200 records, across the 50 s step)."""
    import numpy as np
    _build()
    cfg, _, _, g = GC.case("coop-par")
    setup = tmp_path / "setup-coop-par"
    write_setup(setup, g, cfg.ny, cfg.S, n_timing=n_timing)
    r = subprocess.run([HARNESS, str(setup), "par", "coop", str(tmp_path), "1200"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    recs = read_dat(tmp_path / "parallel" / "out.dat")
    gold = np.load(os.path.join(HERE, "golden", "traj_long.npz"))
    ur = gold["par_coop9_u"]
    assert len(recs) == 1200
    full = GC.read_full(str(tmp_path / "parallel" / "out.dat") + ".full")
    ties = 0
    for k, rec in enumerate(recs):
        eq, tie = GC.six_digit_strings_ok(rec["u"].split(), ur[k], full[k][0])
        assert eq or tie, (k, rec["u"], ur[k])
        ties += tie
    assert ties <= 2, ties


LOOP = os.path.join(HERE, "cpp", "distributed_controller_loop")


def test_controller_loop_builds_and_fails_loudly_without_device(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "cpp"), "distributed_controller_loop"])
    cfg, _, _, g = GC.case("coop-par")
    setup = tmp_path / "setup-coop-par"
    write_setup(setup, g, cfg.ny, cfg.S)
    r = subprocess.run([LOOP, str(setup), "par", "coop"], capture_output=True, text=True)
    assert r.returncode == 1 and "error: cmpc_create" in r.stderr, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cent-par", "coop-par", "ncoop-par", "cent-ser", "coop-ser", "ncoop-ser"])
def test_gpu_distributed_controller_api_matches_nerve_center(name, tmp_path):
    """The per-object DistributedController API (Initialize, SetWeights,
    SetOutputReference, GenerateInitialQP, GetInput, UpdateU,
    GetStateEstimate; distributed_controller.h:131-191; on odd steps their
    timed overloads, :155-183), each sub-controller
    on its own one-slot context and the Jacobi loop run on the host as
    NerveCenter runs it, equals cmpc::NerveCenter bit for bit over 6 steps
    with a moving measured output (applied inputs, plans, statuses, state
    estimates)."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "cpp"), "distributed_controller_loop"])
    cfg, _, _, g = GC.case(name)
    ctype, plant = name.split("-")
    setup = tmp_path / f"setup-{name}"
    write_setup(setup, g, cfg.ny, cfg.S)
    r = subprocess.run([LOOP, str(setup), plant, ctype, "50", "6"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("step ")]
    assert len(lines) == 6 and all(" equal " in l for l in lines), r.stdout
    # UpdateAndSolveQP refuses a mis-sized QP wherever it is called
    assert "ACCEPTED" not in r.stdout
    if ctype != "cent":
        assert "mis-sized QP: refused" in r.stdout, r.stdout
    # steps 1, 3, 5 ran through the timed overloads (UpdateU / GenerateInitialQP
    # / GetInput on a CpuTimer, distributed_controller.h:155-183): the same
    # bits, and the timers accumulated
    assert sum("(timed overloads)" in l for l in lines) == 3, r.stdout
    assert "timed overloads: GenerateInitialQP" in r.stdout and "timers: not accumulated" not in r.stdout
