"""The profile pipeline's own tools, on synthetic inputs (CPU): the marker
cut of a kernel trace (tools/headline_pass_stats.py) and the bench kernel's
machine-code hash (tools/kernel_hash.py) that ties PMC traffic to the code it
was measured on."""
import csv
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")
BUILD = "void cmpc_build_rows_kernel<11, 3, 4, 2, 2, 2, 4, false, 3, 0>(BuildParams)"
SOLVE = "void (anonymous namespace)::cmpc_solve_kernel<4, 2, 4, false, false>(SolveParams)"
MARK = "void at::native::sleep(long)"


def _trace(path, timed_builds, timed_iters, pass_builds, pass_iters):
    """A kernel trace: marker, the timed steps, marker, marker, the iterate
    event pass, marker (durations in us, back to back, 1 us apart)."""
    rows, t = [], 1_000_000

    def add(name, dur_us):
        nonlocal t
        rows.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + int(dur_us * 1000)})
        t += int(dur_us * 1000) + 1000

    add(MARK, 5)
    for b, i in zip(timed_builds, timed_iters):
        add(BUILD, b)
        add(SOLVE, i)
    add(MARK, 5)
    add("void cmpc_other_kernel(int)", 3)
    add(MARK, 5)
    for b, i in zip(pass_builds, pass_iters):
        add(BUILD, b)
        add(SOLVE, i)
    add(MARK, 5)
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)


def _line(path, build_us, iterate_us, stride):
    line = {"roofline": {"avg_launch_ms": build_us / 1e3},
            "kernels_ms_per_step": {"iterate": iterate_us / 1e3, "build_event_stride": stride}}
    with open(path, "w") as fh:
        fh.write("bench.py: a log line\n" + json.dumps(line) + "\n")


def test_headline_pass_stats_cuts_at_markers(tmp_path):
    timed_b = [240.0 + k for k in range(10)]       # 240 .. 249
    pass_b = [230.0] * 10
    _trace(tmp_path / "t.csv", timed_b, [30.0] * 10, pass_b, [31.0] * 10)
    _line(tmp_path / "run.json", 250.0, 33.0, 5)   # the profiled run's own events
    _line(tmp_path / "ref.json", 240.0, 32.0, 5)   # an unprofiled reference line
    out = tmp_path / "out.csv"
    r = subprocess.run([sys.executable, os.path.join(TOOLS, "headline_pass_stats.py"), str(tmp_path / "t.csv"),
                        str(tmp_path / "run.json"), str(tmp_path / "ref.json"), str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    rows = {(x["pass"], "build" if "build" in x["kernel"] else "solve"): x for x in csv.DictReader(open(out))}
    tb = rows[("timed_steps", "build")]
    assert int(tb["calls"]) == 10 and float(tb["rocprof_avg_us"]) == pytest.approx(244.5)
    assert float(tb["ratio"]) == pytest.approx(244.5 / 240.0, abs=1e-4)
    assert float(tb["run_ratio"]) == pytest.approx(244.5 / 250.0, abs=1e-4)
    # the launch between the passes is in neither
    assert all("other" not in x["kernel"] for x in rows.values())
    pi = rows[("iterate_event_pass", "solve")]
    assert float(pi["rocprof_avg_us"]) == pytest.approx(31.0)
    assert float(pi["ratio"]) == pytest.approx(31.0 / 32.0, abs=1e-4)
    assert float(pi["run_ratio"]) == pytest.approx(31.0 / 33.0, abs=1e-4)
    # the timed pass's iterate has no events to compare with
    assert rows[("timed_steps", "solve")]["ratio"] == ""
    # the event-stamped launches: every 5th timed build from the first (240, 245)
    st = rows[("timed_steps_stamped", "build")]
    assert int(st["calls"]) == 2 and float(st["rocprof_avg_us"]) == pytest.approx(242.5)
    assert float(st["run_ratio"]) == pytest.approx(242.5 / 250.0, abs=1e-4)


def test_headline_pass_stats_refuses_a_trace_without_four_markers(tmp_path):
    _trace(tmp_path / "t.csv", [240.0], [30.0], [230.0], [31.0])
    rows = list(csv.DictReader(open(tmp_path / "t.csv")))
    with open(tmp_path / "t3.csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows[1:])                      # the first marker dropped
    _line(tmp_path / "run.json", 250.0, 33.0, 1)
    r = subprocess.run([sys.executable, os.path.join(TOOLS, "headline_pass_stats.py"), str(tmp_path / "t3.csv"),
                        str(tmp_path / "run.json")], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "expected 4 marker launches" in r.stderr


def test_kernel_hash_finds_the_bench_kernel():
    lib = os.path.join(ROOT, "compressor-mpc_amd", "cmpc", "libcmpc.so")
    if not os.path.exists(lib):
        pytest.skip("libcmpc.so not built")
    key = "cmpc_build_rows_kernelILi11ELi3ELi4ELi2ELi2ELi2ELi4ELb0ELi3ELi0EE"
    r = subprocess.run([sys.executable, os.path.join(TOOLS, "kernel_hash.py"), lib, key],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    h, size, sym = r.stdout.split()
    assert re.fullmatch(r"[0-9a-f]{16}", h) and int(size) > 1000 and key in sym
    # deterministic
    again = subprocess.run([sys.executable, os.path.join(TOOLS, "kernel_hash.py"), lib, key],
                           capture_output=True, text=True, timeout=60)
    assert again.stdout == r.stdout
    r = subprocess.run([sys.executable, os.path.join(TOOLS, "kernel_hash.py"), lib, "no_such_kernel"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "not found" in r.stderr
