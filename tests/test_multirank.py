"""Multi-rank scenario sharding, world size 2 over gloo on CPU.

Each rank owns a contiguous block of whole scenarios (both sub-controllers of a
scenario stay on one rank, so the Jacobi exchange needs no collective), steps
it, and the results are all-gathered.  On CPU the step is the oracle (the
compute stand-in here; the GPU variant below runs the product kernels); the
gathered result must equal a single-process step over the whole batch bit for
bit, since scenarios are independent.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from cmpc.sharding import qp_slice, shard_arrays, shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 65537):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = shard_range(n, world, r)
                seen.extend(range(s, s + c))
            assert seen == list(range(n))
            sizes = [shard_range(n, world, r)[1] for r in range(world)]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_qp_slice_keeps_subcontrollers_together():
    S = 2
    for r in range(3):
        s, c = shard_range(11, 3, r)
        sl = qp_slice(s, c, S)
        assert sl.start % S == 0 and sl.stop % S == 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem(B):
    from cmpc import reference_config
    from cmpc.configs import reference_setup
    from cmpc.problem import controller_arrays
    from cmpc.synthetic import synthetic_batch
    cfg = reference_config("par", "coop", p=20)
    arr = controller_arrays(cfg, reference_setup("par", "coop"))
    lin, u, du, ws = synthetic_batch(cfg, B, seed=77, n_distinct=B)
    return cfg, arr, lin, u, du, ws


def _oracle_step(cfg, arr, lin, u, du, ws, K):
    import _oracle as O
    from cmpc._abi import CmpcDims
    B = lin.shape[0] // cfg.S
    dims = CmpcDims.from_config(cfg, B)
    u, du, ws = u.copy(), du.copy(), ws.copy()
    O.step(dims, arr, lin, K, u, du, ws, init=True)
    out = O.step(dims, arr, lin, K, u, du, ws, flags=1)
    return out[0], out[1], u


def _worker(rank, world, port, B, K, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cmpc.sharding import gather_to_all
        cfg, arr, lin, u, du, ws = _problem(B)
        lin_r, u_r, du_r, ws_r = shard_arrays(rank, world, cfg.S, lin, u, du, ws)
        d, st, u_new = _oracle_step(cfg, arr, lin_r, u_r, du_r, ws_r, K)
        d_all = gather_to_all(d, B * cfg.S, cfg.S)
        st_all = gather_to_all(st, B * cfg.S, cfg.S)
        u_all = gather_to_all(u_new, B * cfg.S, cfg.S)
        if rank == 0:
            q.put((d_all, st_all, u_all))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_matches_single_process():
    B, K, world = 37, 9, 2          # odd B: unequal shards
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    d_all, st_all, u_all = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg, arr, lin, u, du, ws = _problem(B)
    d_ref, st_ref, u_ref = _oracle_step(cfg, arr, lin, u, du, ws, K)
    assert np.array_equal(d_all, d_ref)
    assert np.array_equal(st_all, st_ref)
    assert np.array_equal(u_all, u_ref)


def _product_step(cfg, arr, lin, u, du, ws, K):
    import cmpc
    B = lin.shape[0] // cfg.S
    with cmpc.Context(cfg, B, device=0) as ctx:
        ctx.configure(arr)
        ctx.set_state(u, du, ws)
        ctx.upload_lin(lin)
        ctx.build()
        ctx.init_warmstart()
        ctx.step(K, cmpc.CMPC_APPLY_MOVE)
        d, st, _ = ctx.download()
        u_new, _, _ = ctx.get_state()
    return d, st, u_new


def _gpu_worker(rank, world, port, B, K, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from cmpc.sharding import gather_to_all
        cfg, arr, lin, u, du, ws = _problem(B)
        lin_r, u_r, du_r, ws_r = shard_arrays(rank, world, cfg.S, lin, u, du, ws)
        d, st, u_new = _product_step(cfg, arr, lin_r, u_r, du_r, ws_r, K)
        out = [gather_to_all(a, B * cfg.S, cfg.S) for a in (d, st, u_new)]
        if rank == 0:
            q.put(tuple(out))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_two_ranks_match_single_process():
    """Two ranks (sharing the box's GPU) step their shards with the product
    kernels; the gathered plans equal one process stepping the whole batch."""
    B, K, world = 1001, 9, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, B, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    d_all, st_all, u_all = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cfg, arr, lin, u, du, ws = _problem(B)
    d_ref, st_ref, u_ref = _product_step(cfg, arr, lin, u, du, ws, K)
    assert np.array_equal(d_all, d_ref)
    assert np.array_equal(st_all, st_ref)
    assert np.array_equal(u_all, u_ref)


def _rccl_worker(port, q):
    """One rank with a real RCCL (nccl) communicator of world size 1."""
    import torch
    import torch.distributed as dist
    import cmpc
    from cmpc.configs import reference_setup
    from cmpc.coupled import CoupledRank, synthetic_g_ext
    from cmpc.sharding import gather_to_all
    from cmpc.synthetic import synthetic_batch
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        # scenario sharding's result gather on the device
        a = np.arange(2 * 37 * 3, dtype=np.float64).reshape(2 * 37, 3)
        g_ok = bool(np.array_equal(gather_to_all(a, 2 * 37, 2), a))
        # config 4's plan all-gather (all_gather_into_tensor) against the local copy
        cfg = cmpc.reference_config("par", "coop", p=20)
        arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
        S_local, B, K = 8, 64, 9
        nqp = B * S_local
        lin, u_old, _, _ = synthetic_batch(cfg, nqp // cfg.S, seed=77, n_distinct=64)
        plans = []
        for force in (False, True):
            ctx = cmpc.Context(cfg, nqp // cfg.S, device=0)
            try:
                ctx.configure(arr)
                ctx.set_state(u_old, np.zeros((nqp, cfg.nV)), np.zeros(nqp, np.uint32))
                ctx.upload_lin(lin)
                ctx.build()
                ctx.init_warmstart()
                _, _, G = ctx.download_qp()
                G_ext = torch.from_numpy(synthetic_g_ext(G, S_local, S_local, 0)).cuda()
                cr = CoupledRank(ctx, S_local, S_local, 0, 1, G_ext, force_collective=force)
                for _ in range(2):
                    cr.step(K)
                torch.cuda.synchronize()
                du, st, _ = ctx.download()
                plans.append((du, st))
            finally:
                ctx.close()
        c_ok = bool(np.array_equal(plans[0][0], plans[1][0]) and np.array_equal(plans[0][1], plans[1][1]))
        # the bench's timing reductions
        t = torch.tensor([1.5], dtype=torch.float64, device="cuda:0")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier()
        q.put((g_ok, c_ok, float(t.item()), int((plans[1][1] == 0).sum()), nqp))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_rccl_single_rank_paths():
    """The multi-GPU code paths on a one-GPU box: an RCCL (nccl) process group
    of one rank runs the device gather of the scenario shards, config 4's plan
    all_gather_into_tensor (equal bit for bit to the local copy it replaces)
    and the bench's barrier and max reduction.  (RCCL refuses two ranks on one
    device; the 8-GPU run is the driver's.)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    g_ok, c_ok, tmax, n_ok, nqp = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert g_ok and c_ok
    assert tmax == 1.5
    assert n_ok == nqp


@pytest.mark.gpu
def test_gpu_bench_force_dist_single_rank():
    """bench.py under torch.distributed.run with one rank and --force-dist:
    the RCCL process group, barrier, max over ranks and the coupled section's
    all-gather run as in the driver's N-GPU launch, and the line reports the
    RCCL exchange."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "1", "--force-dist", "--steps", "4", "--warmup", "1", "--no-cpu",
           "--batch", "4096", "--input-batches", "2", "--coupled-batch", "512",
           "--settle-seconds", "0.02"]
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["qp_status_ok_fraction"] == 1.0
    assert d["coupled"]["exchange"].startswith("RCCL")
    assert d["coupled"]["qp_status_ok_fraction"] == 1.0
    # config 4's own 64-sub-controller system: all 64 on
    # this one rank, its coupling matrix's HBM fraction from the iterate events
    c64 = d["coupled_s64"]
    assert c64["S_total"] == 64 and c64["S_local"] == 64 and c64["qp_per_gpu"] == 64 * 512
    assert c64["qp_status_ok_fraction"] == 1.0
    assert 0.0 < c64["G_ext_hbm_frac"] < 1.0
    assert d["n_gpus"] == d["gpus_requested"] == 1
    assert len(d["rank_ms_per_step"]) == 1 and abs(d["rank_ms_per_step"][0] - d["ms_per_step"]) < 1e-9
    # the recorded run's solver load beside the synthetic one
    assert d["recorded_run_working_set_changes_per_qp_step"] == d["recorded_run"]["working_set_changes_per_qp_step"]
    assert d["recorded_run_working_set_changes_per_qp_step"] < d["working_set_changes_per_qp_step"]


def _bench_module():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_bench_launch_plan():
    """bench.py --gpus N starts N ranks itself when no launcher did (VERDICT
    r5, next 1); a launcher's WORLD_SIZE must equal --gpus; RCCL needs one
    visible GPU per rank (gloo rehearsals may share one)."""
    b = _bench_module()
    never = lambda: pytest.fail("device count asked without need")  # noqa: E731
    assert b.launch_plan(1, "nccl", {}, never) == ("here", None)
    assert b.launch_plan(8, "nccl", {"WORLD_SIZE": "8"}, never) == ("here", None)
    assert b.launch_plan(1, "nccl", {"WORLD_SIZE": "1"}, never) == ("here", None)
    assert b.launch_plan(8, "nccl", {}, lambda: 8) == ("spawn", 8)
    assert b.launch_plan(2, "gloo", {}, never) == ("spawn", 2)
    with pytest.raises(SystemExit, match="1 visible"):
        b.launch_plan(8, "nccl", {}, lambda: 1)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        b.launch_plan(8, "nccl", {"WORLD_SIZE": "2"}, never)
    with pytest.raises(SystemExit, match="WORLD_SIZE=1"):
        b.launch_plan(2, "gloo", {"WORLD_SIZE": "1"}, never)


def test_bench_spawn_ranks_relays_rank0_and_exit_code(tmp_path, capfd):
    """spawn_ranks runs torch.distributed.run as a child (not exec), the ranks
    see WORLD_SIZE = N and the self-launch marker, rank 0's stdout line is
    relayed, and the child's exit code is returned."""
    import json
    b = _bench_module()
    script = tmp_path / "rank.py"
    script.write_text(
        "import json, os, sys\n"
        "r = int(os.environ['RANK'])\n"
        "if r == 0:\n"
        "    print(json.dumps({'world': int(os.environ['WORLD_SIZE']), 'argv': sys.argv[1:],\n"
        "                      'marker': os.environ.get('" + b.SELF_LAUNCH_ENV + "')}), flush=True)\n"
        "sys.exit(3 if '--fail' in sys.argv else 0)\n")
    rc = b.spawn_ranks(2, ["--gpus", "2"], script=str(script))
    out = capfd.readouterr().out
    assert rc == 0
    d = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
    assert d == {"world": 2, "argv": ["--gpus", "2"], "marker": "1"}
    assert b.spawn_ranks(2, ["--fail"], script=str(script)) != 0


def test_bench_spawn_ranks_forwards_termination(tmp_path):
    """A time limit on `bench.py --gpus N` (SIGTERM to the parent) reaches the
    torch.distributed.run child and its ranks: the parent returns promptly
    instead of leaving ranks behind."""
    import signal
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "rank.py"
    pidfile = tmp_path / "pids"
    script.write_text("import os, time\n"
                      f"open({str(pidfile)!r} + os.environ['RANK'], 'w').write(str(os.getpid()))\n"
                      "time.sleep(600)\n")
    driver = ("import importlib.util, sys\n"
              f"spec = importlib.util.spec_from_file_location('b', {os.path.join(root, 'bench.py')!r})\n"
              "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
              f"sys.exit(b.spawn_ranks(2, [], script={str(script)!r}))\n")
    p = subprocess.Popen([sys.executable, "-c", driver])
    t0 = time.time()
    while not all(os.path.exists(f"{pidfile}{r}") for r in range(2)):
        assert time.time() - t0 < 120 and p.poll() is None
        time.sleep(0.2)
    ranks = [int(open(f"{pidfile}{r}").read()) for r in range(2)]
    p.send_signal(signal.SIGTERM)
    p.wait(timeout=60)
    assert p.returncode != 0
    t1 = time.time()
    while any(os.path.exists(f"/proc/{pid}") and "zombie" not in open(f"/proc/{pid}/status").read().lower()
              for pid in ranks):
        assert time.time() - t1 < 30, "a rank outlived the terminated parent"
        time.sleep(0.2)
