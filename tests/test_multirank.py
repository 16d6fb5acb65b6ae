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
