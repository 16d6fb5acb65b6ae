"""Sub-controller-sharded cooperative iteration:
S_total sub-controllers per scenario over `world` ranks, plans all-gathered
once per Jacobi iteration (cmpc/coupled.py, coupled.hip).

CPU: layout-independence of the synthetic coupling, the rank-major plan
indexing, and the sharded loop over gloo (world size 2, the oracle's solver as
the compute) equal to one process.  GPU: the product kernel equals the same
loop with the oracle's solver on the product's QPs (bit-exact solver), and two
ranks sharing the GPU equal one."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import _oracle as O
from cmpc.coupled import coupled_jacobi, coupling_weights, others, synthetic_g_ext

S_TOTAL, B, K = 8, 6, 9
# SURVEY config 4's real partition (8 ranks x 8 sub-controllers), rehearsed on
# CPU with a small batch
S_TOTAL8, B8 = 64, 2


def test_coupling_weights_are_layout_independent():
    w = coupling_weights(3, 5, S_TOTAL)
    assert w.shape == (S_TOTAL - 1,)
    assert np.all(w > 0) and w.max() <= 0.6
    # the same (scenario, s, j) triple gives the same weight in any sharding
    G = np.random.default_rng(0).normal(size=(B * S_TOTAL, 4, 4))
    full = synthetic_g_ext(G, S_TOTAL, S_TOTAL, 0).reshape(4, (S_TOTAL - 1) * 4, B, S_TOTAL)
    for world in (2, 4):
        sl = S_TOTAL // world
        for r in range(world):
            Gr = G.reshape(B, S_TOTAL, 4, 4)[:, r * sl:(r + 1) * sl].reshape(-1, 4, 4)
            part = synthetic_g_ext(Gr, S_TOTAL, sl, r * sl).reshape(4, (S_TOTAL - 1) * 4, B, sl)
            assert np.array_equal(part, full[:, :, :, r * sl:(r + 1) * sl])


def test_rank_major_plan_indexing():
    world, sl = 4, 2
    du_all = np.arange(world * B * sl * 4, dtype=float).reshape(world, B, sl, 4)
    o = others(du_all, b=2, s=5, S_total=world * sl, S_local=sl)
    expect = [du_all[j // sl, 2, j % sl] for j in range(world * sl) if j != 5]
    assert np.array_equal(o, np.concatenate(expect))


# ---- the loop with the oracle's solver as the compute ----------------------

def problem(S_total=S_TOTAL, Bn=B):
    import cmpc
    from cmpc.configs import reference_setup
    from cmpc.synthetic import synthetic_batch
    from cmpc._abi import CmpcDims
    cfg = cmpc.reference_config("par", "coop", p=20)
    arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
    nrec = Bn * S_total                    # record (b, s_global) = b * S_total + s
    lin, u_old, _, _ = synthetic_batch(cfg, nrec // cfg.S, seed=12)
    dims = CmpcDims.from_config(cfg, 1)
    H, f, G = [], [], []
    for q in range(nrec):
        h, ff, _, _, g = O.build_qp(dims, lin[q], u_old[q], arr.y_ref[q % cfg.S], arr.ywt[q % cfg.S],
                                    arr.uwt[q % cfg.S])
        H.append(h); f.append(ff); G.append(g)
    return cfg, arr, np.array(H), np.array(f), np.array(G), u_old


def oracle_loop(cfg, arr, H, f, G, u_old, rank, world, gather, S_total=S_TOTAL, Bn=B):
    """This rank's QPs through coupled_jacobi with or_qp_solve (the oracle)."""
    sl = S_total // world
    glob = [b * S_total + rank * sl + i for b in range(Bn) for i in range(sl)]
    Gx = synthetic_g_ext(G[glob], S_total, sl, rank * sl).reshape(4, -1, len(glob))
    ws = np.zeros(len(glob), np.uint32)
    nu = cfg.nu

    def solve(du_all, apply):
        du_all = du_all.reshape(world, Bn, sl, 4)
        out = np.zeros((len(glob), 4))
        for i, q in enumerate(glob):
            b, li = divmod(i, sl)
            s_cfg = q % cfg.S
            d = others(du_all, b, rank * sl + li, S_total, sl)
            fk = [float(v) for v in f[q]]
            for j in range(S_total - 1):          # the kernel's order: j, then a, then v
                for a in range(4):
                    for v in range(4):
                        fk[a] = fk[a] + float(Gx[a, j * 4 + v, i]) * float(d[j * 4 + v])
            lo = np.tile(arr.lower[s_cfg] - u_old[q, :nu], 2)
            up = np.tile(arr.upper[s_cfg] - u_old[q, :nu], 2)
            x, info = O.qp_solve(H[q], np.array(fk), lo, up, np.tile(arr.rate_lower[s_cfg], 2),
                                 np.tile(arr.rate_upper[s_cfg], 2), nu, int(ws[i]))
            ws[i] = info.ws
            out[i] = x
        return out

    return coupled_jacobi(K, solve, gather, np.zeros((len(glob), 4)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cpu_worker(rank, world, port, q, S_total=S_TOTAL, Bn=B):
    import torch
    import torch.distributed as dist
    torch.set_num_threads(1)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg, arr, H, f, G, u_old = problem(S_total, Bn)

        def gather(du_local):
            parts = [torch.zeros(du_local.shape, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(du_local)))
            return torch.stack(parts).numpy()

        du = oracle_loop(cfg, arr, H, f, G, u_old, rank, world, gather, S_total, Bn)
        allp = gather(du)
        if rank == 0:
            q.put(allp)
    finally:
        dist.destroy_process_group()


def _sharded_equals_one(world, S_total, Bn):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_cpu_worker, args=(r, world, port, q, S_total, Bn)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        got = q.get(timeout=600)
    finally:
        for p in ps:
            p.join(timeout=120)
    for p in ps:
        assert p.exitcode == 0
    cfg, arr, H, f, G, u_old = problem(S_total, Bn)
    ref = oracle_loop(cfg, arr, H, f, G, u_old, 0, 1, lambda d: d[None], S_total, Bn)
    # rank-major [world][B][sl][4] -> global [B][S_total][4]
    sl = S_total // world
    got = got.reshape(world, Bn, sl, 4).transpose(1, 0, 2, 3).reshape(-1, 4)
    assert np.array_equal(got, ref)
    return ref


def test_sharded_loop_two_ranks_gloo_equals_one():
    _sharded_equals_one(2, S_TOTAL, B)


def test_sharded_loop_config4_partition_eight_ranks_gloo_equals_one():
    """SURVEY config 4's own partition: 8 ranks x S_local = 8 sub-controllers,
    S_total = 64 per scenario (rank-major plan indexing over 8 ranks), the
    plans all-gathered over gloo once per Jacobi iteration, the oracle's
    solver as the compute: bit-exact with one process running all 64."""
    ref = _sharded_equals_one(8, S_TOTAL8, B8)
    assert np.abs(ref).max() > 0  # the coupling moved the plans


def test_abi_refuses_coupled_reads_beyond_the_callers_buffers():
    """cmpc_coupled_iterate's own checks (cmpc_coupled_validate, host only):
    a one-rank plan buffer for S_total = 64 sub-controllers with S_local = 8
    (the layout that faulted the GPU in round 3) is refused in C with an
    error naming du_all, as is a G_ext shorter than the kernel reads."""
    import ctypes
    import cmpc
    from cmpc._abi import CmpcDims, load_library
    lib = load_library()
    cfg = cmpc.reference_config("par", "coop", p=50)
    S_local, Bsc = 8, 4096
    nqp = Bsc * S_local
    dims = CmpcDims.from_config(cfg, nqp // cfg.S)
    nV = cfg.nV
    g_len = nV * 63 * nV * nqp
    one_rank = nqp * nV
    rc = lib.cmpc_coupled_validate(ctypes.byref(dims), 64, S_local, 0, g_len, one_rank)
    assert rc == -1
    assert b"du_all" in lib.cmpc_last_error()
    rc = lib.cmpc_coupled_validate(ctypes.byref(dims), 64, S_local, 0, g_len - 1, 64 * Bsc * nV)
    assert rc == -1 and b"G_ext" in lib.cmpc_last_error()
    assert lib.cmpc_coupled_validate(ctypes.byref(dims), 64, S_local, 0, g_len, 64 * Bsc * nV) == 0
    assert lib.cmpc_coupled_validate(ctypes.byref(dims), 8, S_local, 0, nV * 7 * nV * nqp, one_rank) == 0
    assert lib.cmpc_coupled_validate(ctypes.byref(dims), 64, S_local, 64, g_len, 64 * Bsc * nV) == -1


# ---- GPU: the product kernel -----------------------------------------------

def product_rank(rank, world, group_gather=None, S_total=S_TOTAL, Bn=B):
    import torch
    import cmpc
    from cmpc.coupled import CoupledRank
    from cmpc.configs import reference_setup
    from cmpc.synthetic import synthetic_batch
    # the inputs of problem() (its oracle QPs are not needed here)
    cfg = cmpc.reference_config("par", "coop", p=20)
    arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
    lin, u_old, _, _ = synthetic_batch(cfg, Bn * S_total // cfg.S, seed=12)
    sl = S_total // world
    glob = [b * S_total + rank * sl + i for b in range(Bn) for i in range(sl)]
    ctx = cmpc.Context(cfg, len(glob) // cfg.S, device=0)
    ctx.configure(arr)
    # one build kernel for every sharding: AUTO picks by batch size, and the
    # two kernels agree to 1e-11, not bit for bit (test_gpu_parity.py)
    ctx.set_build_variant(cmpc.CMPC_BUILD_ROWS)
    ctx.set_state(np.ascontiguousarray(u_old[glob]), np.zeros((len(glob), cfg.nV)),
                  np.zeros(len(glob), np.uint32))
    ctx.upload_lin(np.ascontiguousarray(lin[glob]))
    ctx.build()
    Hd, fd, Gd = ctx.download_qp()
    Gx = torch.from_numpy(synthetic_g_ext(Gd, S_total, sl, rank * sl)).cuda()
    cr = CoupledRank(ctx, S_total, sl, rank, world, Gx)
    cr.step(K)
    torch.cuda.synchronize()
    return cfg, arr, ctx, cr, Hd, fd, Gd, u_old[glob]


@pytest.mark.gpu
def test_gpu_coupled_kernel_equals_oracle_loop():
    cfg, arr, ctx, cr, Hd, fd, Gd, u_g = product_rank(0, 1)
    du_gpu = cr.du_local.cpu().numpy()
    # the oracle loop on the product's own QPs
    n = len(u_g)
    glob = list(range(n))
    H = np.zeros((n, 4, 4)); f = np.zeros((n, 4)); G = np.zeros((n, 4, 4))
    H[:], f[:], G[:] = Hd, fd, Gd
    ref = oracle_loop(cfg, arr, H, f, G, np.ascontiguousarray(u_g), 0, 1, lambda d: d[None])
    ctx.close()
    assert np.array_equal(du_gpu, ref)


def _gpu_worker(rank, world, port, q, S_total=S_TOTAL, Bn=B):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, _, ctx, cr, *_ = product_rank(rank, world, S_total=S_total, Bn=Bn)
        parts = [torch.zeros(cr.du_local.shape, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, cr.du_local.cpu())
        if rank == 0:
            q.put(torch.stack(parts).numpy())
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_coupled_two_ranks_equal_one():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = q.get(timeout=600)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    *_, ctx1, cr1, _, _, _, _ = product_rank(0, 1)
    one = cr1.du_local.cpu().numpy()
    ctx1.close()
    sl = S_TOTAL // world
    got = got.reshape(world, B, sl, 4).transpose(1, 0, 2, 3).reshape(-1, 4)
    assert np.array_equal(got, one)


@pytest.mark.gpu
def test_gpu_coupled_config4_partition_eight_ranks_equal_one():
    """SURVEY config 4's own partition through the product kernel: 8 gloo
    ranks on the one GPU, each a CoupledRank with S_local = 8 of S_total = 64
    sub-controllers (s_offset = 8 r: every rank offset 0 ... 56, rank-major
    plan indexing over 8 ranks in cmpc_coupled_iterate), 256 scenarios, the
    plans all-gathered once per Jacobi iteration (the exchange that replaces
    include/nerve_center.h:280-285): bit-exact with one process running all
    64 sub-controllers."""
    world, S_total, Bn = 8, 64, 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gpu_worker, args=(r, world, port, q, S_total, Bn)) for r in range(world)]
    for p in ps:
        p.start()
    got = q.get(timeout=600)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    *_, ctx1, cr1, _, _, _, _ = product_rank(0, 1, S_total=S_total, Bn=Bn)
    one = cr1.du_local.cpu().numpy()
    ctx1.close()
    sl = S_total // world
    got = got.reshape(world, Bn, sl, 4).transpose(1, 0, 2, 3).reshape(-1, 4)
    assert np.array_equal(got, one)
    assert np.abs(one).max() > 0


@pytest.mark.gpu
def test_gpu_config4_full_size_matches_oracle():
    """SURVEY config 4 at its real size on one GPU: 64 sub-controllers per
    scenario (p = 50 coop QPs, synthetic coupling), 4 096 scenarios
    (262 144 QPs, 2.1 GB of G_ext), K = 9 Jacobi iterations through
    CoupledRank (world size 1).  Every QP's status over the whole batch,
    and 16 whole scenarios (1 024 QPs) bit-exact against the oracle's loop
    on the product's own QPs (same f_k summation order, or_qp_solve)."""
    import torch
    import cmpc
    from cmpc.configs import reference_setup
    from cmpc.coupled import CoupledRank
    from cmpc.synthetic import synthetic_batch
    S_total, Bsc, K4 = 64, 4096, 9
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
    nqp = Bsc * S_total
    lin, u_old, _, _ = synthetic_batch(cfg, nqp // cfg.S, seed=64, n_distinct=1024)
    ctx = cmpc.Context(cfg, nqp // cfg.S, device=0)
    try:
        ctx.configure(arr)
        ctx.set_state(u_old, np.zeros((nqp, cfg.nV)), np.zeros(nqp, np.uint32))
        ctx.upload_lin(lin)
        ctx.build()
        H, f, G = ctx.download_qp()
        Gx_host = synthetic_g_ext(G, S_total, S_total, 0)           # (4 * 63 * 4, nqp)
        Gx = torch.from_numpy(Gx_host).cuda()
        cr = CoupledRank(ctx, S_total, S_total, 0, 1, Gx)
        cr.step(K4)
        torch.cuda.synchronize()
        du_gpu = cr.du_local.cpu().numpy()
        _, st, nw = ctx.download()
        _, _, ws_gpu = ctx.get_state()
    finally:
        ctx.close()
    print("config 4: QPs", nqp, "status OK", (st == 0).mean(), "with active constraints",
          (ws_gpu != 0).mean())
    assert (st == 0).mean() > 0.999
    # 16 whole scenarios through the oracle's loop (vectorised over the
    # sample's QPs, the kernel's summation order j, then a, then v)
    sample = np.linspace(0, Bsc - 1, 16).astype(int)
    qs = (sample[:, None] * S_total + np.arange(S_total)[None, :]).reshape(-1)
    G3 = Gx_host.reshape(4, (S_total - 1) * 4, nqp)[:, :, qs]      # (4, 252, nq_s)
    nu = cfg.nu
    ws = np.zeros(len(qs), np.uint32)
    st_o = np.zeros(len(qs), np.int32)
    prev = np.zeros((len(sample), S_total, 4))
    for k in range(K4):
        fk = f[qs].copy()
        for s in range(S_total):
            rows = np.arange(len(sample)) * S_total + s
            jj = 0
            for j in range(S_total):
                if j == s:
                    continue
                for a in range(4):
                    for v in range(4):
                        fk[rows, a] = fk[rows, a] + G3[a, jj * 4 + v, rows] * prev[:, j, v]
                jj += 1
        new = np.zeros_like(prev)
        for i, q in enumerate(qs):
            s_cfg = q % cfg.S
            lo = np.tile(arr.lower[s_cfg] - u_old[q, :nu], 2)
            up = np.tile(arr.upper[s_cfg] - u_old[q, :nu], 2)
            x, info = O.qp_solve(H[q], fk[i], lo, up, np.tile(arr.rate_lower[s_cfg], 2),
                                 np.tile(arr.rate_upper[s_cfg], 2), nu, int(ws[i]))
            ws[i] = info.ws
            st_o[i] = info.status
            new[i // S_total, i % S_total] = x
        prev = new
    assert np.array_equal(st[qs], st_o)
    assert np.array_equal(ws_gpu[qs], ws)
    assert np.array_equal(du_gpu[qs], prev.reshape(-1, 4))


@pytest.mark.gpu
def test_gpu_coupled_pipeline_tiles_equal_one():
    """CoupledPipeline (bench.py's config-4 section): the rank's scenarios as
    two tiles on their own streams, each tile's gather overlapping the other
    tile's iteration, give bit for bit the plans, statuses and working sets
    of one CoupledRank over all scenarios (two steps, K = 9)."""
    import torch
    import cmpc
    from cmpc.configs import reference_setup
    from cmpc.coupled import CoupledPipeline, make_coupled_tiles
    from cmpc.synthetic import synthetic_batch
    S_total, Bsc, K4 = 8, 512, 9
    cfg = cmpc.reference_config("par", "coop", p=50)
    arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
    lin, u_old, _, _ = synthetic_batch(cfg, Bsc * S_total // cfg.S, seed=88, n_distinct=256)
    res = []
    for tiles in (1, 2):
        crs, streams = make_coupled_tiles(cfg, arr, lin, u_old, S_total, S_total, 0, 1, 0, tiles,
                                          build_variant=cmpc.CMPC_BUILD_ROWS)
        try:
            pipe = CoupledPipeline(crs, streams)
            pipe.step(K4)
            pipe.step(K4)
            torch.cuda.synchronize()
            du = np.concatenate([c.du_local.cpu().numpy() for c in crs])
            st = np.concatenate([c.ctx.download()[1] for c in crs])
            ws = np.concatenate([c.ctx.get_state()[2] for c in crs])
        finally:
            for c in crs:
                c.ctx.close()
        res.append((du, st, ws))
    assert (res[0][1] == 0).mean() > 0.999
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)


def test_coupled_rank_rejects_layout_beyond_gathered_plans():
    """The coupled kernel reads the plans of all S_total sub-controllers from
    du_all [S_total / S_local ranks]: a CoupledRank whose world does not
    cover S_total (e.g. S_total = 64 with S_local = 8 on one rank) is refused
    on the host before any launch."""
    from cmpc.coupled import CoupledRank

    class _Ctx:
        B = 8
        cfg = type("cfg", (), {"S": 2, "nV": 4})()

    with pytest.raises(ValueError, match="S_total"):
        CoupledRank(_Ctx(), 64, 8, 0, 1, None)
