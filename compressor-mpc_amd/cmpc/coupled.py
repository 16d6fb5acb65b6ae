"""Sub-controller-sharded cooperative MPC.

S_total sub-controllers per scenario; each rank (one per GPU) owns S_local of
them for all its scenarios.  The cooperative iteration's exchange
(nerve_center.h:280-285: every sub-controller reads every other one's move
plan) is an all-gather of the plans once per Jacobi iteration, over RCCL
(torch.distributed "nccl") on GPUs, or gloo on CPU.

The reference's plants have two compressors, so a 64-sub-controller system is
synthetic.
- Each sub-controller's own QP (H, f) is the coop p=50 QP of a 2-compressor
  plant built by cmpc_build.
- Its coupling to the other S_total - 1 sub-controllers is a dense
  G_ext = [w_{s,1} G, ..., w_{s,S_total-1} G]. Here G is the real 4x4
  Su'W Su_other of its own build. The weights decay with ring distance,
  w = rho^d (1 + 0.1 * sin(1.7 b + 2.3 s + 3.1 j)), which is deterministic in
  (scenario, s, j) and independent of the rank layout.
"""
import ctypes

import numpy as np

RHO = 0.5


def coupling_weights(b, s, S_total: int) -> np.ndarray:
    """w_{s,j} for the S_total - 1 other sub-controllers j (global order);
    b, s may be arrays (broadcast over a leading axis)."""
    b = np.asarray(b)[..., None]
    s = np.asarray(s)[..., None]
    j = np.arange(S_total)
    d = np.minimum(np.abs(j - s), S_total - np.abs(j - s))
    w = RHO ** d * (1.0 + 0.1 * np.sin(1.7 * b + 2.3 * s + 3.1 * j))
    keep = j != s
    return w[keep].reshape(w.shape[:-1] + (S_total - 1,))


def synthetic_g_ext(G_local: np.ndarray, S_total: int, S_local: int, s_offset: int,
                    b_offset: int = 0) -> np.ndarray:
    """Element-major G_ext [nV*(S_total-1)*nV][nqp] for this rank's QPs
    (q = b*S_local + local index, scenarios b_offset + b for a tile of the
    rank's scenarios).  G_local: (nqp, nV, nVo=nV) from the build."""
    nqp, nV, _ = G_local.shape
    q = np.arange(nqp)
    b, sl = b_offset + q // S_local, q % S_local
    w = coupling_weights(b, s_offset + sl, S_total)            # (nqp, S_total-1)
    out = np.einsum("qj,qav->ajvq", w, G_local)                # (nV, S_total-1, nV, nqp)
    return np.ascontiguousarray(out.reshape(nV * (S_total - 1) * nV, nqp))


def others(du_all: np.ndarray, b: int, s: int, S_total: int, S_local: int) -> np.ndarray:
    """du_other of global sub-controller s of scenario b from rank-major
    gathered plans du_all [world][B][S_local][nV] (as the kernel reads them)."""
    rows = []
    for j in range(S_total):
        if j == s:
            continue
        r, sl = divmod(j, S_local)
        rows.append(du_all[r, b, sl])
    return np.concatenate(rows)


def coupled_jacobi(K: int, solve_iteration, gather, du_local0):
    """The cooperative loop of one control step: K times, gather every
    rank's current plans (du_local: this rank's [nqp, nV]) and run one
    Jacobi iteration on the local QPs.  solve_iteration(du_all, apply_move)
    returns the new local plans."""
    du_local = du_local0
    for k in range(K):
        du_all = gather(du_local)
        du_local = solve_iteration(du_all, k == K - 1)
    return du_local


class CoupledRank:
    """One rank of the sharded loop on its GPU: a cmpc.Context holding this
    rank's B scenarios x S_local sub-controllers (coop dims, S = 2 setup),
    G_ext, the local and gathered plan buffers, and the RCCL all-gather."""

    def __init__(self, ctx, S_total: int, S_local: int, rank: int, world: int, G_ext, group=None,
                 force_collective: bool = False):
        import torch
        self.torch = torch
        self.ctx, self.S_total, self.S_local = ctx, S_total, S_local
        self.rank, self.world, self.group = rank, world, group
        # world size 1 copies the plans locally unless told to run the
        # collective (a one-rank RCCL communicator: the multi-GPU code path)
        self.force_collective = force_collective
        self.s_offset = rank * S_local
        nqp = ctx.B * ctx.cfg.S
        if nqp % S_local:
            raise ValueError("B*S must be a multiple of S_local")
        # the kernel reads every other sub-controller's plan from du_all
        # [S_total / S_local ranks][nqp][nV]: a layout with fewer ranks than
        # that would read past the gathered plans
        if S_local * world != S_total:
            raise ValueError(f"S_total ({S_total}) must be S_local ({S_local}) x world ({world})")
        self.B = nqp // S_local
        nV = ctx.cfg.nV
        dev = G_ext.device
        self.G_ext = G_ext
        # world size 1 without the collective: the plans ping-pong between two
        # buffers (an iteration reads the one the previous iteration wrote and
        # writes the other), so no gather copy is needed.  A kernel may not
        # read and write the same plan buffer: its waves run side by side.
        self.local_only = world == 1 and not force_collective
        self._plans = [torch.zeros(nqp, nV, dtype=torch.float64, device=dev)
                       for _ in range(2 if self.local_only else 1)]
        self._cur = 0  # the buffer holding the current plans
        self._all = (None if self.local_only else
                     torch.zeros(world, nqp, nV, dtype=torch.float64, device=dev))
        # one stream for the library and torch's collectives
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)

    @property
    def du_local(self):
        """This rank's current plans [nqp][nV] (the next gather's input)."""
        return self._plans[self._cur]

    @property
    def du_all(self):
        """The gathered plans [world][nqp][nV] the next iteration reads."""
        if self.local_only:
            return self._plans[self._cur].view(1, *self._plans[self._cur].shape)
        return self._all

    def gather(self):
        import torch.distributed as dist
        if self.local_only:  # the current plans are the gathered ones
            return
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(self._all, self.du_local, group=self.group)
        else:  # gloo: CPU staging
            parts = [self.torch.zeros_like(self.du_local, device="cpu") for _ in range(self.world)]
            dist.all_gather(parts, self.du_local.cpu(), group=self.group)
            self._all.copy_(self.torch.stack(parts))

    def iterate(self, apply_move: bool):
        from . import CMPC_APPLY_MOVE
        from ._abi import check
        lib = self.ctx.lib
        src = self.du_all
        nxt = 1 - self._cur if self.local_only else self._cur
        out = self._plans[nxt]
        check(lib.cmpc_coupled_iterate(
            self.ctx._h, self.S_total, self.S_local, self.s_offset,
            ctypes.c_void_p(self.G_ext.data_ptr()), self.G_ext.numel(),
            ctypes.c_void_p(src.data_ptr()), src.numel(),
            ctypes.c_void_p(out.data_ptr()), CMPC_APPLY_MOVE if apply_move else 0),
            "cmpc_coupled_iterate")
        self._cur = nxt

    def step(self, K: int):
        """build + K gathered Jacobi iterations (the first move applied)."""
        self.ctx.build()
        for k in range(K):
            self.gather()
            self.iterate(k == K - 1)


class CoupledPipeline:
    """One rank's share split into scenario tiles, each a CoupledRank on its
    own context and HIP stream (overlap the gather with the
    next scenario tile's solve).  Iteration k runs tile by tile: the
    all-gather of tile t waits only for tile t's previous iteration, so it
    overlaps the coupled iteration of the tile before it, and the tiles'
    kernels may run side by side.  Every rank issues the collectives in the
    same order (tile-major within an iteration).  The tiles are independent
    sets of scenarios: the results equal one CoupledRank over all of them."""

    def __init__(self, tiles, streams):
        self.tiles, self.streams = tiles, streams

    def step(self, K: int):
        import torch
        for cr, s in zip(self.tiles, self.streams):
            with torch.cuda.stream(s):
                cr.ctx.build()
        for k in range(K):
            for cr, s in zip(self.tiles, self.streams):
                with torch.cuda.stream(s):
                    cr.gather()
                    cr.iterate(k == K - 1)


def make_coupled_tiles(cfg, arr, lin, u_old, S_total: int, S_local: int, rank: int, world: int,
                       device: int, tiles: int, group=None, force_collective: bool = False,
                       build_variant: int = 0):
    """Contexts, G_ext and CoupledRanks for `tiles` scenario tiles of one
    rank's records (lin, u_old: B*S_local rows, q = b*S_local + i), each on
    its own stream; build + warm-start initialisation done.  build_variant
    (cmpc_set_build_variant) pins the build kernel: AUTO picks it by batch
    size, and the two kernels' H, f, G differ in rounding."""
    import torch

    from . import Context
    nqp = lin.shape[0]
    B = nqp // S_local
    if B % tiles:
        raise ValueError("the rank's scenarios must split evenly into tiles")
    bt = B // tiles
    dev = f"cuda:{device}"
    out, streams = [], []
    for t in range(tiles):
        rows = slice(t * bt * S_local, (t + 1) * bt * S_local)
        s = torch.cuda.Stream(device=device) if tiles > 1 else torch.cuda.current_stream(device)
        ctx = Context(cfg, bt * S_local // cfg.S, device=device)
        try:
            ctx.configure(arr)
            if build_variant:
                ctx.set_build_variant(build_variant)
            n = bt * S_local
            ctx.set_state(np.ascontiguousarray(u_old[rows]), np.zeros((n, cfg.nV)), np.zeros(n, np.uint32))
            ctx.upload_lin(np.ascontiguousarray(lin[rows]))
            ctx.build()
            ctx.init_warmstart()
            _, _, G = ctx.download_qp()
            G_ext = torch.from_numpy(synthetic_g_ext(G, S_total, S_local, rank * S_local, t * bt)).to(dev)
            # the copy ran on the current stream; the tile's stream reads G_ext
            s.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(s):
                out.append(CoupledRank(ctx, S_total, S_local, rank, world, G_ext, group=group,
                                       force_collective=force_collective))
        except Exception:
            ctx.close()
            for cr in out:
                cr.ctx.close()
            raise
        streams.append(s)
    return out, streams


def run_coupled_bench(rank: int, world: int, device: int, S_local: int = 8, B: int = 4096, p: int = 50,
                      K: int = 9, steps: int = 20, warmup: int = 3, settle_seconds: float = 0.25,
                      S_total: int = 0, group=None, force_collective: bool = False,
                      tiles: int = 1) -> dict:
    """SURVEY config 4 on this rank: B scenarios x S_local sub-controllers
    (global indices rank * S_local + i of S_total = S_local * world), one
    step = build + K x (all-gather of the plans, coupled Jacobi iteration),
    the first move applied in the last iteration; with tiles > 1 the
    scenarios run as that many tiles on their own streams, each tile's
    gather overlapping another tile's iteration (CoupledPipeline).  The
    caller has set up the process group (nccl = RCCL over xGMI between GPUs)
    when world > 1.  Returns this rank's timings; the whole-job value needs
    the max over ranks of `elapsed_s` (the caller's barrier + all-reduce)."""
    import time

    import torch
    import torch.distributed as dist

    from . import controller_arrays, reference_config
    from .configs import reference_setup
    from .synthetic import synthetic_batch

    S_total = S_total or S_local * world
    cfg = reference_config("par", "coop", p=p)
    arr = controller_arrays(cfg, reference_setup("par", "coop"))
    nqp = B * S_local
    collective = world > 1 or force_collective
    crs, streams, err = [], [], None
    try:
        lin, u_old, _, _ = synthetic_batch(cfg, nqp // cfg.S, seed=500 + rank, n_distinct=1024)
        crs, streams = make_coupled_tiles(cfg, arr, lin, u_old, S_total, S_local, rank, world, device,
                                          tiles, group=group, force_collective=force_collective)
    except Exception as e:  # noqa: BLE001 -- agreed on below, then re-raised
        err = e
    if collective:
        # every rank agrees that its set-up succeeded before the first
        # collective of the timed section: a rank that failed alone would
        # otherwise leave its peers waiting in (or mis-pairing) the gathers
        on_gpu = dist.get_backend(group) == "nccl"
        ok = torch.tensor([0 if err else 1], dtype=torch.int32,
                          device=f"cuda:{device}" if on_gpu else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
        if int(ok.item()) == 0 and err is None:
            err = RuntimeError("coupled section: set-up failed on another rank")
    if err is not None:
        for c in crs:
            c.ctx.close()
        raise err
    try:
        cr = CoupledPipeline(crs, streams)
        for _ in range(warmup):
            cr.step(K)
        torch.cuda.synchronize(device)
        t_end = time.perf_counter() + settle_seconds
        while time.perf_counter() < t_end:
            cr.step(K)
            torch.cuda.synchronize(device)
        if world > 1 or force_collective:
            dist.barrier(group=group)
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(steps):
            cr.step(K)
        torch.cuda.synchronize(device)
        elapsed = time.perf_counter() - t0
        # the exchange alone: events around each tile's gathers (on its
        # stream) in a second pass; summed over the tiles per iteration
        ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(K)] for _ in crs]
        for c, s in zip(crs, streams):
            with torch.cuda.stream(s):
                c.ctx.build()
        for k in range(K):
            for t, (c, s) in enumerate(zip(crs, streams)):
                with torch.cuda.stream(s):
                    ev[t][k][0].record()
                    c.gather()
                    ev[t][k][1].record()
                    c.iterate(k == K - 1)
        torch.cuda.synchronize(device)
        gather_ms = sum(a.elapsed_time(b) for et in ev for a, b in et) / K
        # the coupled iterate kernel alone (library events on its stream), a
        # third pass: G_ext's HBM fraction
        from . import CMPC_KERNEL_ITERATE
        for c in crs:
            c.ctx.enable_timing(True, only=(CMPC_KERNEL_ITERATE,))
        for _ in range(max(1, steps // 2)):
            cr.step(K)
        torch.cuda.synchronize(device)
        it = [c.ctx.kernel_time(CMPC_KERNEL_ITERATE) for c in crs]
        for c in crs:
            c.ctx.enable_timing(False)
        iterate_ms = sum(ms / max(n, 1) for ms, n in it)  # per iteration, summed over the tiles
        g_bytes = sum(c.G_ext.numel() for c in crs) * 8
        st = np.concatenate([c.ctx.download()[1] for c in crs])
        return {"elapsed_s": elapsed, "steps": steps, "qp_per_gpu": nqp, "S_total": S_total,
                "S_local": S_local, "B": B, "p": p, "K": K, "tiles": tiles,
                "G_ext_MB_per_gpu": g_bytes / 1e6,
                "gather_ms_per_iteration": gather_ms,
                "gather_bytes_per_iteration": world * nqp * cfg.nV * 8,
                "iterate_kernel_ms": iterate_ms,
                "G_ext_hbm_GBs": g_bytes / (iterate_ms * 1e-3) / 1e9 if iterate_ms > 0 else None,
                "G_ext_hbm_frac": g_bytes / (iterate_ms * 1e-3) / 8e12 if iterate_ms > 0 else None,
                "qp_status_ok_fraction": float((st == 0).mean())}
    finally:
        for c in crs:
            c.ctx.close()
