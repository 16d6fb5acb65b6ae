#!/usr/bin/env python3
"""cooperative MPC with S_total sub-controllers per
scenario, S_local per GPU, plans all-gathered over RCCL once per Jacobi
iteration (cmpc/coupled.py).  Launch with torch.distributed.run for N GPUs
(one rank per GPU); world size 1 runs the same loop with a local gather.

Prints one JSON line (rank 0): QP solves/s for the whole job and the time
split (build, coupled iterations, gathers)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--s-local", type=int, default=8, help="sub-controllers per GPU")
    ap.add_argument("--s-total", type=int, default=0, help="default: s_local * world")
    ap.add_argument("--batch", type=int, default=4096, help="scenarios")
    ap.add_argument("--p", type=int, default=50)
    ap.add_argument("--K", type=int, default=9)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-seconds", type=float, default=0.25)
    args = ap.parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import cmpc
    from cmpc.configs import reference_setup
    from cmpc.coupled import CoupledRank, synthetic_g_ext
    from cmpc.synthetic import synthetic_batch

    S_local = args.s_local
    S_total = args.s_total or S_local * world
    B, K = args.batch, args.K
    cfg = cmpc.reference_config("par", "coop", p=args.p)
    arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
    nqp = B * S_local
    lin, u_old, _, _ = synthetic_batch(cfg, nqp // cfg.S, seed=500 + rank, n_distinct=1024)
    ctx = cmpc.Context(cfg, nqp // cfg.S, device=local)
    ctx.configure(arr)
    ctx.set_state(u_old, np.zeros((nqp, cfg.nV)), np.zeros(nqp, np.uint32))
    ctx.upload_lin(lin)
    ctx.build()
    _, _, G = ctx.download_qp()
    G_ext = torch.from_numpy(synthetic_g_ext(G, S_total, S_local, rank * S_local)).to(f"cuda:{local}")
    cr = CoupledRank(ctx, S_total, S_local, rank, world, G_ext)
    for _ in range(args.warmup):
        cr.step(K)
    torch.cuda.synchronize()
    # settle: the clock ramps over the first ~40 ms of load (tools/time_clock_ramp.py)
    t_end = time.perf_counter() + args.settle_seconds
    while time.perf_counter() < t_end:
        cr.step(K)
        torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_gather = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.build()
        for k in range(K):
            tg = time.perf_counter()
            cr.gather()
            if rank == 0 and world > 1 and _ == 0:
                torch.cuda.synchronize()
                t_gather += time.perf_counter() - tg
            cr.iterate(k == K - 1)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        dist.barrier()
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    _, st, _ = ctx.download()
    out = {
        "metric": "QP solves/sec (whole job), cooperative MPC sharded by sub-controller",
        "value": world * nqp * K * args.steps / el, "unit": "QP solves/s", "n_gpus": world,
        "steps": args.steps, "ms_per_step": el / args.steps * 1e3,
        "config": {"workload": f"SURVEY config 4: {S_total} sub-controllers per scenario, "
                               f"{S_local} per GPU, {B} scenarios, p={args.p}, K={K}",
                   "S_total": S_total, "S_local": S_local, "B": B,
                   "G_ext_MB_per_gpu": G_ext.numel() * 8 / 1e6,
                   "exchange": "RCCL all_gather_into_tensor of B x S_local x nV plans per iteration"
                               if world > 1 else "local (world size 1)"},
        "first_step_gather_ms_total": t_gather * 1e3,
        "qp_status_ok_fraction": float((st == 0).mean()),
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
