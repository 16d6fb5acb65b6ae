"""Scenario sharding across ranks (one process per GPU).

The north-star workload is many independent scenarios of a 2-sub-controller
cooperative plant.  Its only exchange (the Jacobi plan exchange, nerve_center.h
:280-285) is between the S sub-controllers of one scenario.  Those sit in
adjacent QP slots q = b*S + s of one rank and exchange by lane shuffles inside
the solve kernel.  Ranks therefore own whole scenarios and need no data-path
collective.  torch.distributed is used only for:
- the timing barrier and the max over ranks;
- gathering results for verification.
"""
from typing import Tuple

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of scenarios [start, start + count) owned by rank.
    Sizes differ by at most one; every scenario is owned exactly once."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError((world, rank))
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def qp_slice(start: int, count: int, S: int) -> slice:
    """QP slots of scenarios [start, start + count) (scenario-major layout)."""
    return slice(start * S, (start + count) * S)


def shard_arrays(rank: int, world: int, S: int, *arrays):
    """Per-rank views of scenario-major per-QP arrays (leading dim = B*S)."""
    n_qp = arrays[0].shape[0]
    if n_qp % S:
        raise ValueError("leading dimension must be a multiple of S")
    start, count = shard_range(n_qp // S, world, rank)
    sl = qp_slice(start, count, S)
    return tuple(np.ascontiguousarray(a[sl]) for a in arrays)


def gather_to_all(local: np.ndarray, n_total_qp: int, S: int, group=None) -> np.ndarray:
    """All-gather the per-rank per-QP results into the global scenario-major
    array.  On gloo the exchange runs on host tensors; on nccl (RCCL) the
    padded shard and the receive buffers are placed on the rank's current GPU
    and the result is copied back to the host."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    B = n_total_qp // S
    counts = [shard_range(B, world, r)[1] * S for r in range(world)]
    maxc = max(counts)
    dev = (torch.device("cuda", torch.cuda.current_device())
           if dist.get_backend(group) == "nccl" else torch.device("cpu"))
    t = torch.from_numpy(np.ascontiguousarray(local))
    pad = torch.zeros((maxc,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
    pad[: t.shape[0]] = t.to(dev)
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return np.concatenate([o[:c].cpu().numpy() for o, c in zip(outs, counts)], axis=0)
