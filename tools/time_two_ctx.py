#!/usr/bin/env python3
"""Step throughput with the bench's batch rotation spread over N contexts
(each on its own HIP stream), so that one batch's iterate can run beside the
next batch's build.  Batch b is always stepped by context b % N, so a batch's
state is only touched in order on one stream.

usage: python tools/time_two_ctx.py [N_CTX ...]   (default: 1 2)
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "compressor-mpc_amd"))
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402


def main():
    ncs = [int(a) for a in sys.argv[1:]] or [1, 2]
    cfg = cmpc.reference_config("par", "coop", p=50)
    arrays = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
    B, S, K, NB = 65536, cfg.S, 9, 4
    batches, states0 = [], []
    for b in range(NB):
        lin, u, du, w = synthetic_batch(cfg, B, seed=1002 + 101 * 0 + b, n_distinct=min(B, 2048))
        batches.append(torch.from_numpy(lin).cuda())
        states0.append(tuple(torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (u, du, w.view(np.int32))))
    results = {}
    for nc in ncs:
        states = [tuple(a.clone() for a in st) for st in states0]
        torch.cuda.synchronize()
        ctxs = []
        for _ in range(nc):
            c = cmpc.Context(cfg, B, device=0)
            c.configure(arrays)
            ctxs.append(c)

        def step(i, flags=cmpc.CMPC_APPLY_MOVE):
            b = i % NB
            c = ctxs[b % nc]
            c.bind_lin(batches[b].data_ptr())
            c.bind_state(*(a.data_ptr() for a in states[b]))
            c.step(K, flags)

        for b in range(NB):
            c = ctxs[b % nc]
            c.bind_lin(batches[b].data_ptr())
            c.bind_state(*(a.data_ptr() for a in states[b]))
            c.build()
            c.init_warmstart()
        for c in ctxs:
            c.synchronize()
        for n in range(400):  # clock settle (a fixed count: the states stay comparable)
            step(n, 0)
        for c in ctxs:
            c.synchronize()
        for rep in range(3):
            t0 = time.perf_counter()
            steps = 200
            for i in range(steps):
                step(i)
            for c in ctxs:
                c.synchronize()
            dt = (time.perf_counter() - t0) / steps
            print(f"contexts {nc} rep {rep}: {dt * 1e3:.4f} ms/step  {B * S * K / dt:.4e} QP/s", flush=True)
        results[nc] = [torch.cat([a.flatten().double() for a in st]).cpu() for st in states]
        for c in ctxs:
            c.close()
    if len(results) > 1:
        ks = list(results)
        same = all(torch.equal(x, y) for x, y in zip(results[ks[0]], results[ks[1]]))
        print("states after the same steps bit-identical across context counts:", same)


if __name__ == "__main__":
    main()
