#!/usr/bin/env python3
"""CPU emulation of the row build kernel's hand-off protocol for one delayed
input (build_rows.hip, rows_layout.cpp): the writer of step t stores entry
m - 1 + t of the line (or of the ring of D + m entries, stepping back at each
wrap), the move-k gather reader of step s >= D reads entry (m - 1 - k) + s - D,
with the kernel's segment bounds (D, p - D, the wraps) and its unrolled
blocks.  Checks that every read returns h_{s-k-D} (zero before the line
starts) for horizons up to the 16-bound limit.  Used by tests/test_abi.py."""
import os
import re

# the kernel's horizon unroll (CMPC_ROWS_U, cmpc_internal.h)
KERNEL_U = int(re.search(r"#define CMPC_ROWS_U (\d+)", open(os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "..", "compressor-mpc_amd", "csrc",
    "cmpc_internal.h")).read()).group(1))


def check(p, D, M=2, U=KERNEL_U):
    full = (M - 1) + max(0, p - D)
    ring = D + M if full > D + M else 0
    L = ring if ring else full
    mem = [None] * L
    for e in range(M - 1):
        mem[e] = 0.0  # history zeros
    segs = set()

    def add(v):
        if 0 < v < p:
            segs.add(v)
    add(D)
    add(p - D)
    if ring:
        t = ring - (M - 1)
        while t < p - D:
            add(t)
            t += ring
        for k in range(M):
            t = ring + D - (M - 1 - k)
            while t < p:
                add(t)
                t += ring
    segs = sorted(segs)
    wq = (M - 1) if p - D > 0 else None
    winc = 1 if p - D > 0 else 0
    wsw = p - D if p - D > 0 else -1
    wwr = ring - (M - 1) if ring else -1
    rq = {k: None for k in range(M)}  # None: the zero area
    rinc = {k: 0 for k in range(M)}
    rwr = {k: (ring + D - (M - 1 - k)) if ring else -1 for k in range(M)}
    errs = 0
    r = 0

    def step(u):
        nonlocal errs
        t = r + u
        if wq is not None:
            idx = wq + u * winc
            if not 0 <= idx < L:
                raise IndexError(("write", p, D, t, idx))
            mem[idx] = t
        for k in range(M):
            want = t - k - D
            if rq[k] is None:
                got = 0.0
            else:
                idx = rq[k] + u * rinc[k]
                if not 0 <= idx < L:
                    raise IndexError(("read", p, D, t, k, idx))
                got = mem[idx]
            if got != (want if want >= 0 else 0.0):
                errs += 1

    for sg in range(len(segs) + 1):
        r_end = segs[sg] if sg < len(segs) else p
        while r + U <= r_end:
            for u in range(U):
                step(u)
            if wq is not None:
                wq += U * winc
            for k in range(M):
                if rq[k] is not None:
                    rq[k] += U * rinc[k]
            r += U
        while U > 2 and r + 2 <= r_end:  # the two-step remainder blocks
            step(0)
            step(1)
            if wq is not None:
                wq += 2 * winc
            for k in range(M):
                if rq[k] is not None:
                    rq[k] += 2 * rinc[k]
            r += 2
        while r < r_end:
            step(0)
            if wq is not None:
                wq += winc
            for k in range(M):
                if rq[k] is not None:
                    rq[k] += rinc[k]
            r += 1
        for k in range(M):
            if r == D:
                rq[k], rinc[k] = M - 1 - k, 1
            if r == rwr[k]:
                rq[k] -= ring
                rwr[k] += ring
        if r == wwr:
            wq -= ring
            wwr += ring
        if r == wsw:
            wq, winc, wwr = None, 0, -1
    return errs, ring, len(segs)


if __name__ == "__main__":
    for p in (20, 50, 81, 82, 83, 100, 120, 200, 250):
        print(p, check(p, 40))
