#!/usr/bin/env python3
"""Compare .dat records written by tools/run_closed_loop.py --out (on the GPU
box) with the reference's results/<plant>/run1/<cfg>.dat, line by line,
skipping the wall-time line of every record.  Runs in the build container
(reads /root/reference).  A line differs "only in zero residue" when its
tokens agree after mapping |v| < 1e-12 to 0 (the parallel plant's y[2]).

usage: python tools/diff_dat.py DIR   (DIR holds <par|ser>_<cfg>.dat)"""
import sys

CASES = [("par", "centralized", "parallel"), ("par", "coop9", "parallel"), ("par", "ncoop9", "parallel"),
         ("ser", "centralized", "serial"), ("ser", "coop9", "serial"), ("ser", "ncoop9", "serial")]


def norm(line):
    return ["0" if abs(float(t)) < 1e-12 else t for t in line.split()]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dat"
    for p, c, full in CASES:
        a = open(f"{d}/{p}_{c}.dat").read().split("\n")
        b = open(f"/root/reference/results/{full}/run1/{c}.dat").read().split("\n")
        diff = [i for i in range(min(len(a), len(b))) if i % 6 != 4 and a[i] != b[i]]
        real = [i for i in diff if norm(a[i]) != norm(b[i])]
        print(f"{p}_{c}: lines {len(a)} / {len(b)}; differing (wall time skipped) {len(diff)}; "
              f"beyond zero residue {len(real)}" + (f"; first {real[0]}: {a[real[0]]!r} vs {b[real[0]]!r}"
                                                    if real else ""))


if __name__ == "__main__":
    main()
