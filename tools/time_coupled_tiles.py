#!/usr/bin/env python3
"""Config-4 coupled step on one GPU (world size 1, S_local = S_total = 8)
with 1, 2 and 4 scenario tiles (cmpc.coupled.CoupledPipeline).
usage: python tools/time_coupled_tiles.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "compressor-mpc_amd"))
from cmpc.coupled import run_coupled_bench  # noqa: E402

for S_total in (8,):
    for tiles in (1, 2, 4):
        r = run_coupled_bench(0, 1, 0, S_local=8, B=4096, K=9, steps=20, tiles=tiles)
        r["ms_per_step"] = r["elapsed_s"] / r["steps"] * 1e3
        print(json.dumps({k: r[k] for k in ("S_total", "tiles", "ms_per_step", "gather_ms_per_iteration",
                                            "qp_status_ok_fraction")}), flush=True)
