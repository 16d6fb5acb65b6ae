#!/usr/bin/env python3
"""Config-4 coupled bench section alone (world 1, S_local = S_total = 8,
B = 4096, K = 9), for a kernel trace: python tools/coupled_once.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "compressor-mpc_amd"))
from cmpc.coupled import run_coupled_bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
r = run_coupled_bench(0, 1, 0, S_local=8, B=4096, K=9, steps=steps)
r["ms_per_step"] = r["elapsed_s"] / r["steps"] * 1e3
print(json.dumps(r))
