#!/usr/bin/env python3
"""Random search over the row kernel's LDS paddings with the bank model of
tools/lds_rows_sim.py, under the 4-workgroups-per-CU LDS budget."""
import json
import random
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from lds_rows_sim import PAR_COOP, layout, simulate  # noqa: E402

p = int(sys.argv[1]) if len(sys.argv) > 1 else 50
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
budget = int(sys.argv[3]) if len(sys.argv) > 3 else 40960
d = dict(PAR_COOP, p=p)
keys = ["pad_0", "pad_1", "pad_2", "pad_3", "pad_dump", "pad_z", "pad_zr", "pad_LQ", "pad_yl", "pad_yls", "pad_w", "pad_WL"]
rng = random.Random(1)
best = ({}, simulate(d, layout(d), 0)[1])
print("baseline", best[1])
for it in range(n):
    over = dict(best[0])
    for k in rng.sample(keys, rng.randint(1, 3)):
        over[k] = rng.randint(0, 15)
    if rng.random() < 0.3:
        o = list(range(4)); rng.shuffle(o); over["order"] = o
    L = layout(d, over)
    if L["bytes"] > budget:
        continue
    t = simulate(d, L, 0)[1]
    if t < best[1]:
        best = (over, t)
        print(it, round(t, 3), L["bytes"], json.dumps(over), flush=True)
        if t == 0:
            break
L = layout(d, best[0])
print("best", json.dumps(best[0]), "bytes", L["bytes"])
for w in range(4):
    print(w, simulate(d, L, w))
