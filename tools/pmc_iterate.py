"""The bench's step loop (4 resident batches, build + iterate(9)), for a PMC
pass on the iterate kernel: `move` applies the first move each step
(the bench's timed steps), `nomove` does not.  GPU only.
usage: rocprofv3 --pmc ... -- python3 tools/pmc_iterate.py move|nomove [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "move"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 24
B, NB = 65536, 4
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
recs, sts = [], []
for b in range(NB):
    lin, u, du, w = synthetic_batch(cfg, B, seed=1002 + b, n_distinct=2048)
    recs.append(torch.from_numpy(lin).cuda())
    sts.append(tuple(torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (u, du, w.view(np.int32))))
ctx = cmpc.Context(cfg, B)
ctx.configure(arr)


def bind(i):
    st = sts[i % NB]
    ctx.bind_lin(recs[i % NB].data_ptr())
    ctx.bind_state(st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr())


for b in range(NB):
    bind(b)
    ctx.build()
    ctx.init_warmstart()
for i in range(2 * NB):  # converge the warm starts (the bench's warmup)
    bind(i)
    ctx.step(9, 0)
flags = cmpc.CMPC_APPLY_MOVE if mode == "move" else 0
for i in range(steps):
    bind(i)
    ctx.step(9, flags)
ctx.synchronize()
ctx.close()
print("done", mode, steps)
