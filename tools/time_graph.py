"""Step time with plain launches vs a HIP graph of the step (build + iterate)
captured through torch.cuda.graph on the context's stream, one graph per
input batch.  usage: python tools/time_graph.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))
import torch  # noqa: E402
import cmpc  # noqa: E402
from cmpc.configs import reference_setup  # noqa: E402
from cmpc.synthetic import synthetic_batch  # noqa: E402

B, K, NB, STEPS = 65536, 9, 4, 200
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
batches = []
for b in range(NB):
    lin, u, du, ws = synthetic_batch(cfg, B, seed=1002 + b, n_distinct=2048)
    if b == 0:
        u0, du0, ws0 = u, du, ws
    batches.append(torch.from_numpy(lin).cuda())
s = torch.cuda.Stream()
with cmpc.Context(cfg, B) as ctx:
    ctx.set_stream(s.cuda_stream)
    ctx.configure(arr)
    ctx.set_state(u0, du0, ws0)
    ctx.bind_lin(batches[0].data_ptr())
    ctx.build()
    ctx.init_warmstart()
    ctx.synchronize()

    def plain(n, i0=0):
        for i in range(n):
            ctx.bind_lin(batches[(i0 + i) % NB].data_ptr())
            ctx.step(K, 0)
        ctx.synchronize()

    plain(16)
    graphs = []
    with torch.cuda.stream(s):
        for b in range(NB):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                ctx.bind_lin(batches[b].data_ptr())
                ctx.step(K, 0)
            graphs.append(g)
    torch.cuda.synchronize()

    def graphed(n):
        with torch.cuda.stream(s):
            for i in range(n):
                graphs[i % NB].replay()
        torch.cuda.synchronize()

    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        plain(16)
    for rep in range(3):
        t0 = time.perf_counter(); plain(STEPS); tp = (time.perf_counter() - t0) / STEPS
        t0 = time.perf_counter(); graphed(STEPS); tg = (time.perf_counter() - t0) / STEPS
        print(f"plain {tp * 1e3:.4f} ms/step   graph {tg * 1e3:.4f} ms/step", flush=True)
