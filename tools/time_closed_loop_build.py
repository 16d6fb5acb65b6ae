import os, sys, time
sys.path.insert(0, "/root/repo/compressor-mpc_amd")
import numpy as np, torch, cmpc
from cmpc.configs import reference_setup
from cmpc.synthetic import synthetic_operating_points, synthetic_u_old
B, K = 65536, 9
cfg = cmpc.reference_config("par", "coop", p=50)
arr = cmpc.controller_arrays(cfg, reference_setup("par", "coop"))
xs, us, ys = synthetic_operating_points(cfg, B, seed=77, n_distinct=2048)
tx, tu, ty = (torch.from_numpy(a).cuda() for a in (xs, us, ys))
S = cfg.S
with cmpc.Context(cfg, B) as ctx:
    ctx.configure(arr)
    def reset():
        ctx.set_state(synthetic_u_old(cfg, B, np.random.default_rng(78)), np.zeros((B * S, cfg.nV)), np.zeros(B * S, np.uint32))
        ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr()); ctx.build(); ctx.init_warmstart(); ctx.synchronize()
    reset()
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        for _ in range(8): ctx.build()
        ctx.synchronize()
    def run(flags, n=30, produce=True):
        ctx.enable_timing(True)
        for _ in range(n):
            if produce: ctx.produce_lin(tx.data_ptr(), tu.data_ptr(), ty.data_ptr())
            ctx.step(K, flags)
        ctx.synchronize()
        b = ctx.kernel_time(cmpc.CMPC_KERNEL_BUILD); it = ctx.kernel_time(cmpc.CMPC_KERNEL_ITERATE)
        ctx.enable_timing(False)
        u, _, ws = ctx.get_state()
        return b[0]/b[1], it[0]/it[1], np.abs(u).max(), (ws != 0).mean()
    for rep in range(2):
        reset(); print("produce+step flags=0    ", run(0), flush=True)
        reset(); print("produce+step APPLY_MOVE ", run(cmpc.CMPC_APPLY_MOVE), flush=True)
        print("  then step APPLY, no produce", run(cmpc.CMPC_APPLY_MOVE, produce=False), flush=True)
        reset(); print("step flags=0, no produce", run(0, produce=False), flush=True)
