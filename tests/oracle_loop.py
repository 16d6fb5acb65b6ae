"""The closed loop of cmpc/driver.py restated with the oracle — TEST
INFRASTRUCTURE ONLY (the checker; the product never imports this).

Per sampling instant (the reference's NerveCenter::GetNextInputWithTiming
inside the harness's integrate_const callback):
  y = plant output                               or_plant_output
  observer a posteriori per QP, relinearise      or_observe_post, or_lin_record
  build + K Jacobi iterations (cold solves first) or_step
  observer a priori + u_old per QP               or_observe_prior
  nerve-level u_old += own first moves           (nerve_center.h:313-319)
  SetInput through the delay line; integrate, or at a segment end SetOffset
  and a new Integrate call                       or_time_delay, or_sim_interval
"""
import numpy as np

import _oracle as O
from cmpc._abi import CmpcDims

CTRL = (0, 3, 4, 7)   # ControlInputIndex of both plants
TS = 0.05


class OracleClosedLoop:
    def __init__(self, cfg, arrays, M, K, segments=None, x0=None):
        self.cfg, self.arr, self.M, self.K = cfg, arrays, M, K
        self.dims = CmpcDims.from_config(cfg, 1)
        self.L = O.layout(self.dims)
        xd, u_def = O.plant_default(cfg.plant)
        x0 = xd if x0 is None else np.asarray(x0, dtype=np.float64)
        segs = segments or [([0.0] * len(u_def), float("inf"))]
        offs = [u_def + np.asarray(d, dtype=np.float64) for d, _ in segs]
        self.u_off = offs[0].copy()                       # the controller's (NerveCenter::Initialize)
        self.sched = [(float(segs[i - 1][1]), offs[i]) for i in range(1, len(segs))]
        self.sim = O.PlantSim(cfg.plant, x0, offs[0])
        S, nq = cfg.S, cfg.S
        y0 = O.plant_output(cfg.plant, x0)
        self.xh = np.repeat(x0[None, :], nq, axis=0)
        self.dx = np.zeros((nq, self.L.ntot))
        self.yo = np.repeat(y0[None, :], nq, axis=0)
        self.C = [O.plant_linearize(cfg.plant, x0, self.u_off)[2] for _ in range(nq)]
        self.u_old = np.zeros((nq, cfg.nu_tot))
        self.du_old = np.zeros((nq, cfg.nV))
        self.ws = np.zeros(nq, np.uint32)
        self.u_ctrl = np.zeros(cfg.nu_tot)
        self.k = 0
        self.t_seg, self.seg_step = 0.0, 0   # integrate_const's start time and step count

    def step(self):
        cfg, S = self.cfg, self.cfg.S
        t = self.t_seg + self.seg_step * TS
        y = O.plant_output(cfg.plant, self.sim.x)
        u_lin = self.u_off.copy()
        u_lin[list(CTRL)] += self.u_ctrl
        recs = np.zeros((S, self.L.rec_len))
        for q in range(S):
            O.observe_post(cfg.ns, cfg.ndist, self.C[q], self.M[q], y, self.yo[q], self.dx[q], self.xh[q])
            self.C[q] = O.plant_linearize(cfg.plant, self.xh[q], u_lin)[2]
            r = O.lin_record(cfg, self.dims, q, self.xh[q], u_lin)
            r[self.L.off_x:self.L.off_x + self.L.naug] = self.dx[q, cfg.ns:]
            r[self.L.off_y:self.L.off_y + cfg.ny] = y[cfg.out_idx[q]]
            recs[q] = r
        du, st, *_ = O.step(self.dims, self.arr, np.ascontiguousarray(recs), self.K, self.u_old,
                            self.du_old, self.ws, init=(self.k == 0))
        for q in range(S):
            O.observe_prior(self.dims, recs[q], du[q, :cfg.nu], self.u_old[q], self.dx[q])
            own = cfg.input_order[q][:cfg.nu]
            self.u_ctrl[own] += du[q, :cfg.nu]
        self.sim.set_input(self.u_ctrl)
        if self.sched and t >= self.sched[0][0] - 1e-9:
            self.t_seg, self.seg_step = self.sched[0][0], 0
            self.sim.u_offset[:] = self.sched.pop(0)[1]
            self.sim.dt[0] = TS
        else:
            self.sim.integrate(t, t + TS)
            self.seg_step += 1
        self.k += 1
        return y
