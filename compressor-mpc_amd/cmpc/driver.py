"""Closed-loop driver: the reference's missing
common-simulation.inc, rebuilt from its surviving pieces and
batched over B scenarios on the device:

  per sampling instant t_k = t0 + k Ts (integrate_const's observer callback,
  simulation_system.h:48, :108-116):
    y      = plant output at x(t_k)                  SimulationSystem::GetOutput
    u      = NerveCenter::GetNextInputWithTiming(y)  nerve_center.h:134-182:
               observe a posteriori + linearise per sub-controller,
               condensed QP build, K Jacobi iterations, UpdateU (observer a
               priori + u_old), UpdateUOld (the nerve-level u_old_)
    record (t, x, u, y, ns) in the 6-line .dat format
    SetInput(u)   -> input delay line -> plant input  simulation_system.h:67-70
    integrate the plant over [t_k, t_k + Ts]          (controlled Dormand-Prince)

  The setup file's `simulation` segments are one Integrate call each, the
  plant-input offset stepped in between (SetOffset, simulation_system.h:64;
  the controller keeps its own offset, so the step is an unmeasured
  disturbance).  integrate_const observes both ends of its interval, so the
  instant at a segment boundary is observed twice: the last observation of
  one call (no integration follows), SetOffset, then the first of the next
  call at the same plant state, whose step-size control starts again from
  Ts.  The reference's records show exactly that (results/*/run1/*.dat: the
  records printed at t = 50 and 50.05 hold the same plant state, and every
  record is one controller call); the record count, not integrate_const's
  time, labels them.

Everything between two records runs on the GPU (sim.hip, observer.hip,
produce.hip, cmpc_kernels.hip); torch tensors are the device buffers.
"""
import time

import numpy as np

from . import CMPC_TRACE, Context
from .configs import ControllerConfig
from .sim import REF_CONTROL_INDEX, REF_DELAYS, REF_EPS, REF_TS, PlantSimulator


def _fmt(v: float) -> str:
    """std::ostream default formatting of a double (precision 6, %g)."""
    return "%g" % v


def eigen_row(vals) -> str:
    """Eigen's default matrix output of a vector printed transposed: every
    coefficient right-aligned to the widest one, separated by one space."""
    s = [_fmt(float(v)) for v in vals]
    w = max(len(t) for t in s)
    return " ".join(t.rjust(w) for t in s)


class DatWriter:
    """The reference's per-sample record (results/*.dat):
    t / x / u / y / wall-ns / blank."""

    def __init__(self, path_or_file):
        self.f = open(path_or_file, "w") if isinstance(path_or_file, str) else path_or_file
        self.own = isinstance(path_or_file, str)

    def record(self, t: float, x, u, y, ns: int):
        self.f.write(f"{_fmt(t)}\n{eigen_row(x)}\n{eigen_row(u)}\n{eigen_row(y)}\n{int(ns)}\n\n")

    def close(self):
        if self.own:
            self.f.close()


class ClosedLoop:
    """B closed loops (plant + NerveCenter) of one configuration on one GPU.

    cfg, arrays    controller configuration and weights/constraints/y_ref
    M              per sub-controller observer gains ((ns + ndist) x n_outputs)
    x0, u_offset   (B, ns), (B, n_inputs) host arrays: initial plant state and
                   the input offset u_init_full (NerveCenter::Initialize)
    K              Jacobi iterations per step (n-iterations)
    """

    def __init__(self, cfg: ControllerConfig, arrays, M, x0, u_offset, K: int, device: int = 0,
                 Ts: float = REF_TS, p_in: float = 1.0, p_out: float = 1.0):
        import torch
        self.torch = torch
        torch.cuda.init()
        dev = torch.device("cuda", device)
        self.cfg, self.K, self.Ts, self.dev = cfg, K, Ts, dev
        self.p_in, self.p_out = p_in, p_out
        B = x0.shape[0]
        self.B, S = B, cfg.S
        self.sim = PlantSimulator(cfg.plant, B, device, p_in, p_out, REF_DELAYS, REF_CONTROL_INDEX)
        self.ctx = Context(cfg, B, device=device)
        self.ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        self.ctx.configure(arrays)
        self.ctx.set_state(np.zeros((B * S, cfg.nu_tot)), np.zeros((B * S, cfg.nV)),
                           np.zeros(B * S, np.uint32))
        for s in range(S):
            self.ctx.set_observer(s, M[s])
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)
        self.x0, self.u_offset = t(x0), t(u_offset)
        self.u_ctrl = torch.zeros(B, cfg.nu_tot, dtype=torch.float64, device=dev)  # NerveCenter::u_old_
        self.u_lin = torch.zeros_like(self.u_offset)   # GetPlantInput(u_old_, u_offset_)
        self.io = np.ascontiguousarray(cfg.input_order, dtype=np.int32)
        self.k = 0
        self._sched = []   # pending (t_start, plant-input offset (B, n_inputs) device)

    def set_segments(self, segments, u_default):
        """The setup file's `simulation` segments ([(offset change, end time)],
        SetupFile.segments) over the plant's default input u_default (offset
        changes and u_default may be per scenario, (B, n_inputs)): segment 0's
        offset is the initial one (call before initialize); segment i's is set
        after the last instant of segment i-1 (its end time), which no
        integration follows (module docstring)."""
        torch = self.torch
        u_default = np.asarray(u_default, dtype=np.float64)
        # per-scenario defaults and changes broadcast: (n_inputs,) or (B, n_inputs)
        shape = (self.B, u_default.shape[-1])
        offs = [np.array(np.broadcast_to(u_default + np.asarray(d, dtype=np.float64), shape)) for d, _ in segments]
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev)
        self.u_offset = t(offs[0])
        self._sched = [(float(segments[i - 1][1]), t(offs[i])) for i in range(1, len(segments))]

    def initialize(self, dx_init=None):
        """SimulationSystem(x0, u_offset) + NerveCenter::Initialize(x0, 0,
        u_offset, y(x0), dx_init): the observers' state, the records at x0,
        the first build and the cold InitializeQPProblem solves."""
        self.sim.reset(self.x0, self.u_offset, self.Ts)
        y0 = self.sim.output()
        dx = 0 if dx_init is None else self.torch.from_numpy(np.ascontiguousarray(dx_init)).to(self.dev)
        self.ctx.observer_init(self.x0.data_ptr(), self.u_offset.data_ptr(), y0.data_ptr(),
                               dx.data_ptr() if dx_init is not None else 0, Ts=self.Ts,
                               p_in=self.p_in, p_out=self.p_out)
        self.ctx.build()
        self.ctx.init_warmstart()
        self.k = 0
        self.t_seg, self.seg_step = 0.0, 0   # integrate_const's start time and step count

    def step(self, trace: bool = False):
        """One sampling instant: returns (t, y) of the instant; the plant has
        advanced to the next one.  trace: the Jacobi iterations record their
        working-set changes (CMPC_TRACE); self.last_changes is then their
        total over the K iterations and all QP slots of this instant."""
        from ._abi import check, iptr
        t = 0.0 + self.k * self.Ts   # the record's label (record count)
        # integrate_const's own time: start_time + step * dt of the current
        # Integrate call; its interval ends at time + dt
        t_int = self.t_seg + self.seg_step * self.Ts
        y = self.sim.output()
        # GetNextInputWithTiming(y): linearisation input GetPlantInput(u_old_,
        # u_offset_) with the controller's own offset (fixed at Initialize; the
        # plant's may have stepped, see set_segments)
        self.sim.plant_input_offset(self.u_ctrl, self.u_offset, self.u_lin)
        self.ctx.observe_step(self.u_lin.data_ptr(), y.data_ptr())
        self.ctx.build()
        self.ctx.iterate(self.K, CMPC_TRACE if trace else 0)
        if trace:
            _, ntr = self.ctx.download_trace(self.K)
            self.last_changes = int(ntr.sum())
        self.ctx.observe_apply()
        check(self.ctx.lib.cmpc_accumulate_moves(self.ctx._h, iptr(self.io),
                                                 self.torch_ptr(self.u_ctrl)), "cmpc_accumulate_moves")
        # SetInput(u) through the delay line, then the plant over [t, t + Ts];
        # at the end of a segment's Integrate call: SetOffset and a new call
        self.sim.set_input(self.u_ctrl)
        if self._sched and t_int >= self._sched[0][0] - 1e-9:
            self.t_seg = self._sched[0][0]
            self.seg_step = 0
            self.sim.set_offset(self._sched.pop(0)[1])
            self.sim.restart(self.Ts)
        else:
            self.sim.integrate(t_int, t_int + self.Ts, REF_EPS, REF_EPS)
            self.seg_step += 1
        self.k += 1
        return t, y

    def plant_failures(self):
        """Scenarios whose plant integration failed in any interval since
        initialize (the simulator's status is sticky: 1 step-size control, 2
        more than 500 steps in an interval, 3 non-finite), as (count, status
        per scenario).  The reference's odeint throws and ends the run; here a
        failed scenario stops where it failed and the rest carry on."""
        st = self.sim.download()[3]
        return int((st != 0).sum()), st

    @staticmethod
    def torch_ptr(t):
        import ctypes
        return ctypes.c_void_p(t.data_ptr())

    def run(self, n_steps: int, writer: DatWriter = None, scenario: int = 0):
        """n_steps sampling instants; writes scenario `scenario`'s records
        (x and y at the instant, the controller output u) when a writer is
        given.  Returns the wall time per step (s)."""
        torch = self.torch
        t_tot = 0.0
        for _ in range(n_steps):
            x_now = self.sim.download()[0][scenario] if writer else None
            torch.cuda.synchronize(self.dev)
            t0 = time.perf_counter()
            t, y = self.step()
            torch.cuda.synchronize(self.dev)
            el = time.perf_counter() - t0
            t_tot += el
            if writer:
                writer.record(t, x_now, self.u_ctrl[scenario].cpu().numpy(), y[scenario].cpu().numpy(),
                              int(el * 1e9))
        return t_tot / max(n_steps, 1)

    def close(self):
        self.ctx.close()
        self.sim.close()
