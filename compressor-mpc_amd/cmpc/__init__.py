"""cmpc — MI355X-native condensed-QP hot path of katie-jones/compressor-mpc.

Python host view of the C ABI (include/cmpc.h).  Every compute call goes to
libcmpc.so (HIP kernels for gfx950); there is no CPU fallback.

    ctx = Context(cfg, B)                 # NerveCenter/DistributedController ctors
    ctx.configure(arrays)                 # SetWeights / SetOutputReference / constraints
    ctx.set_state(u_old, du_old, ws)      # Initialize
    ctx.upload_lin(lin)                   # AugmentedLinearizedSystem::Update results
    ctx.init_warmstart()                  # InitializeQPProblem
    ctx.step(K)                           # GetNextInputWithTiming (build + K Jacobi iterations)
    du, status, nwsr = ctx.download()
"""
import ctypes

import numpy as np

from . import _abi
from ._abi import (CMPC_BUILD_AUTO, CMPC_BUILD_ROWS, CMPC_BUILD_SPLIT, CMPC_BUILD_WAVE, CMPC_SOLVE_AUTO, CMPC_SOLVE_LANE,
                   CMPC_SOLVE_ROWS, CMPC_STEP_AUTO, CMPC_STEP_FUSED, CMPC_STEP_SPLIT, CMPC_KERNEL_STEP,
                   CMPC_APPLY_MOVE, CMPC_KERNEL_BUILD, CMPC_KERNEL_ITERATE,
                   CMPC_KERNEL_PRODUCE, CMPC_KERNEL_OBSERVE_POST, CMPC_KERNEL_OBSERVE_PRIOR, CMPC_QP_INFEASIBLE,
                   CMPC_QP_MAX_NWSR, CMPC_QP_NOT_PD, CMPC_QP_NONFINITE, CMPC_QP_OK, CMPC_TRACE, CmpcDims,
                   CmpcLayout, bptr, check, dptr, iptr, load_library, uptr)
from .configs import ControllerConfig, SetupFile, reference_config, reference_observer_gain, reference_setup
from .problem import ControllerArrays, controller_arrays, plant_input_from_plans

__all__ = ["Context", "ControllerConfig", "SetupFile", "reference_config", "reference_setup",
           "reference_observer_gain", "controller_arrays",
           "plant_input_from_plans", "plant_lin_record", "plant_default", "plant_output",
           "layout_of", "rows_lds_model", "qp_solve_batch", "CMPC_APPLY_MOVE", "CMPC_TRACE", "CMPC_QP_OK",
           "CMPC_QP_MAX_NWSR", "CMPC_QP_INFEASIBLE", "CMPC_QP_NOT_PD",
           "CMPC_QP_NONFINITE"]


def layout_of(dims: CmpcDims) -> CmpcLayout:
    L = CmpcLayout()
    check(load_library().cmpc_layout_of(ctypes.byref(dims), ctypes.byref(L)), "cmpc_layout_of")
    return L


def rows_lds_model(dims: CmpcDims):
    """(packed, chosen, lds_bytes): the row build kernel's modelled extra LDS
    cycles per wave-step for regions packed back to back and for the layout
    cmpc_build uses (rows_layout.cpp), and its LDS bytes per workgroup."""
    a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
    check(load_library().cmpc_rows_lds_model(ctypes.byref(dims), ctypes.byref(a), ctypes.byref(b),
                                              ctypes.byref(n)), "cmpc_rows_lds_model")
    return a.value, b.value, n.value


def plant_default(plant: int):
    x = np.zeros(16)
    u = np.zeros(16)
    check(load_library().cmpc_plant_default(plant, dptr(x), dptr(u)), "cmpc_plant_default")
    ns, ni = (11, 9) if plant == 0 else (10, 8)
    return x[:ns].copy(), u[:ni].copy()


def plant_output(plant: int, x) -> np.ndarray:
    y = np.zeros(4)
    check(load_library().cmpc_plant_output(plant, dptr(np.ascontiguousarray(x, np.float64)),
                                            dptr(y)), "cmpc_plant_output")
    return y


def plant_lin_record(cfg: ControllerConfig, dims: CmpcDims, s: int, x, u_full, Ts=0.05,
                     p_in=1.0, p_out=1.0, out=None) -> np.ndarray:
    """AugmentedLinearizedSystem::Update for sub-controller s -> lin record
    (fills Aorig, Bin, Csel, fd; dx_aug and yprev are left as they are)."""
    L = layout_of(dims)
    rec = np.zeros(L.rec_len) if out is None else out
    io = np.ascontiguousarray(cfg.input_order[s], dtype=np.int32)
    oi = np.ascontiguousarray(cfg.out_idx[s], dtype=np.int32)
    check(load_library().cmpc_plant_lin_record(
        cfg.plant, p_in, p_out, Ts, dptr(np.ascontiguousarray(x, np.float64)),
        dptr(np.ascontiguousarray(u_full, np.float64)), iptr(io), iptr(oi), ctypes.byref(dims),
        dptr(rec)), "cmpc_plant_lin_record")
    return rec


def qp_solve_batch(H, g, lb, ub, lbA, ubA, nu, ws_in=None, max_chg=10, device=0):
    """The device QP solver alone over a batch (parity / known-answer tests)."""
    H = np.ascontiguousarray(H, np.float64)
    nqp, n = g.shape
    c = lambda a: np.ascontiguousarray(a, np.float64)
    ws_in = np.zeros(nqp, np.uint32) if ws_in is None else np.ascontiguousarray(ws_in, np.uint32)
    x = np.zeros((nqp, n))
    status = np.zeros(nqp, np.int32)
    nchg = np.zeros(nqp, np.int32)
    ws_out = np.zeros(nqp, np.uint32)
    trace = np.zeros((nqp, 16), np.uint8)
    ntrace = np.zeros(nqp, np.int32)
    lib = load_library()
    lib.cmpc_qp_solve_batch.restype = ctypes.c_int
    check(lib.cmpc_qp_solve_batch(device, n, nu, nqp, dptr(H), dptr(c(g)), dptr(c(lb)),
                                  dptr(c(ub)), dptr(c(lbA)), dptr(c(ubA)), uptr(ws_in), max_chg,
                                  dptr(x), iptr(status), iptr(nchg), uptr(ws_out), bptr(trace),
                                  iptr(ntrace)), "cmpc_qp_solve_batch")
    return x, status, nchg, ws_out, trace, ntrace


def qp_solve_batch_map(H, f, G, d, lb, ub, lbA, ubA, nu, ws_in=None, max_chg=10, device=0):
    """One Jacobi-iteration solve per QP in the map form (g = f + G d), the
    solve of cmpc_iterate / DistributedSolver::UpdateAndSolveQP."""
    H = np.ascontiguousarray(H, np.float64)
    nqp, n = f.shape
    G = np.ascontiguousarray(G, np.float64).reshape(nqp, n, -1)
    nvo = G.shape[2]
    c = lambda a: np.ascontiguousarray(a, np.float64)
    ws_in = np.zeros(nqp, np.uint32) if ws_in is None else np.ascontiguousarray(ws_in, np.uint32)
    x = np.zeros((nqp, n))
    status = np.zeros(nqp, np.int32)
    nchg = np.zeros(nqp, np.int32)
    ws_out = np.zeros(nqp, np.uint32)
    trace = np.zeros((nqp, 16), np.uint8)
    ntrace = np.zeros(nqp, np.int32)
    lib = load_library()
    check(lib.cmpc_qp_solve_batch_map(device, n, nu, nvo, nqp, dptr(H), dptr(c(f)), dptr(G), dptr(c(d)),
                                      dptr(c(lb)), dptr(c(ub)), dptr(c(lbA)), dptr(c(ubA)), uptr(ws_in), max_chg,
                                      dptr(x), iptr(status), iptr(nchg), uptr(ws_out), bptr(trace), iptr(ntrace)),
          "cmpc_qp_solve_batch_map")
    return x, status, nchg, ws_out, trace, ntrace


def _torch_runtime_first():
    """torch bundles its own HIP runtime; when the library's runtime opens the
    device first, torch's later initialisation reports no GPUs.  If the
    caller uses torch for device buffers (it is imported), bring its runtime
    up before the library's."""
    import sys
    torch = sys.modules.get("torch")
    if torch is not None:
        try:
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass


class Context:
    """One batched NerveCenter over B scenarios of cfg.S sub-controllers."""

    def __init__(self, cfg: ControllerConfig, B: int, device: int = 0):
        self.lib = load_library()
        self.cfg = cfg
        self.B = B
        self.dims = CmpcDims.from_config(cfg, B)
        self.layout = layout_of(self.dims)
        self.nqp = B * cfg.S
        self._h = ctypes.c_void_p()
        _torch_runtime_first()
        check(self.lib.cmpc_create(ctypes.byref(self._h), ctypes.byref(self.dims), device),
              "cmpc_create")

    # -- lifecycle -------------------------------------------------------
    def close(self):
        if self._h:
            self.lib.cmpc_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle: int):
        check(self.lib.cmpc_set_stream(self._h, ctypes.c_void_p(stream_handle)), "cmpc_set_stream")

    # -- configuration ---------------------------------------------------
    def configure(self, a: ControllerArrays):
        for s in range(self.cfg.S):
            check(self.lib.cmpc_set_weights(self._h, s, dptr(np.ascontiguousarray(a.uwt[s])),
                                            dptr(np.ascontiguousarray(a.ywt[s]))), "set_weights")
            check(self.lib.cmpc_set_constraints(
                self._h, s, dptr(np.ascontiguousarray(a.lower[s])),
                dptr(np.ascontiguousarray(a.upper[s])), dptr(np.ascontiguousarray(a.rate_lower[s])),
                dptr(np.ascontiguousarray(a.rate_upper[s]))), "set_constraints")
            check(self.lib.cmpc_set_reference(self._h, s, dptr(np.ascontiguousarray(a.y_ref[s]))),
                  "set_reference")

    def set_state(self, u_old=None, du_old=None, ws=None):
        c = lambda a, dt: None if a is None else np.ascontiguousarray(a, dt)
        u_old, du_old, ws = c(u_old, np.float64), c(du_old, np.float64), c(ws, np.uint32)
        check(self.lib.cmpc_set_state(self._h, dptr(u_old) if u_old is not None else None,
                                      dptr(du_old) if du_old is not None else None,
                                      uptr(ws) if ws is not None else None), "set_state")

    def get_state(self):
        u_old = np.zeros((self.nqp, self.cfg.nu_tot))
        du_old = np.zeros((self.nqp, self.layout.nV))
        ws = np.zeros(self.nqp, np.uint32)
        check(self.lib.cmpc_get_state(self._h, dptr(u_old), dptr(du_old), uptr(ws)), "get_state")
        return u_old, du_old, ws

    def upload_lin(self, lin: np.ndarray):
        lin = np.ascontiguousarray(lin, np.float64)
        assert lin.size == self.nqp * self.layout.rec_len
        check(self.lib.cmpc_upload_lin(self._h, dptr(lin)), "upload_lin")

    def lin_device_ptr(self) -> int:
        return self.lib.cmpc_lin_device(self._h)

    def bind_lin(self, device_ptr: int = 0):
        """Bind an external device-resident record array (0 = own buffer)."""
        check(self.lib.cmpc_bind_lin(self._h, ctypes.c_void_p(device_ptr or None)), "cmpc_bind_lin")

    def bind_state(self, u_old_ptr: int = 0, du_old_ptr: int = 0, ws_ptr: int = 0):
        """Bind external device-resident state arrays (u_old B*S x nu_tot f64,
        du_old B*S x nV f64, ws B*S u32; all three, or 0 for the own buffers)."""
        vp = lambda p: ctypes.c_void_p(p or None)
        check(self.lib.cmpc_bind_state(self._h, vp(u_old_ptr), vp(du_old_ptr), vp(ws_ptr)),
              "cmpc_bind_state")

    def produce_lin(self, x_ptr: int, u_full_ptr: int, y_ptr: int, dx_aug_ptr: int = 0,
                    Ts: float = 0.05, p_in: float = 1.0, p_out: float = 1.0):
        """Device producer (cmpc_produce_lin): linearise + discretise the plant
        for every scenario on the GPU and write this context's lin records.
        Arguments are device pointers (e.g. torch tensor .data_ptr())."""
        io = np.ascontiguousarray(self.cfg.input_order, dtype=np.int32)
        oi = np.ascontiguousarray(self.cfg.out_idx, dtype=np.int32)
        check(self.lib.cmpc_produce_lin(
            self._h, self.cfg.plant, p_in, p_out, Ts, iptr(io), iptr(oi), ctypes.c_void_p(x_ptr),
            ctypes.c_void_p(u_full_ptr), ctypes.c_void_p(dx_aug_ptr or None), ctypes.c_void_p(y_ptr)),
            "cmpc_produce_lin")

    # -- observer + receding-horizon update --------
    def set_observer(self, s: int, M: np.ndarray):
        """ObserverMatrix of sub-controller s, (ns + ndist) x n_outputs."""
        M = np.ascontiguousarray(M, dtype=np.float64)
        check(self.lib.cmpc_set_observer(self._h, s, M.shape[1], dptr(M)), "cmpc_set_observer")

    @property
    def observer_len(self) -> int:
        return self.lib.cmpc_observer_len(self._h)

    def observer_init(self, x_ptr: int, u_full_ptr: int, y_ptr: int, dx_init_ptr: int = 0,
                      Ts: float = 0.05, p_in: float = 1.0, p_out: float = 1.0):
        """DistributedController::Initialize for every slot: observer state at
        (x_init[b], y_init[b], dx_init) and the records at x_init (device ptrs)."""
        io = np.ascontiguousarray(self.cfg.input_order, dtype=np.int32)
        oi = np.ascontiguousarray(self.cfg.out_idx, dtype=np.int32)
        check(self.lib.cmpc_observer_init(
            self._h, self.cfg.plant, p_in, p_out, Ts, iptr(io), iptr(oi), ctypes.c_void_p(x_ptr),
            ctypes.c_void_p(u_full_ptr), ctypes.c_void_p(y_ptr), ctypes.c_void_p(dx_init_ptr or None)),
            "cmpc_observer_init")

    def observe_step(self, u_full_ptr: int, y_ptr: int):
        """ObserveAPosteriori + x_hat update, then the records at x_hat."""
        check(self.lib.cmpc_observe_step(self._h, ctypes.c_void_p(u_full_ptr), ctypes.c_void_p(y_ptr)),
              "cmpc_observe_step")

    def control_step(self, u_full_ptr: int, y_ptr: int, K: int):
        """NerveCenter::GetNextInput on the device (cmpc_control_step): observe_step,
        step(K, 0) and observe_apply, one kernel launch where the batch allows."""
        check(self.lib.cmpc_control_step(self._h, ctypes.c_void_p(u_full_ptr), ctypes.c_void_p(y_ptr), K),
              "cmpc_control_step")

    def control_step_download(self, u_full: np.ndarray, y: np.ndarray, K: int):
        """cmpc_control_step_download: the control step from host arrays and its
        plans, statuses and nWSR (polled completion for one-workgroup batches)."""
        du = np.zeros((self.nqp, self.layout.nV))
        status = np.zeros(self.nqp, np.int32)
        nwsr = np.zeros(self.nqp, np.int32)
        check(self.lib.cmpc_control_step_download(self._h, dptr(np.ascontiguousarray(u_full, np.float64)),
                                                  dptr(np.ascontiguousarray(y, np.float64)), K, dptr(du),
                                                  iptr(status), iptr(nwsr)), "cmpc_control_step_download")
        return du, status, nwsr

    def observe_apply(self):
        """UpdateU: ObserveAPriori with the own first move, then u_old += du."""
        check(self.lib.cmpc_observe_apply(self._h), "cmpc_observe_apply")

    def observer_state(self) -> np.ndarray:
        """(B*S, observer_len): [x_hat ns][dx_aug ntot][y_old n_out][C n_out x ns]."""
        out = np.zeros((self.B * self.cfg.S, self.observer_len))
        check(self.lib.cmpc_get_observer_state(self._h, dptr(out)), "cmpc_get_observer_state")
        return out

    def set_observer_state(self, st: np.ndarray):
        st = np.ascontiguousarray(st, dtype=np.float64)
        assert st.shape == (self.B * self.cfg.S, self.observer_len)
        check(self.lib.cmpc_set_observer_state(self._h, dptr(st)), "cmpc_set_observer_state")

    def download_lin(self) -> np.ndarray:
        """The context's own record buffer (B*S, rec_len), e.g. after produce_lin."""
        out = np.zeros((self.B * self.cfg.S, self.layout.rec_len))
        check(self.lib.cmpc_download_lin(self._h, dptr(out)), "cmpc_download_lin")
        return out

    # -- hot path --------------------------------------------------------
    def build(self):
        check(self.lib.cmpc_build(self._h), "cmpc_build")

    def set_build_variant(self, variant: int):
        """CMPC_BUILD_AUTO / CMPC_BUILD_WAVE (one QP per wave) / CMPC_BUILD_ROWS
        (four QPs per wave, one per DPP row) / CMPC_BUILD_SPLIT (one QP per two
        waves: chain and gather, every ny)."""
        check(self.lib.cmpc_set_build_variant(self._h, int(variant)), "cmpc_set_build_variant")

    def last_build_kernel(self) -> int:
        """CMPC_BUILD_WAVE / CMPC_BUILD_ROWS / CMPC_BUILD_SPLIT: the kernel the
        last build() ran."""
        v = self.lib.cmpc_last_build_kernel(self._h)
        check(min(v, 0), "cmpc_last_build_kernel")
        return v


    def set_solve_variant(self, variant: int):
        """CMPC_SOLVE_AUTO / CMPC_SOLVE_LANE (one QP per lane) / CMPC_SOLVE_ROWS
        (one QP per 16-lane row): the kernel of iterate / init_warmstart."""
        check(self.lib.cmpc_set_solve_variant(self._h, int(variant)), "cmpc_set_solve_variant")

    def last_solve_kernel(self) -> int:
        """CMPC_SOLVE_LANE / CMPC_SOLVE_ROWS: the kernel the last solve ran."""
        v = self.lib.cmpc_last_solve_kernel(self._h)
        check(min(v, 0), "cmpc_last_solve_kernel")
        return v

    def set_step_variant(self, variant: int):
        """CMPC_STEP_AUTO / CMPC_STEP_SPLIT (build + iterate launches) /
        CMPC_STEP_FUSED (one launch: the build kernel runs the iterations)."""
        check(self.lib.cmpc_set_step_variant(self._h, int(variant)), "cmpc_set_step_variant")

    def last_step_fused(self) -> bool:
        v = self.lib.cmpc_last_step_fused(self._h)
        check(min(v, 0), "cmpc_last_step_fused")
        return bool(v)
    def init_warmstart(self):
        check(self.lib.cmpc_init_warmstart(self._h), "cmpc_init_warmstart")

    def iterate(self, K: int, flags: int = 0):
        check(self.lib.cmpc_iterate(self._h, K, flags), "cmpc_iterate")

    def step(self, K: int, flags: int = 0):
        check(self.lib.cmpc_step(self._h, K, flags), "cmpc_step")

    def synchronize(self):
        check(self.lib.cmpc_synchronize(self._h), "cmpc_synchronize")

    # -- results ---------------------------------------------------------
    def download(self):
        du = np.zeros((self.nqp, self.layout.nV))
        status = np.zeros(self.nqp, np.int32)
        nwsr = np.zeros(self.nqp, np.int32)
        check(self.lib.cmpc_download(self._h, dptr(du), iptr(status), iptr(nwsr)), "download")
        return du, status, nwsr

    def download_qp(self):
        nV, nVo = self.layout.nV, self.layout.nVo
        H = np.zeros((self.nqp, nV, nV))
        f = np.zeros((self.nqp, nV))
        G = np.zeros((self.nqp, nV, max(nVo, 1)))
        check(self.lib.cmpc_download_qp(self._h, dptr(H), dptr(f), dptr(G)), "download_qp")
        return H, f, G[:, :, :nVo]

    def download_trace(self, K: int):
        trace = np.zeros((self.nqp, K, 16), np.uint8)
        ntrace = np.zeros((self.nqp, K), np.int32)
        check(self.lib.cmpc_download_trace(self._h, bptr(trace), iptr(ntrace)), "download_trace")
        return trace, ntrace

    def enable_timing(self, on: bool = True, only=None):
        """Kernel timing: every kernel (on), none, or only the kernel ids in
        `only` (CMPC_KERNEL_*)."""
        flag = int(bool(on))
        if on and only is not None:
            flag = 0
            for k in only:
                flag |= 2 << k
        check(self.lib.cmpc_enable_timing(self._h, flag), "enable_timing")

    def set_timing_stride(self, stride: int):
        """Time only every stride-th launch of each timed kernel."""
        check(self.lib.cmpc_set_timing_stride(self._h, int(stride)), "cmpc_set_timing_stride")

    def kernel_time(self, kernel: int):
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        check(self.lib.cmpc_kernel_time(self._h, kernel, ctypes.byref(ms), ctypes.byref(n)),
              "kernel_time")
        return ms.value, n.value
