"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the checker (a CPU restatement of the reference path); the
product never imports this module.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "compressor-mpc_amd"))

from cmpc._abi import CmpcDims, CmpcLayout, dptr, iptr, uptr, bptr  # noqa: E402

ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")


class OrQpInfo(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("nchg", ctypes.c_int32),
                ("ws", ctypes.c_uint32), ("ntrace", ctypes.c_int32),
                ("trace", ctypes.c_uint8 * 16), ("margin", ctypes.c_double)]


class OrCfg(ctypes.Structure):
    P = ctypes.POINTER(ctypes.c_double)
    _fields_ = [("y_ref", P), ("ywt", P), ("uwt", P), ("lower", P), ("upper", P),
                ("rate_lower", P), ("rate_upper", P)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(ORACLE_LIB)
        P = ctypes.POINTER
        d, i32, u32 = ctypes.c_double, ctypes.c_int32, ctypes.c_uint32
        L.or_plant_default.argtypes = [ctypes.c_int, P(d), P(d)]
        L.or_plant_output.argtypes = [ctypes.c_int, P(d), P(d)]
        L.or_plant_linearize.argtypes = [ctypes.c_int, d, d, P(d), P(d), P(d), P(d), P(d), P(d)]
        L.or_discretize_rk4.argtypes = [ctypes.c_int, ctypes.c_int, d, P(d), P(d), P(d),
                                        P(d), P(d), P(d)]
        L.or_layout_of.argtypes = [P(CmpcDims), P(CmpcLayout)]
        L.or_lin_record.argtypes = [ctypes.c_int, d, d, d, P(d), P(d), P(i32), P(i32),
                                    P(CmpcDims), P(d)]
        L.or_generate_prediction.argtypes = [P(CmpcDims), P(d), P(d), P(d), P(d), P(d)]
        L.or_build_qp.argtypes = [P(CmpcDims), P(d), P(d), P(d), P(d), P(d), P(d), P(d),
                                  P(d), P(d), P(d)]
        L.or_qp_solve.argtypes = [ctypes.c_int, ctypes.c_int, P(d), P(d), P(d), P(d), P(d),
                                  P(d), u32, ctypes.c_int, P(d), P(OrQpInfo)]
        L.or_qp_solve_map.argtypes = [ctypes.c_int, ctypes.c_int, P(d), P(d), ctypes.c_int, P(d),
                                      P(d), P(d), P(d), P(d), P(d), u32, ctypes.c_int, P(d),
                                      P(OrQpInfo)]
        L.or_step.argtypes = [P(CmpcDims), P(OrCfg), P(d), ctypes.c_int, u32, ctypes.c_int,
                              ctypes.c_int, P(d), P(d), P(u32), P(d), P(i32), P(i32),
                              P(ctypes.c_uint8), P(i32), P(d)]
        _lib = L
    return _lib


def layout(dims: CmpcDims) -> CmpcLayout:
    L = CmpcLayout()
    assert lib().or_layout_of(ctypes.byref(dims), ctypes.byref(L)) == 0
    return L


def plant_default(plant: int):
    x = np.zeros(16)
    u = np.zeros(16)
    lib().or_plant_default(plant, dptr(x), dptr(u))
    ns, ni = (11, 9) if plant == 0 else (10, 8)
    return x[:ns].copy(), u[:ni].copy()


def plant_output(plant: int, x):
    y = np.zeros(4)
    lib().or_plant_output(plant, dptr(np.ascontiguousarray(x, dtype=np.float64)), dptr(y))
    return y


def lin_record(cfg, dims, s, x, u_full, Ts=0.05, p_in=1.0, p_out=1.0):
    L = layout(dims)
    rec = np.zeros(L.rec_len)
    io = np.asarray(cfg.input_order[s], dtype=np.int32)
    oi = np.asarray(cfg.out_idx[s], dtype=np.int32)
    rc = lib().or_lin_record(cfg.plant, p_in, p_out, Ts,
                             dptr(np.ascontiguousarray(x, dtype=np.float64)),
                             dptr(np.ascontiguousarray(u_full, dtype=np.float64)),
                             iptr(io), iptr(oi), ctypes.byref(dims), dptr(rec))
    assert rc == 0
    return rec


def build_qp(dims, rec, u_old, y_ref, ywt, uwt):
    L = layout(dims)
    R = dims.p * dims.ny
    H = np.zeros((L.nV, L.nV)); f = np.zeros(L.nV)
    YPW = np.zeros((R, L.nV)); Suo = np.zeros((R, max(L.nVo, 1)))
    G = np.zeros((L.nV, max(L.nVo, 1)))
    c = lambda a: np.ascontiguousarray(a, dtype=np.float64)
    lib().or_build_qp(ctypes.byref(dims), dptr(c(rec)), dptr(c(u_old)), dptr(c(y_ref)),
                      dptr(c(ywt)), dptr(c(uwt)), dptr(H), dptr(f), dptr(YPW), dptr(Suo),
                      dptr(G) if L.nVo else None)
    return H, f, YPW, Suo[:, :L.nVo], G[:, :L.nVo]


def generate_prediction(dims, rec):
    L = layout(dims)
    R = dims.p * dims.ny
    Su = np.zeros((R, L.nV)); Sx = np.zeros((R, L.naug)); Sf = np.zeros((R, dims.ns))
    Suo = np.zeros((R, max(L.nVo, 1)))
    lib().or_generate_prediction(ctypes.byref(dims), dptr(np.ascontiguousarray(rec)),
                                 dptr(Su), dptr(Sx), dptr(Sf), dptr(Suo))
    return Su, Sx, Sf, Suo[:, :L.nVo]


def qp_solve(H, g, lb, ub, lbA, ubA, nu, ws_in=0, max_chg=10):
    n = len(g)
    x = np.zeros(n)
    info = OrQpInfo()
    c = lambda a: np.ascontiguousarray(a, dtype=np.float64)
    lib().or_qp_solve(n, nu, dptr(c(H)), dptr(c(g)), dptr(c(lb)), dptr(c(ub)), dptr(c(lbA)),
                      dptr(c(ubA)), int(ws_in), max_chg, dptr(x), ctypes.byref(info))
    return x, info


def qp_solve_map(H, f, G, d, lb, ub, lbA, ubA, nu, ws_in=0, max_chg=10):
    """The Jacobi iteration's solve in the map form (or_qp.c step A): g = f + G d."""
    n = len(f)
    nvo = int(np.asarray(d).size)
    x = np.zeros(n)
    info = OrQpInfo()
    c = lambda a: np.ascontiguousarray(a, dtype=np.float64)
    Gc = c(np.asarray(G).reshape(n, nvo)) if nvo else None
    dc = c(d) if nvo else None
    lib().or_qp_solve_map(n, nu, dptr(c(H)), dptr(c(f)), nvo, dptr(Gc) if nvo else None,
                          dptr(dc) if nvo else None, dptr(c(lb)), dptr(c(ub)), dptr(c(lbA)),
                          dptr(c(ubA)), int(ws_in), max_chg, dptr(x), ctypes.byref(info))
    return x, info


def step(dims, arrays, lin, K, u_old, du_old, ws, flags=0, init=False, threads=1,
         want_trace=False, margin=None):
    """Batched oracle step; state arrays are updated in place.  margin: an
    optional (B*S,) float64 array that receives each QP slot's smallest
    decision margin over the step's solves (or_qp.c)."""
    L = layout(dims)
    nq = dims.B * dims.S
    du = np.zeros((nq, L.nV)); status = np.zeros(nq, np.int32); nwsr = np.zeros(nq, np.int32)
    trace = np.full((nq, max(K, 1), 16), 0xFF, np.uint8) if want_trace else None
    ntrace = np.zeros((nq, max(K, 1)), np.int32) if want_trace else None
    keep = [np.ascontiguousarray(getattr(arrays, k), dtype=np.float64) for k in
            ("y_ref", "ywt", "uwt", "lower", "upper", "rate_lower", "rate_upper")]
    cfg = OrCfg(*[dptr(a) for a in keep])
    assert u_old.flags["C_CONTIGUOUS"] and du_old.flags["C_CONTIGUOUS"]
    rc = lib().or_step(ctypes.byref(dims), ctypes.byref(cfg), dptr(lin), K, flags, int(init),
                       threads, dptr(u_old), dptr(du_old), uptr(ws), dptr(du), iptr(status),
                       iptr(nwsr), bptr(trace) if want_trace else None,
                       iptr(ntrace) if want_trace else None,
                       dptr(margin) if margin is not None else None)
    assert rc == 0
    return du, status, nwsr, trace, ntrace


def _observer_sigs():
    L = lib()
    if getattr(L, "_obs_sigs", False):
        return L
    P, d = ctypes.POINTER, ctypes.c_double
    L.or_observe_post.argtypes = [ctypes.c_int] * 3 + [P(d)] * 6
    L.or_observe_post.restype = None
    L.or_observe_prior.argtypes = [P(CmpcDims), P(d), P(d), P(d), P(d)]
    L.or_observe_prior.restype = ctypes.c_int
    L._obs_sigs = True
    return L


def observe_post(ns, ndist, Cp, M, y, y_old, dx, x_hat):
    """or_observe_post; y_old, dx, x_hat (float64, contiguous) updated in place."""
    n_out = len(y)
    Cp = np.ascontiguousarray(Cp, dtype=np.float64)
    M = np.ascontiguousarray(M, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    for a in (y_old, dx, x_hat):
        assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    _observer_sigs().or_observe_post(ns, ndist, n_out, dptr(Cp), dptr(M), dptr(y), dptr(y_old),
                                     dptr(dx), dptr(x_hat))


def observe_prior(dims, rec, du_own, u_old, dx):
    """or_observe_prior; u_old, dx updated in place."""
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    du_own = np.ascontiguousarray(du_own, dtype=np.float64)
    for a in (u_old, dx):
        assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    rc = _observer_sigs().or_observe_prior(ctypes.byref(dims), dptr(rec), dptr(du_own), dptr(u_old),
                                           dptr(dx))
    assert rc == 0


def plant_linearize(plant: int, x, u_full, p_in=1.0, p_out=1.0):
    """or_plant_linearize: continuous (A, B, C, f); C is n_outputs x ns."""
    ns, ni, no, nci = (ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int())
    lib().or_plant_dims(plant, ctypes.byref(ns), ctypes.byref(ni), ctypes.byref(no), ctypes.byref(nci))
    ns, no, nci = ns.value, no.value, nci.value
    A, B, C, f = np.zeros(ns * ns), np.zeros(ns * nci), np.zeros(no * ns), np.zeros(ns)
    lib().or_plant_linearize(plant, p_in, p_out, dptr(np.ascontiguousarray(x, dtype=np.float64)),
                             dptr(np.ascontiguousarray(u_full, dtype=np.float64)), dptr(A), dptr(B),
                             dptr(C), dptr(f))
    return A.reshape(ns, ns), B.reshape(ns, nci), C.reshape(no, ns), f


def _sim_sigs():
    L = lib()
    if getattr(L, "_sim_sigs", False):
        return L
    P, d, i32 = ctypes.POINTER, ctypes.c_double, ctypes.c_int32
    L.or_sim_interval.argtypes = [ctypes.c_int, d, d, P(d), P(d), d, d, P(d), d, d]
    L.or_sim_interval.restype = ctypes.c_int
    L.or_plant_derivative.argtypes = [ctypes.c_int, d, d, P(d), P(d), P(d)]
    L.or_time_delay_init.argtypes = [ctypes.c_int, P(i32), P(d), P(i32)]
    L.or_time_delay.argtypes = [ctypes.c_int, P(i32), P(d), P(i32), P(d), P(d)]
    L.or_plant_input.argtypes = [ctypes.c_int, ctypes.c_int, P(i32), P(d), P(d), P(d)]
    L._sim_sigs = True
    return L


class PlantSim:
    """The harness's SimulationSystem (oracle): TimeDelay -> GetPlantInput ->
    controlled Dormand-Prince per observation interval (or_sim.c)."""

    def __init__(self, plant, x0, u_offset, delays=(0, 40, 0, 40), control_index=(0, 3, 4, 7),
                 p_in=1.0, p_out=1.0, dt0=0.05, eps=1e-6):
        self.L = _sim_sigs()
        self.plant, self.p_in, self.p_out, self.eps = plant, p_in, p_out, eps
        self.x = np.array(x0, dtype=np.float64)
        self.u_offset = np.array(u_offset, dtype=np.float64)
        self.delays = np.array(delays, dtype=np.int32)
        self.cidx = np.array(control_index, dtype=np.int32)
        self.ring = np.zeros(max(1, int(self.delays.sum())))
        self.cur = np.zeros(len(delays), np.int32)
        self.L.or_time_delay_init(len(delays), iptr(self.delays), dptr(self.ring), iptr(self.cur))
        self.u_full = self.u_offset.copy()
        self.dt = np.array([dt0])

    def set_input(self, u_control):
        u_next = np.ascontiguousarray(u_control, dtype=np.float64)
        out = np.zeros(len(self.delays))
        self.L.or_time_delay(len(self.delays), iptr(self.delays), dptr(self.ring), iptr(self.cur),
                             dptr(u_next), dptr(out))
        self.L.or_plant_input(len(self.u_offset), len(self.delays), iptr(self.cidx),
                              dptr(self.u_offset), dptr(out), dptr(self.u_full))

    def integrate(self, t, t_end):
        rc = self.L.or_sim_interval(self.plant, self.p_in, self.p_out, dptr(self.u_full),
                                    dptr(self.x), t, t_end, dptr(self.dt), self.eps, self.eps)
        assert rc >= 0
        return rc
