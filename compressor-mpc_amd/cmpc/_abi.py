"""ctypes view of the C ABI declared in include/cmpc.h.

The product library is compressor-mpc_amd/cmpc/libcmpc.so (HIP, gfx950),
built in-tree by compressor-mpc_amd/csrc/Makefile.  There is no CPU fallback:
if the library is missing or cannot be loaded, load_library() raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CMPC_LIBRARY") or os.path.join(_HERE, "libcmpc.so")

CMPC_MAX_INPUTS = 8
CMPC_MAX_NV = 8
CMPC_MAX_NS = 15
CMPC_NWSR_MAX = 10

CMPC_QP_OK = 0
CMPC_QP_MAX_NWSR = 1
CMPC_QP_INFEASIBLE = 2
CMPC_QP_NOT_PD = 3
CMPC_QP_NONFINITE = 4

CMPC_APPLY_MOVE = 1
CMPC_TRACE = 2

CMPC_KERNEL_BUILD = 0
CMPC_KERNEL_ITERATE = 1
CMPC_KERNEL_PRODUCE = 2
CMPC_KERNEL_OBSERVE_POST = 3
CMPC_KERNEL_OBSERVE_PRIOR = 4
CMPC_KERNEL_STEP = 5
CMPC_KERNEL_COUNT = 6

CMPC_BUILD_AUTO = 0
CMPC_BUILD_WAVE = 1
CMPC_BUILD_ROWS = 2
CMPC_BUILD_SPLIT = 3
CMPC_SOLVE_AUTO = 0
CMPC_SOLVE_LANE = 1
CMPC_SOLVE_ROWS = 2
CMPC_STEP_AUTO = 0
CMPC_STEP_SPLIT = 1
CMPC_STEP_FUSED = 2


class CmpcDims(ctypes.Structure):
    _fields_ = [("ns", ctypes.c_int32), ("ndist", ctypes.c_int32),
                ("nu_tot", ctypes.c_int32), ("nu", ctypes.c_int32),
                ("ny", ctypes.c_int32), ("p", ctypes.c_int32), ("m", ctypes.c_int32),
                ("delay", ctypes.c_int32 * CMPC_MAX_INPUTS),
                ("S", ctypes.c_int32), ("B", ctypes.c_int32)]

    @classmethod
    def from_config(cls, cfg, B: int) -> "CmpcDims":
        d = cls()
        d.ns, d.ndist, d.nu_tot, d.nu, d.ny = cfg.ns, cfg.ndist, cfg.nu_tot, cfg.nu, cfg.ny
        d.p, d.m, d.S, d.B = cfg.p, cfg.m, cfg.S, B
        for i, v in enumerate(cfg.delays):
            d.delay[i] = v
        return d


class CmpcLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("nd", "n_delay_states", "naug", "nobs", "ntot", "nV", "nuo", "nVo",
                 "off_A", "off_B", "off_C", "off_f", "off_x", "off_y", "rec_len")]


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def uptr(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def bptr(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


# Every symbol include/cmpc.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "cmpc_layout_of", "cmpc_create", "cmpc_destroy", "cmpc_set_stream",
    "cmpc_last_error", "cmpc_get_layout", "cmpc_set_weights", "cmpc_set_constraints",
    "cmpc_set_reference", "cmpc_set_state", "cmpc_get_state", "cmpc_upload_lin",
    "cmpc_lin_device", "cmpc_build", "cmpc_set_build_variant", "cmpc_rows_lds_model", "cmpc_last_build_kernel", "cmpc_set_solve_variant", "cmpc_last_solve_kernel", "cmpc_set_step_variant", "cmpc_last_step_fused", "cmpc_init_warmstart", "cmpc_iterate", "cmpc_step",
    "cmpc_synchronize", "cmpc_download", "cmpc_download_qp", "cmpc_download_trace",
    "cmpc_enable_timing", "cmpc_kernel_time", "cmpc_set_timing_stride", "cmpc_plant_dims", "cmpc_plant_default",
    "cmpc_plant_output", "cmpc_plant_lin_record", "cmpc_qp_solve_batch", "cmpc_qp_solve_batch_map", "cmpc_bind_lin",
    "cmpc_bind_state",
    "cmpc_produce_lin", "cmpc_download_lin", "cmpc_coupled_iterate", "cmpc_coupled_validate",
    "cmpc_get_input", "cmpc_get_input_host", "cmpc_update_u", "cmpc_update_u_host",
    "cmpc_set_observer", "cmpc_observer_len", "cmpc_observer_init", "cmpc_observe_step",
    "cmpc_observe_apply", "cmpc_get_observer_state", "cmpc_set_observer_state",
    "cmpc_observer_init_host", "cmpc_observe_step_host", "cmpc_control_step", "cmpc_control_step_host", "cmpc_control_step_download",
    "cmpc_sim_create", "cmpc_sim_destroy", "cmpc_sim_set_stream", "cmpc_sim_reset",
    "cmpc_sim_set_input", "cmpc_sim_set_offset", "cmpc_sim_restart", "cmpc_sim_plant_input_offset",
    "cmpc_sim_plant_input", "cmpc_sim_integrate", "cmpc_sim_output",
    "cmpc_sim_synchronize", "cmpc_sim_state", "cmpc_sim_input", "cmpc_sim_step_size",
    "cmpc_sim_status", "cmpc_accumulate_moves", "cmpc_sim_download", "cmpc_sim_reset_host",
    "cmpc_sim_set_input_host", "cmpc_sim_set_offset_host", "cmpc_sim_output_host",
)

_lib = None


def load_library(path: str = LIB_PATH):
    """Load libcmpc.so.  Raises (never falls back) if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} not found: build it with `make -C compressor-mpc_amd/csrc` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    # One HIP runtime per process: torch ships its own libamdhip64 (same
    # soname).  Loaded first, it also serves this library; loaded after ours,
    # torch brings in a second runtime that finds no GPU ("No HIP GPUs are
    # available") and whose device pointers and streams ours cannot use.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    c_void = ctypes.c_void_p
    i32, u32, dbl = ctypes.c_int32, ctypes.c_uint32, ctypes.c_double
    sig = {
        "cmpc_layout_of": ([P(CmpcDims), P(CmpcLayout)], ctypes.c_int),
        "cmpc_create": ([P(c_void), P(CmpcDims), ctypes.c_int], ctypes.c_int),
        "cmpc_destroy": ([c_void], ctypes.c_int),
        "cmpc_set_stream": ([c_void, c_void], ctypes.c_int),
        "cmpc_last_error": ([], ctypes.c_char_p),
        "cmpc_get_layout": ([c_void, P(CmpcLayout)], ctypes.c_int),
        "cmpc_set_weights": ([c_void, ctypes.c_int, P(dbl), P(dbl)], ctypes.c_int),
        "cmpc_set_constraints": ([c_void, ctypes.c_int, P(dbl), P(dbl), P(dbl), P(dbl)],
                                 ctypes.c_int),
        "cmpc_set_reference": ([c_void, ctypes.c_int, P(dbl)], ctypes.c_int),
        "cmpc_set_state": ([c_void, P(dbl), P(dbl), P(u32)], ctypes.c_int),
        "cmpc_get_state": ([c_void, P(dbl), P(dbl), P(u32)], ctypes.c_int),
        "cmpc_upload_lin": ([c_void, P(dbl)], ctypes.c_int),
        "cmpc_lin_device": ([c_void], c_void),
        "cmpc_download_lin": ([c_void, P(dbl)], ctypes.c_int),
        "cmpc_bind_lin": ([c_void, c_void], ctypes.c_int),
        "cmpc_bind_state": ([c_void, c_void, c_void, c_void], ctypes.c_int),
        "cmpc_build": ([c_void], ctypes.c_int),
        "cmpc_set_build_variant": ([c_void, ctypes.c_int], ctypes.c_int),
        "cmpc_last_build_kernel": ([c_void], ctypes.c_int),
        "cmpc_set_solve_variant": ([c_void, ctypes.c_int], ctypes.c_int),
        "cmpc_last_solve_kernel": ([c_void], ctypes.c_int),
        "cmpc_set_step_variant": ([c_void, ctypes.c_int], ctypes.c_int),
        "cmpc_last_step_fused": ([c_void], ctypes.c_int),
        "cmpc_rows_lds_model": ([P(CmpcDims), P(dbl), P(dbl), P(ctypes.c_int32)], ctypes.c_int),
        "cmpc_init_warmstart": ([c_void], ctypes.c_int),
        "cmpc_iterate": ([c_void, ctypes.c_int, u32], ctypes.c_int),
        "cmpc_step": ([c_void, ctypes.c_int, u32], ctypes.c_int),
        "cmpc_synchronize": ([c_void], ctypes.c_int),
        "cmpc_download": ([c_void, P(dbl), P(i32), P(i32)], ctypes.c_int),
        "cmpc_download_qp": ([c_void, P(dbl), P(dbl), P(dbl)], ctypes.c_int),
        "cmpc_download_trace": ([c_void, P(ctypes.c_uint8), P(i32)], ctypes.c_int),
        "cmpc_enable_timing": ([c_void, ctypes.c_int], ctypes.c_int),
        "cmpc_set_timing_stride": ([c_void, ctypes.c_int], ctypes.c_int),
        "cmpc_kernel_time": ([c_void, ctypes.c_int, P(dbl), P(ctypes.c_int64)], ctypes.c_int),
        "cmpc_plant_dims": ([ctypes.c_int, P(ctypes.c_int), P(ctypes.c_int), P(ctypes.c_int),
                             P(ctypes.c_int)], ctypes.c_int),
        "cmpc_plant_default": ([ctypes.c_int, P(dbl), P(dbl)], ctypes.c_int),
        "cmpc_plant_output": ([ctypes.c_int, P(dbl), P(dbl)], ctypes.c_int),
        "cmpc_plant_lin_record": ([ctypes.c_int, dbl, dbl, dbl, P(dbl), P(dbl), P(i32), P(i32),
                                   P(CmpcDims), P(dbl)], ctypes.c_int),
        "cmpc_produce_lin": ([c_void, ctypes.c_int, dbl, dbl, dbl, P(i32), P(i32), c_void, c_void,
                              c_void, c_void], ctypes.c_int),
        "cmpc_set_observer": ([c_void, ctypes.c_int, ctypes.c_int, P(dbl)], ctypes.c_int),
        "cmpc_observer_len": ([c_void], ctypes.c_int),
        "cmpc_observer_init": ([c_void, ctypes.c_int, dbl, dbl, dbl, P(i32), P(i32), c_void, c_void,
                                c_void, c_void], ctypes.c_int),
        "cmpc_observe_step": ([c_void, c_void, c_void], ctypes.c_int),
        "cmpc_observe_apply": ([c_void], ctypes.c_int),
        "cmpc_control_step": ([c_void, c_void, c_void, ctypes.c_int], ctypes.c_int),
        "cmpc_control_step_host": ([c_void, P(dbl), P(dbl), ctypes.c_int], ctypes.c_int),
        "cmpc_control_step_download": ([c_void, P(dbl), P(dbl), ctypes.c_int, P(dbl), P(i32), P(i32)],
                                       ctypes.c_int),
        "cmpc_observer_init_host": ([c_void, ctypes.c_int, dbl, dbl, dbl, P(i32), P(i32), P(dbl),
                                     P(dbl), P(dbl), P(dbl)], ctypes.c_int),
        "cmpc_observe_step_host": ([c_void, P(dbl), P(dbl)], ctypes.c_int),
        "cmpc_sim_create": ([P(c_void), ctypes.c_int, ctypes.c_int, ctypes.c_int, dbl, dbl,
                             ctypes.c_int, P(i32), P(i32)], ctypes.c_int),
        "cmpc_sim_destroy": ([c_void], ctypes.c_int),
        "cmpc_sim_set_stream": ([c_void, c_void], ctypes.c_int),
        "cmpc_sim_reset": ([c_void, c_void, c_void, dbl], ctypes.c_int),
        "cmpc_sim_set_input": ([c_void, c_void], ctypes.c_int),
        "cmpc_sim_set_offset": ([c_void, c_void], ctypes.c_int),
        "cmpc_sim_restart": ([c_void, ctypes.c_double], ctypes.c_int),
        "cmpc_sim_plant_input_offset": ([c_void, c_void, c_void, c_void], ctypes.c_int),
        "cmpc_sim_plant_input": ([c_void, c_void, c_void], ctypes.c_int),
        "cmpc_sim_integrate": ([c_void, dbl, dbl, dbl, dbl], ctypes.c_int),
        "cmpc_sim_output": ([c_void, c_void], ctypes.c_int),
        "cmpc_sim_synchronize": ([c_void], ctypes.c_int),
        "cmpc_sim_download": ([c_void, P(dbl), P(dbl), P(dbl), P(i32)], ctypes.c_int),
        "cmpc_sim_reset_host": ([c_void, P(dbl), P(dbl), dbl], ctypes.c_int),
        "cmpc_sim_set_input_host": ([c_void, P(dbl)], ctypes.c_int),
        "cmpc_sim_set_offset_host": ([c_void, P(dbl)], ctypes.c_int),
        "cmpc_sim_output_host": ([c_void, P(dbl)], ctypes.c_int),
        "cmpc_sim_state": ([c_void], c_void),
        "cmpc_sim_input": ([c_void], c_void),
        "cmpc_sim_step_size": ([c_void], c_void),
        "cmpc_sim_status": ([c_void], c_void),
        "cmpc_accumulate_moves": ([c_void, P(i32), c_void], ctypes.c_int),
        "cmpc_get_observer_state": ([c_void, P(dbl)], ctypes.c_int),
        "cmpc_set_observer_state": ([c_void, P(dbl)], ctypes.c_int),
        "cmpc_get_input": ([c_void, c_void, u32], ctypes.c_int),
        "cmpc_get_input_host": ([c_void, P(dbl), u32], ctypes.c_int),
        "cmpc_update_u": ([c_void, c_void], ctypes.c_int),
        "cmpc_update_u_host": ([c_void, P(dbl)], ctypes.c_int),
        "cmpc_coupled_validate": ([P(CmpcDims), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                   ctypes.c_size_t], ctypes.c_int),
        "cmpc_coupled_iterate": ([c_void, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void, ctypes.c_size_t,
                                  c_void, ctypes.c_size_t, c_void, u32], ctypes.c_int),
        "cmpc_qp_solve_batch": ([ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P(dbl),
                                 P(dbl), P(dbl), P(dbl), P(dbl), P(dbl), P(u32), ctypes.c_int,
                                 P(dbl), P(i32), P(i32), P(u32), P(ctypes.c_uint8), P(i32)],
                                ctypes.c_int),
        "cmpc_qp_solve_batch_map": ([ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     P(dbl), P(dbl), P(dbl), P(dbl), P(dbl), P(dbl), P(dbl), P(dbl), P(u32),
                                     ctypes.c_int, P(dbl), P(i32), P(i32), P(u32), P(ctypes.c_uint8), P(i32)],
                                    ctypes.c_int),
    }
    for name, (argtypes, restype) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None:  # (an older library build: A/B timing runs; tests/test_abi.py checks the exports)
            continue
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = lib
    return lib


def check(rc: int, what: str = "cmpc call"):
    if rc != 0:
        msg = load_library().cmpc_last_error()
        raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
