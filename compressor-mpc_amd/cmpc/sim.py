"""Batched plant simulation on the GPU — the
reference harness's SimulationSystem (include/simulation_system.h) for B
scenarios: input delay line (TimeDelay, time_delay.h:41-58), controlled
Dormand-Prince over one sampling interval per call (integrate_const,
simulation_system.h:108-116), plant outputs.  Arrays are torch tensors on
the device (plumbing: the simulation itself is the HIP kernel in sim.hip)."""
import ctypes

import numpy as np

from ._abi import check, load_library

REF_DELAYS = (0, 40, 0, 40)          # Delays of both plants (control-input order)
REF_CONTROL_INDEX = (0, 3, 4, 7)     # ControlInputIndex: plant input of each control input
REF_TS = 0.05                        # sampling time of results/*.dat
REF_EPS = 1e-6                       # Integrate's max_rel_error / max_abs_error


class PlantSimulator:
    """SimulationSystem for B scenarios of one plant (0 parallel, 1 serial)."""

    def __init__(self, plant: int, B: int, device: int = 0, p_in: float = 1.0, p_out: float = 1.0,
                 delays=REF_DELAYS, control_index=REF_CONTROL_INDEX):
        import torch
        self.torch = torch
        self.lib = load_library()
        self.plant, self.B, self.device = plant, B, device
        ns, ni, no, nci = (ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int())
        check(self.lib.cmpc_plant_dims(plant, ctypes.byref(ns), ctypes.byref(ni), ctypes.byref(no),
                                       ctypes.byref(nci)), "cmpc_plant_dims")
        self.ns, self.ni, self.no = ns.value, ni.value, no.value
        self.nc = len(delays)
        d = np.ascontiguousarray(delays, dtype=np.int32)
        ci = np.ascontiguousarray(control_index, dtype=np.int32)
        if torch.cuda.is_available():
            torch.cuda.init()  # torch's HIP runtime before the library's
        self._h = ctypes.c_void_p()
        check(self.lib.cmpc_sim_create(ctypes.byref(self._h), plant, B, device, p_in, p_out, self.nc,
                                       d.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       ci.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))),
              "cmpc_sim_create")
        self.y = torch.zeros(B, self.no, dtype=torch.float64, device=f"cuda:{device}")
        # the caller's tensors are written on torch's stream: run there too
        self.set_stream(torch.cuda.current_stream(device).cuda_stream)

    def close(self):
        if self._h:
            self.lib.cmpc_sim_destroy(self._h)
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

    def set_stream(self, stream_ptr: int):
        check(self.lib.cmpc_sim_set_stream(self._h, ctypes.c_void_p(stream_ptr)), "cmpc_sim_set_stream")

    def reset(self, x0, u_offset, dt0: float = REF_TS):
        """x0 (B, ns), u_offset (B, n_inputs): device tensors (float64)."""
        check(self.lib.cmpc_sim_reset(self._h, ctypes.c_void_p(x0.data_ptr()),
                                      ctypes.c_void_p(u_offset.data_ptr()), dt0), "cmpc_sim_reset")

    def set_input(self, u_control):
        """SetInput: u_control (B, n_control) device tensor through the delay line."""
        check(self.lib.cmpc_sim_set_input(self._h, ctypes.c_void_p(u_control.data_ptr())),
              "cmpc_sim_set_input")

    def set_offset(self, u_offset):
        """SetOffset: u_offset (B, n_inputs) device tensor; the plant input
        changes with the next set_input."""
        check(self.lib.cmpc_sim_set_offset(self._h, ctypes.c_void_p(u_offset.data_ptr())),
              "cmpc_sim_set_offset")

    def restart(self, dt0: float = REF_TS):
        """A new Integrate call: the carried step size starts again at dt0."""
        check(self.lib.cmpc_sim_restart(self._h, dt0), "cmpc_sim_restart")

    def plant_input_offset(self, u_control, u_offset, out):
        """GetPlantInput over a given offset (the controller's u_offset_)."""
        check(self.lib.cmpc_sim_plant_input_offset(self._h, ctypes.c_void_p(u_control.data_ptr()),
                                                   ctypes.c_void_p(u_offset.data_ptr()),
                                                   ctypes.c_void_p(out.data_ptr())),
              "cmpc_sim_plant_input_offset")

    def plant_input(self, u_control, out):
        """GetPlantInput without the delay line into out (B, n_inputs)."""
        check(self.lib.cmpc_sim_plant_input(self._h, ctypes.c_void_p(u_control.data_ptr()),
                                            ctypes.c_void_p(out.data_ptr())), "cmpc_sim_plant_input")

    def integrate(self, t: float, t_end: float, eps_abs: float = REF_EPS, eps_rel: float = REF_EPS):
        check(self.lib.cmpc_sim_integrate(self._h, t, t_end, eps_abs, eps_rel), "cmpc_sim_integrate")

    def output(self, out=None):
        """GetOutput into out (B, n_outputs) (default: self.y)."""
        out = self.y if out is None else out
        check(self.lib.cmpc_sim_output(self._h, ctypes.c_void_p(out.data_ptr())), "cmpc_sim_output")
        return out

    def synchronize(self):
        check(self.lib.cmpc_sim_synchronize(self._h), "cmpc_sim_synchronize")

    def download(self):
        """Host copies: (x (B, ns), plant input (B, n_inputs), step size (B,), status (B,))."""
        x = np.zeros((self.B, self.ns))
        u = np.zeros((self.B, self.ni))
        dt = np.zeros(self.B)
        st = np.zeros(self.B, np.int32)
        P = ctypes.POINTER
        check(self.lib.cmpc_sim_download(self._h, x.ctypes.data_as(P(ctypes.c_double)),
                                         u.ctypes.data_as(P(ctypes.c_double)),
                                         dt.ctypes.data_as(P(ctypes.c_double)),
                                         st.ctypes.data_as(P(ctypes.c_int32))), "cmpc_sim_download")
        return x, u, dt, st

    def state_ptr(self) -> int:
        return self.lib.cmpc_sim_state(self._h)

    def input_ptr(self) -> int:
        return self.lib.cmpc_sim_input(self._h)
