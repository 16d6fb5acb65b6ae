"""Reference controller configurations (compile-time constants of the reference,
restated as run-time dimensions).

Sources (katie-jones/compressor-mpc):
  include/parallel_compressors_constants.h:68-94   (parallel plant)
  include/serial_compressors_constants.h:82-110    (serial plant)
  include/common-variables.h:20-112                (controller type selection)
  include/parallel_compressors.h:13-23, include/serial_compressors.h:13-30

A configuration fixes, per sub-controller s:
  input_order[s]  ControlInputIndices of its AugmentedLinearizedSystem (own
                  inputs first, then the other controllers' inputs)
  out_idx[s]      ControlledOutputIndices
and the shared dims (ns, ndist, nu_tot, nu, ny, p, m, delays).
"""
from dataclasses import dataclass, field
from typing import List

PLANT_PARALLEL = 0
PLANT_SERIAL = 1

# Delays = ConstexprArray<0, 40, 0, 40>; n_disturbance_states = 4
REF_DELAYS = (0, 40, 0, 40)
REF_NDIST = 4
REF_P = 100
REF_M = 2
REF_TS = 0.05  # sampling time of results/*.dat records
PLANT_N_INPUTS = {PLANT_PARALLEL: 9, PLANT_SERIAL: 8}   # parallel_compressors.h:19, serial_compressors.h:19


@dataclass
class ControllerConfig:
    plant: int
    controller: str                 # "cent" | "coop" | "ncoop"
    ns: int
    nu_tot: int
    nu: int
    ny: int
    input_order: List[List[int]]    # per sub-controller
    out_idx: List[List[int]]        # per sub-controller
    delays: tuple = REF_DELAYS
    ndist: int = REF_NDIST
    p: int = REF_P
    m: int = REF_M

    @property
    def S(self) -> int:
        return len(self.input_order)

    @property
    def nV(self) -> int:
        return self.m * self.nu

    @property
    def nVo(self) -> int:
        return self.m * (self.nu_tot - self.nu)

    def own_inputs(self, s: int) -> List[int]:
        """Plant control-input indices owned by sub-controller s
        (ControlInputIndexType = first nu entries of ControlInputIndices)."""
        return self.input_order[s][: self.nu]

    def with_horizon(self, p: int, m: int = None) -> "ControllerConfig":
        c = ControllerConfig(**{k: getattr(self, k) for k in self.__dataclass_fields__})
        c.p = p
        if m is not None:
            c.m = m
        return c


def reference_config(plant: str, controller: str, p: int = REF_P, m: int = REF_M) -> ControllerConfig:
    """plant: 'par'|'ser'; controller: 'cent'|'coop'|'ncoop'."""
    if plant in ("par", "parallel"):
        pl, ns = PLANT_PARALLEL, 11
        ctrl_out = [0, 1, 3]                       # ControlledOutputIndices
        nc_out = [[0, 3], [1, 3]]                  # NCControlledOutputIndices1/2
    elif plant in ("ser", "serial"):
        pl, ns = PLANT_SERIAL, 10
        ctrl_out = [0, 1, 2, 3]                    # NullIndexArray<4>
        nc_out = [[0, 1], [2, 3]]                  # NCControlledOutputIndices1/2
    else:
        raise ValueError(plant)
    ci1, ci2 = [0, 1, 2, 3], [2, 3, 0, 1]          # ControlInputIndices1/2
    if controller in ("cent", "centralized"):
        return ControllerConfig(pl, "cent", ns, 4, 4, len(ctrl_out), [ci1], [ctrl_out], p=p, m=m)
    if controller in ("coop", "cooperative"):
        return ControllerConfig(pl, "coop", ns, 4, 2, len(ctrl_out), [ci1, ci2],
                                [ctrl_out, ctrl_out], p=p, m=m)
    if controller in ("ncoop", "noncoop"):
        return ControllerConfig(pl, "ncoop", ns, 4, 2, 2, [ci1, ci2], nc_out, p=p, m=m)
    raise ValueError(controller)


@dataclass
class SetupFile:
    """Run parameters of a reference setup file (setup/setup-<ctrl>-<plant>),
    parsed like include/read_files.h:13-81 (key line, then value lines)."""
    n_iterations: int = 1
    n_timing_iterations: int = 1
    yref: List[float] = field(default_factory=list)
    uwt: List[float] = field(default_factory=list)     # n_control_inputs^2
    ywt: List[List[float]] = field(default_factory=list)  # one ny x ny block per sub-controller
    constraints_lower: List[float] = field(default_factory=list)
    constraints_upper: List[float] = field(default_factory=list)
    rate_lower: List[float] = field(default_factory=list)
    rate_upper: List[float] = field(default_factory=list)
    # `simulation`: segments (plant-input offset change from the default input,
    # n_inputs numbers; end time in s).  Each segment's offset holds from the
    # previous segment's end time on (the reference's harness steps the plant
    # input offset, SimulationSystem::SetOffset, simulation_system.h:64).
    segments: List[tuple] = field(default_factory=list)

    KEYS = ("n-iterations", "n-timing-iterations", "folder-name", "output-filename",
            "yref", "uwt", "ywt", "constraints-lower", "constraints-upper",
            "constraints-rate-lower", "constraints-rate-upper", "simulation")

    def text(self, folder: str = "parallel", output: str = "out.dat") -> str:
        """The setup-file layout parse() and the C++ reader (cmpc::SetupFile,
        read_files.h:13-81) read: key line, value lines, blank line."""
        def mat(vals):
            n = int(round(len(vals) ** 0.5))
            return "\n".join("\t".join("%.17g" % v for v in vals[r * n:(r + 1) * n]) for r in range(n))
        parts = [("n-iterations", str(self.n_iterations)),
                 ("n-timing-iterations", str(self.n_timing_iterations)),
                 ("folder-name", folder), ("output-filename", output),
                 ("yref", " ".join("%.17g" % v for v in self.yref)),
                 ("uwt", mat(self.uwt)), ("ywt", "\n\n".join(mat(b) for b in self.ywt)),
                 ("constraints-lower", "\t".join("%.17g" % v for v in self.constraints_lower)),
                 ("constraints-upper", "\t".join("%.17g" % v for v in self.constraints_upper)),
                 ("constraints-rate-lower", "\t".join("%.17g" % v for v in self.rate_lower)),
                 ("constraints-rate-upper", "\t".join("%.17g" % v for v in self.rate_upper))]
        if self.segments:
            parts.append(("simulation", "\n\n".join(" ".join("%.17g" % v for v in d) + "\n%.17g" % te
                                                      for d, te in self.segments)))
        return "".join(f"{k}\n{v}\n\n" for k, v in parts)

    @classmethod
    def parse(cls, text: str, cfg: ControllerConfig) -> "SetupFile":
        blocks, key = {}, None
        for line in text.splitlines():
            s = line.strip()
            if not s or s.startswith("#"):
                continue
            tok = s.split()
            if tok[0] in cls.KEYS:
                key = tok[0]
                blocks.setdefault(key, [])
                continue
            if key is None:
                raise RuntimeError(f"Error reading setup file at line: {line!r}")
            blocks[key].extend(tok)
        num = lambda k: [float(t) for t in blocks.get(k, [])]
        out = cls()
        out.n_iterations = int(num("n-iterations")[0]) if "n-iterations" in blocks else 1
        out.n_timing_iterations = (int(num("n-timing-iterations")[0])
                                   if "n-timing-iterations" in blocks else out.n_iterations)
        out.yref = num("yref")
        out.uwt = num("uwt")
        yw = num("ywt")
        blk = cfg.ny * cfg.ny
        if len(yw) == blk:
            out.ywt = [yw] * cfg.S
        elif len(yw) == blk * cfg.S:
            out.ywt = [yw[i * blk:(i + 1) * blk] for i in range(cfg.S)]
        else:
            raise RuntimeError(f"ywt: expected {blk} or {blk * cfg.S} numbers, got {len(yw)}")
        out.constraints_lower = num("constraints-lower")
        out.constraints_upper = num("constraints-upper")
        out.rate_lower = num("constraints-rate-lower")
        out.rate_upper = num("constraints-rate-upper")
        sim = num("simulation")
        ni = PLANT_N_INPUTS[cfg.plant]
        if len(sim) % (ni + 1):
            raise RuntimeError(f"simulation: segments of {ni} + 1 numbers expected, got {len(sim)}")
        out.segments = [(sim[i:i + ni], sim[i + ni]) for i in range(0, len(sim), ni + 1)]
        return out


# Run parameters of the reference's setup files (setup/setup-<ctrl>-<plant>,
# values copied as data; n-iterations is the Jacobi iteration count K).
# `simulation` blocks: the discharge valve (parallel input 8, default 0.7) and
# the serial plant's input 6 (default 0.393) step at t = 50 s
_PAR_SEG = [([0.0] * 9, 50.0), ([0.0] * 8 + [-0.3], 500.0)]
_SER_SEG = [([0.0] * 8, 50.0), ([0.0] * 6 + [-0.1, 0.0], 500.0)]
_REF_SETUPS = {
    ("par", "cent"): dict(n_iterations=1, yref=[4.5, 4.5, 0, 1.12],
                          uwt=[2e4, 2e5, 2e4, 2e5], ywt=[[1, 1, 5e2]],
                          lo=[-0.3, 0, -0.3, 0], up=[0.3, 1, 0.3, 1],
                          rlo=[-0.1] * 4, rup=[0.1, 1, 0.1, 1], seg=_PAR_SEG),
    ("par", "coop"): dict(n_iterations=9, yref=[4.5, 4.5, 0, 1.12],
                          uwt=[1.9e4, 1.9e5, 1.9e4, 1.9e5], ywt=[[1, 1, 4.2e2]] * 2,
                          lo=[-0.3, 0], up=[0.3, 1], rlo=[-0.1, -0.1], rup=[0.1, 1], seg=_PAR_SEG),
    ("par", "ncoop"): dict(n_iterations=9, yref=[4.5, 4.5, 0, 1.12],
                           uwt=[2.2e4, 2.2e5, 2.2e4, 2.2e5], ywt=[[1, 6e2]] * 2,
                           lo=[-0.3, 0], up=[0.3, 1], rlo=[-0.1, -0.1], rup=[0.1, 1], seg=_PAR_SEG),
    ("ser", "cent"): dict(n_iterations=1, yref=[1.030830, 8.125790, 1.187190, 8.125790],
                          uwt=[2e4, 2.5e5, 2e4, 2.5e5], ywt=[[200, 1, 1000, 8]],
                          lo=[-0.3, 0, -0.3, 0], up=[0.3, 1, 0.3, 1],
                          rlo=[-0.1] * 4, rup=[0.1, 1, 0.1, 1], seg=_SER_SEG),
    ("ser", "coop"): dict(n_iterations=9, yref=[1.030830, 8.125790, 1.187190, 8.125790],
                          uwt=[4.1e4, 5e5, 2.5e4, 5e5], ywt=[[750, 4, 1500, 8]] * 2,
                          lo=[-0.3, 0], up=[0.3, 1], rlo=[-0.1, -0.1], rup=[0.1, 1], seg=_SER_SEG),
    ("ser", "ncoop"): dict(n_iterations=9, yref=[1.030830, 8.125790, 1.187190, 8.125790],
                           uwt=[3e4, 5e5, 3e4, 5e5], ywt=[[1900, 3]] * 2,
                           lo=[-0.3, 0], up=[0.3, 1], rlo=[-0.1, -0.1], rup=[0.1, 1], seg=_SER_SEG),
}


def reference_observer_gain(cfg: ControllerConfig, n_outputs: int = 4):
    """The observer gain M of the reference's runs ((ns + ndist) x n_outputs,
    one per sub-controller): M = [0; I], the measured output error corrects
    the disturbance states only, at unit gain.  The gain is set in the
    harness's missing common-simulation.inc; it is identified from the
    recorded trajectories (tools/fit_observer_gain.py: every other gain of
    the form [0; g I] changes u(t) within the first steps), and with it the
    device closed loop reproduces all 10 000 records of all six reference
    runs (tests/test_closed_loop_golden.py)."""
    import numpy as np
    M = np.zeros((cfg.ns + cfg.ndist, n_outputs))
    M[cfg.ns:cfg.ns + cfg.ndist, :cfg.ndist] = np.eye(cfg.ndist, min(cfg.ndist, n_outputs))
    return M


def reference_setup(plant: str, controller: str) -> SetupFile:
    """The reference's setup file for (plant, controller) as a SetupFile
    (diagonal weight matrices expanded)."""
    key = ({"parallel": "par", "serial": "ser"}.get(plant, plant),
           {"centralized": "cent", "cooperative": "coop", "noncoop": "ncoop"}.get(controller, controller))
    v = _REF_SETUPS[key]
    diag = lambda d: [float(d[i]) if i == j else 0.0 for i in range(len(d)) for j in range(len(d))]
    return SetupFile(n_iterations=v["n_iterations"], n_timing_iterations=v["n_iterations"],
                     yref=[float(t) for t in v["yref"]], uwt=diag(v["uwt"]),
                     ywt=[diag(w) for w in v["ywt"]], constraints_lower=list(map(float, v["lo"])),
                     constraints_upper=list(map(float, v["up"])),
                     rate_lower=list(map(float, v["rlo"])), rate_upper=list(map(float, v["rup"])),
                     segments=[(list(d), t) for d, t in v["seg"]])
