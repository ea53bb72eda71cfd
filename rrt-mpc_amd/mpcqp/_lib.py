"""ctypes binding of ``libmpcqp.so`` (the C-ABI of ``include/mpcqp.h``).

The shared library is built in-tree by ``__graft_entry__.build()`` (hipcc,
``--offload-arch=gfx950``) next to this file.  There is no fallback: if the
library is missing or fails to load, every solver entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

import numpy as np

LIB_NAME = "libmpcqp.so"
LIB_PATH = Path(os.environ.get("MPCQP_LIB", Path(__file__).resolve().parent / LIB_NAME))

# constants mirrored from include/mpcqp.h
MAX_HORIZON = 1024
WIDE_MIN_HORIZON = 33  # MPCQP_WIDE_MIN_HORIZON: a workgroup per QP from here on (N <= 32: one wave)
SOLVED = 1
SOLVED_INACCURATE = 2
MAX_ITER_REACHED = -2
NUMERICAL_ERROR = -10
METHOD_ADMM = 0
METHOD_NEWTON = 1
STATUS_NAMES = {
    SOLVED: "solved",
    SOLVED_INACCURATE: "solved_inaccurate",
    MAX_ITER_REACHED: "maximum_iterations_reached",
    NUMERICAL_ERROR: "numerical_error",
}

# OSQP settings used by the reference (src/control/mpc_controller.py:121-131) plus the
# OSQP defaults it relies on implicitly.
ABI_VERSION = 9  # MPCQP_ABI_VERSION (include/mpcqp.h)
# two QPs per wave for N <= 15 (mpcqp_set_pairing)
PAIR_OFF, PAIR_ON, PAIR_AUTO = 0, 1, 2
PAIRING_MODES = {"off": PAIR_OFF, "on": PAIR_ON, "auto": PAIR_AUTO}
E_DEVICE = -6  # MPCQP_E_DEVICE: a fault surfaced at a stream synchronisation

DEFAULT_SOLVER_SETTINGS = dict(
    rho=0.1,
    sigma=1e-6,
    alpha=1.6,
    eps_abs=1e-3,
    eps_rel=1e-3,
    adaptive_rho_tolerance=5.0,
    max_iter=60000,
    check_termination=25,
    # one Ruiz pass (OSQP's default is 10): on these condensed MPC QPs it halves the ADMM iterations
    # and the worst QPs' polish passes at every horizon and parameter variant measured, with the
    # same optimum and active sets (profiles/r03_s14_*); scaling=10 is OSQP's setting
    scaling=1,
    adaptive_rho=1,
    adaptive_rho_interval=25,
    polish=1,
    polish_max_iter=100,
    debug_state=0,
    polish_from=75,  # with one Ruiz pass; 150 was the tail-tuned choice under OSQP's 10 passes
    polish_attempt_max_iter=30,
    polish_near=3.0,
    reproducible=0,
)


class MpcqpParams(ctypes.Structure):
    """``mpcqp_params`` (include/mpcqp.h)."""

    _fields_ = [
        ("horizon", ctypes.c_int32),
        ("method", ctypes.c_int32),
        ("wheelbase_px", ctypes.c_double),
        ("dt", ctypes.c_double),
        ("q", ctypes.c_double * 16),
        ("r", ctypes.c_double * 4),
        ("q_terminal", ctypes.c_double * 16),
        ("u_bounds", ctypes.c_double * 4),
        ("v_bounds", ctypes.c_double * 2),
        ("du_bounds", ctypes.c_double * 4),
        ("slack_velocity", ctypes.c_double),
        ("slack_input", ctypes.c_double),
        ("slack_rate", ctypes.c_double),
        ("rho", ctypes.c_double),
        ("sigma", ctypes.c_double),
        ("alpha", ctypes.c_double),
        ("eps_abs", ctypes.c_double),
        ("eps_rel", ctypes.c_double),
        ("adaptive_rho_tolerance", ctypes.c_double),
        ("max_iter", ctypes.c_int32),
        ("check_termination", ctypes.c_int32),
        ("scaling", ctypes.c_int32),
        ("adaptive_rho", ctypes.c_int32),
        ("adaptive_rho_interval", ctypes.c_int32),
        ("polish", ctypes.c_int32),
        ("polish_max_iter", ctypes.c_int32),
        ("debug_state", ctypes.c_int32),
        ("polish_from", ctypes.c_int32),
        ("polish_attempt_max_iter", ctypes.c_int32),
        ("polish_near", ctypes.c_double),
        ("reproducible", ctypes.c_int32),
    ]


def to_c_params(params, method: int = METHOD_ADMM, **settings) -> MpcqpParams:
    """Fill ``mpcqp_params`` from an ``MPCParameters``-like object (mpc_controller.py:17-30)."""
    c = MpcqpParams()
    c.horizon = int(params.horizon)
    c.method = int(method)
    c.wheelbase_px = float(params.wheelbase_px)
    c.dt = float(params.dt)
    c.q[:] = [float(v) for v in np.asarray(params.q, dtype=float).reshape(16)]
    c.r[:] = [float(v) for v in np.asarray(params.r, dtype=float).reshape(4)]
    c.q_terminal[:] = [float(v) for v in np.asarray(params.q_terminal, dtype=float).reshape(16)]
    c.u_bounds[:] = [float(v) for v in np.asarray(params.u_bounds, dtype=float).reshape(4)]
    c.v_bounds[:] = [float(v) for v in np.asarray(params.v_bounds, dtype=float).reshape(2)]
    c.du_bounds[:] = [float(v) for v in np.asarray(params.du_bounds, dtype=float).reshape(4)]
    c.slack_velocity = float(getattr(params, "slack_velocity", 1e3))
    c.slack_input = float(getattr(params, "slack_input", 5e2))
    c.slack_rate = float(getattr(params, "slack_rate", 5e2))
    merged = dict(DEFAULT_SOLVER_SETTINGS)
    merged.update(settings)
    for key, value in merged.items():
        setattr(c, key, value)
    return c


REF_BAD_PATH = -2147483648
REF_MAX_POINTS = 6144
FLEET_RUNNING = 0
FLEET_GOAL = 1
FLEET_ABORTED = 2
FLEET_OUT_OF_STEPS = 3
FLEET_REPLAN_RUNNING = 4  # transient inside mpcqp_swarm_step
FLEET_REPLAN_ABORTED = 5
CATMULL_MAX_POINTS = 4096  # deduplicated points per path of mpcqp_catmull_rom


class MpcqpFleet(ctypes.Structure):
    """``mpcqp_fleet`` (include/mpcqp.h): device pointers of the closed-loop fleet state."""

    _fields_ = [
        ("vehicles", ctypes.c_int32),
        ("ref_stride", ctypes.c_int32),
        ("max_steps", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("ref_global", ctypes.c_void_p),
        ("ref_len", ctypes.c_void_p),
        ("goal", ctypes.c_void_p),
        ("state", ctypes.c_void_p),
        ("u_prev", ctypes.c_void_p),
        ("path_idx", ctypes.c_void_p),
        ("phase", ctypes.c_void_p),
        ("steps", ctypes.c_void_p),
        ("mask", ctypes.c_void_p),
        ("status", ctypes.c_void_p),
        ("u0", ctypes.c_void_p),
        ("X", ctypes.c_void_p),
        ("trace", ctypes.c_void_p),
        ("u_trace", ctypes.c_void_p),
    ]


class MpcqpRrtParams(ctypes.Structure):
    """``mpcqp_rrt_params`` (include/mpcqp.h)."""

    _fields_ = [
        ("step", ctypes.c_double),
        ("goal_radius", ctypes.c_double),
        ("rewire_radius", ctypes.c_double),
        ("collision_step", ctypes.c_double),
        ("goal_sample_rate", ctypes.c_double),
        ("max_iterations", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


RRT_MAX_ITERATIONS = 5000


class MpcqpSwarm(ctypes.Structure):
    """``mpcqp_swarm`` (include/mpcqp.h): replan trigger + device replanning of the config-5 swarm."""

    _fields_ = [
        ("rrt", MpcqpRrtParams),
        ("occupancy", ctypes.c_void_p),
        ("prune", ctypes.c_int32),
        ("spline_samples", ctypes.c_int32),
        ("spline_alpha", ctypes.c_double),
        ("dedupe_tol", ctypes.c_double),
        ("desired_speed", ctypes.c_double),
        ("dt", ctypes.c_double),
        ("horizon", ctypes.c_int32),
        ("max_replans", ctypes.c_int32),
        ("replan_distance", ctypes.c_double),
        ("path_cap", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("rng_table", ctypes.c_void_p),
        ("replans", ctypes.c_void_p),
        ("replan_step", ctypes.c_void_p),
        ("start_goal", ctypes.c_void_p),
        ("nodes", ctypes.c_void_p),
        ("count", ctypes.c_void_p),
        ("meta", ctypes.c_void_p),
        ("raw", ctypes.c_void_p),
        ("raw_len", ctypes.c_void_p),
        ("pruned", ctypes.c_void_p),
        ("pruned_len", ctypes.c_void_p),
        ("smooth", ctypes.c_void_p),
        ("smooth_len", ctypes.c_void_p),
        ("new_ref", ctypes.c_void_p),
        ("new_len", ctypes.c_void_p),
    ]


class LibraryError(RuntimeError):
    """A library call refused its arguments or failed to launch (mpcqp_* return code)."""


class DeviceError(RuntimeError):
    """The HIP runtime reported a failure outside a launch: an allocation, or a stream sync at which
    an earlier kernel's fault surfaced (sticky: the device context is unusable afterwards).  Not a
    LibraryError, so the drop-in's map-a-failed-solve-to-None path never swallows it."""


_lib: Optional[ctypes.CDLL] = None

_SYMBOLS = {
    "mpcqp_version": ([], ctypes.c_int),
    "mpcqp_last_error": ([], ctypes.c_char_p),
    "mpcqp_build_id": ([], ctypes.c_char_p),
    "mpcqp_num_rows": ([ctypes.c_int], ctypes.c_int),
    "mpcqp_create": ([ctypes.POINTER(MpcqpParams), ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)],
                     ctypes.c_int),
    "mpcqp_set_params": ([ctypes.c_void_p, ctypes.POINTER(MpcqpParams)], ctypes.c_int),
    "mpcqp_destroy": ([ctypes.c_void_p], None),
    "mpcqp_build": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                     ctypes.c_void_p], ctypes.c_int),
    "mpcqp_solve": ([ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 7, ctypes.c_int),
    "mpcqp_fleet_step": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MpcqpFleet), ctypes.c_void_p],
                         ctypes.c_int),
    "mpcqp_fleet_run": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MpcqpFleet), ctypes.c_int, ctypes.c_int,
                         ctypes.c_void_p], ctypes.c_int),
    "mpcqp_fleet_loop": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MpcqpFleet), ctypes.c_int,
                          ctypes.c_void_p], ctypes.c_int),
    "mpcqp_build_reference": ([ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
                               ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p], ctypes.c_int),
    "mpcqp_rrt_plan": ([ctypes.POINTER(MpcqpRrtParams), ctypes.c_int] + [ctypes.c_void_p] * 8, ctypes.c_int),
    "mpcqp_rrt_paths": ([ctypes.POINTER(MpcqpRrtParams), ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 9,
                        ctypes.c_int),
    "mpcqp_inflate": ([ctypes.c_int] * 4 + [ctypes.c_void_p] * 3, ctypes.c_int),
    "mpcqp_plan_math": ([ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 6, ctypes.c_int),
    "mpcqp_catmull_rom": ([ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                           ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p],
                          ctypes.c_int),
    "mpcqp_swarm_step": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MpcqpFleet), ctypes.POINTER(MpcqpSwarm),
                          ctypes.c_void_p], ctypes.c_int),
    "mpcqp_swarm_run": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MpcqpFleet), ctypes.POINTER(MpcqpSwarm),
                         ctypes.c_int, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
    "mpcqp_swarm_loop": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MpcqpFleet), ctypes.POINTER(MpcqpSwarm),
                          ctypes.c_void_p], ctypes.c_int),
    "mpcqp_model_buffer": ([ctypes.c_void_p], ctypes.c_void_p),
    "mpcqp_model_stride": ([ctypes.c_int], ctypes.c_int),
    "mpcqp_state_buffer": ([ctypes.c_void_p], ctypes.c_void_p),
    "mpcqp_state_stride": ([ctypes.c_int], ctypes.c_int),
    "mpcqp_ws_state_stride": ([ctypes.c_void_p], ctypes.c_int),
    "mpcqp_debug_wave_ops": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_int),
    "mpcqp_debug_stamps": ([ctypes.c_void_p, ctypes.c_int], ctypes.c_int),
    "mpcqp_debug_serve_fault": ([ctypes.c_void_p, ctypes.c_int], ctypes.c_int),
    "mpcqp_stage": ([ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                     ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
    "mpcqp_solve_staged": ([ctypes.c_void_p], ctypes.c_int),
    "mpcqp_solve_served": ([ctypes.c_void_p], ctypes.c_int),
    "mpcqp_set_pairing": ([ctypes.c_void_p, ctypes.c_int], ctypes.c_int),
}


def build_id() -> str:
    """mpcqp_build_id() of the loaded library."""
    return lib().mpcqp_build_id().decode()


def exported_symbols():
    return list(_SYMBOLS)


def lib() -> ctypes.CDLL:
    """Load ``libmpcqp.so``; raises ``LibraryError`` (no fallback) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise LibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950).  The MPC solver has no CPU fallback."
        )
    handle = ctypes.CDLL(str(LIB_PATH))
    any_abi = bool(os.environ.get("MPCQP_ABI_ANY"))
    for name, (argtypes, restype) in _SYMBOLS.items():
        if any_abi and not hasattr(handle, name):  # an older build lacks the newer entry points
            continue
        fn = getattr(handle, name)
        fn.argtypes = argtypes
        fn.restype = restype
    # MPCQP_ABI_ANY: development A/B runs against an older kernel build (tools/diag)
    if handle.mpcqp_version() != ABI_VERSION and not any_abi:
        raise LibraryError(f"libmpcqp ABI version {handle.mpcqp_version()} != {ABI_VERSION}")
    _lib = handle
    return handle


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().mpcqp_last_error().decode(errors="replace")
        raise LibraryError(f"{what} failed ({rc}): {msg}")


__all__ = [
    "MpcqpParams",
    "MpcqpFleet",
    "MpcqpRrtParams",
    "MpcqpSwarm",
    "RRT_MAX_ITERATIONS",
    "FLEET_REPLAN_RUNNING",
    "FLEET_REPLAN_ABORTED",
    "CATMULL_MAX_POINTS",
    "to_c_params",
    "REF_BAD_PATH",
    "REF_MAX_POINTS",
    "FLEET_RUNNING",
    "FLEET_GOAL",
    "FLEET_ABORTED",
    "FLEET_OUT_OF_STEPS",
    "lib",
    "check",
    "LibraryError",
    "DeviceError",
    "DEFAULT_SOLVER_SETTINGS",
    "STATUS_NAMES",
    "SOLVED",
    "SOLVED_INACCURATE",
    "MAX_ITER_REACHED",
    "NUMERICAL_ERROR",
    "METHOD_ADMM",
    "METHOD_NEWTON",
    "MAX_HORIZON",
    "exported_symbols",
]
