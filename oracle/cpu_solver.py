"""ctypes binding of ``oracle/build/libmpcqp_cpu.so`` (the C restatement / CPU baseline).

TEST INFRASTRUCTURE ONLY (see ``mpc_oracle.py`` header): used by ``tests/`` and by
``bench.py``'s ``cpu_baseline`` leg.  The parameter struct is declared here
independently of the product so the checker does not depend on the thing checked.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "libmpcqp_cpu.so"


class CParams(ctypes.Structure):
    """``mpcqp_params`` of ``include/mpcqp.h``."""

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
        ("reproducible", ctypes.c_int32),  # product-side kernel choice; the C restatement ignores it
    ]


def make_cparams(params, method: int = 0, **solver) -> CParams:
    """From any object with ``MPCParameters`` fields (reference, product or oracle)."""
    c = CParams()
    c.horizon = int(params.horizon)
    c.method = int(method)
    c.wheelbase_px = float(params.wheelbase_px)
    c.dt = float(params.dt)
    c.q[:] = [float(v) for v in np.asarray(params.q, float).reshape(16)]
    c.r[:] = [float(v) for v in np.asarray(params.r, float).reshape(4)]
    c.q_terminal[:] = [float(v) for v in np.asarray(params.q_terminal, float).reshape(16)]
    c.u_bounds[:] = [float(v) for v in np.asarray(params.u_bounds, float).reshape(4)]
    c.v_bounds[:] = [float(v) for v in np.asarray(params.v_bounds, float).reshape(2)]
    c.du_bounds[:] = [float(v) for v in np.asarray(params.du_bounds, float).reshape(4)]
    c.slack_velocity = float(getattr(params, "slack_velocity", 1e3))
    c.slack_input = float(getattr(params, "slack_input", 5e2))
    c.slack_rate = float(getattr(params, "slack_rate", 5e2))
    settings = dict(rho=0.1, sigma=1e-6, alpha=1.6, eps_abs=1e-3, eps_rel=1e-3, adaptive_rho_tolerance=5.0,
                    max_iter=60000, check_termination=25, scaling=1, adaptive_rho=1, adaptive_rho_interval=25,
                    polish=1, polish_max_iter=100, polish_from=75, polish_attempt_max_iter=30,
                    polish_near=3.0)
    settings.update(solver)  # the defaults are the product's (mpcqp/_lib.py DEFAULT_SOLVER_SETTINGS)
    for k, v in settings.items():
        setattr(c, k, v)
    return c


def build_library(force: bool = False) -> Path:
    if force or not LIB_PATH.exists():
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build_library()
        L = ctypes.CDLL(str(LIB_PATH))
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        bp = ctypes.POINTER(ctypes.c_uint8)
        L.mpcqp_cpu_solve.argtypes = [ctypes.POINTER(CParams), ctypes.c_int, dp, dp, dp, dp, dp, dp, ip, ip, bp, dp,
                                      ctypes.c_int]
        L.mpcqp_cpu_solve.restype = ctypes.c_int
        L.mpcqp_model_stride.argtypes = [ctypes.c_int]
        L.mpcqp_model_stride.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def cpu_solve(params, x0, ref, u_prev=None, *, method: int = 0, nthreads: int = 0, want_model: bool = False,
              **solver):
    """Batched CPU solve.  x0 (B,4), ref (B,N+1,4), u_prev (B,2) float64."""
    L = lib()
    cp = make_cparams(params, method, **solver)
    N = cp.horizon
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(-1, 4)
    B = x0.shape[0]
    ref = np.ascontiguousarray(ref, dtype=np.float64).reshape(B, N + 1, 4)
    up = None if u_prev is None else np.ascontiguousarray(u_prev, dtype=np.float64).reshape(B, 2)
    out = dict(
        u0=np.zeros((B, 2)),
        X=np.zeros((B, 4, N + 1)),
        U=np.zeros((B, 2, N)),
        status=np.zeros(B, np.int32),
        iters=np.zeros((B, 4), np.int32),
        active=np.zeros((B, 5 * N + 1), np.uint8),
    )
    model = np.zeros((B, L.mpcqp_model_stride(N))) if want_model else None
    dp = ctypes.c_double
    rc = L.mpcqp_cpu_solve(
        ctypes.byref(cp), B, _p(x0, dp), _p(ref, dp), None if up is None else _p(up, dp), _p(out["u0"], dp),
        _p(out["X"], dp), _p(out["U"], dp), _p(out["status"], ctypes.c_int32), _p(out["iters"], ctypes.c_int32),
        _p(out["active"], ctypes.c_uint8), None if model is None else _p(model, dp),
        int(nthreads if nthreads else (os.cpu_count() or 1)))
    if rc != 0:
        raise RuntimeError(f"mpcqp_cpu_solve failed: {rc}")
    if model is not None:
        out["model"] = model
    return out


def cpu_solve_models(params, models, *, method: int = 0, nthreads: int = 0, **solver):
    """The solve from given LTV models (B, mpcqp_model_stride(N)) -- e.g. the GPU's K1 output, so
    the device/glibc sin/cos ulps stay out of an iteration-count comparison."""
    L = lib()
    if not hasattr(L, "_models_bound"):
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        bp = ctypes.POINTER(ctypes.c_uint8)
        L.mpcqp_cpu_solve_models.argtypes = [ctypes.POINTER(CParams), ctypes.c_int, dp, dp, dp, dp, ip, ip, bp,
                                             ctypes.c_int]
        L.mpcqp_cpu_solve_models.restype = ctypes.c_int
        L._models_bound = True
    cp = make_cparams(params, method, **solver)
    N = cp.horizon
    models = np.ascontiguousarray(models, dtype=np.float64)
    B = models.shape[0]
    out = dict(
        u0=np.zeros((B, 2)),
        X=np.zeros((B, 4, N + 1)),
        U=np.zeros((B, 2, N)),
        status=np.zeros(B, np.int32),
        iters=np.zeros((B, 4), np.int32),
        active=np.zeros((B, 5 * N + 1), np.uint8),
    )
    dp = ctypes.c_double
    rc = L.mpcqp_cpu_solve_models(ctypes.byref(cp), B, _p(models, dp), _p(out["u0"], dp), _p(out["X"], dp),
                                  _p(out["U"], dp), _p(out["status"], ctypes.c_int32), _p(out["iters"], ctypes.c_int32),
                                  _p(out["active"], ctypes.c_uint8), int(nthreads if nthreads else (os.cpu_count() or 1)))
    if rc != 0:
        raise RuntimeError(f"mpcqp_cpu_solve_models failed: {rc}")
    return out


def cpu_state(params, model: np.ndarray, state_stride: int, **solver) -> np.ndarray:
    """Scaled QP (GPU state layout) for each model row: (B, state_stride)."""
    L = lib()
    if not hasattr(L, "_state_bound"):
        L.mpcqp_cpu_state.argtypes = [ctypes.POINTER(CParams), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double)]
        L.mpcqp_cpu_state.restype = None
        L._state_bound = True
    cp = make_cparams(params, 0, **solver)
    model = np.ascontiguousarray(model, dtype=np.float64)
    out = np.zeros((model.shape[0], state_stride))
    for b in range(model.shape[0]):
        L.mpcqp_cpu_state(ctypes.byref(cp), _p(model[b], ctypes.c_double), _p(out[b], ctypes.c_double))
    return out


__all__ = ["CParams", "make_cparams", "cpu_solve", "cpu_solve_models", "cpu_state", "build_library", "lib"]
