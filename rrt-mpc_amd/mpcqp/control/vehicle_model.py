"""Kinematic bicycle model in pixel coordinates (``src/control/vehicle_model.py:1-45``).

Host-side numpy, used for the plant step of the closed loop
(``src/pipeline/control_stage.py:127``).  The per-step Jacobians of the MPC
are evaluated on the GPU by ``k_build`` (``csrc/mpcqp.hip``); ``linearize`` here
is kept for API compatibility with the reference module.
"""
from __future__ import annotations

import math

import numpy as np
import numpy.typing as npt

State = npt.NDArray[np.float64]
Control = npt.NDArray[np.float64]


def f_discrete(x: State, u: Control, dt: float, wheelbase_px: float) -> State:
    """Forward Euler integration of the bicycle model (``vehicle_model.py:11-21``).

    The same IEEE operations in the same order as the reference.  cos / sin of one float64 are
    numpy's libm calls, so ``math.cos`` / ``math.sin`` return the same bits (a plain call instead of
    a ufunc dispatch: this runs once per closed-loop step); ``np.tan`` is numpy's own SIMD kernel,
    which differs from libm's tan in the last ulp on ~0.5 % of arguments, so it stays.  The operands
    are taken as Python floats (IEEE double arithmetic, the same bits as on numpy float64 scalars,
    without their per-operation dispatch).
    ``tests/test_host.py`` holds the result to the reference's bit for bit (``vehicle.npz``)."""
    xk, yk, yaw, v = (x.tolist() if type(x) is np.ndarray else [float(t) for t in x])
    a, delta = (u.tolist() if type(u) is np.ndarray else [float(t) for t in u])
    dt, wheelbase_px = float(dt), float(wheelbase_px)
    tan_d = float(np.tan(delta))
    return np.array(
        [
            xk + dt * v * math.cos(yaw),
            yk + dt * v * math.sin(yaw),
            yaw + dt * (v / wheelbase_px) * tan_d,
            v + dt * a,
        ],
        dtype=float,
    )


def linearize(x: State, u: Control, dt: float, wheelbase_px: float):
    """Discrete-time Jacobians ``A``, ``B`` and ``f(x, u)`` (``vehicle_model.py:24-45``)."""
    _, _, yaw, v = x
    _, delta = u
    c, s = np.cos(yaw), np.sin(yaw)
    sec2_d = 1.0 / (np.cos(delta) ** 2 + 1e-9)
    A = np.eye(4)
    A[0, 2] = -dt * v * s
    A[0, 3] = dt * c
    A[1, 2] = dt * v * c
    A[1, 3] = dt * s
    A[2, 3] = dt * (1.0 / wheelbase_px) * np.tan(delta)
    B = np.zeros((4, 2))
    B[3, 0] = dt
    B[2, 1] = dt * (v / wheelbase_px) * sec2_d
    return A, B, f_discrete(x, u, dt, wheelbase_px)


__all__ = ["f_discrete", "linearize"]
