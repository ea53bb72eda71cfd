"""Reference trajectory construction (``src/control/ref_builder.py:10-22``)."""
from __future__ import annotations

import numpy as np

from ..common.geometry import curvature_slowdown, heading_from_path, resample_polyline


def build_reference(path, desired_speed: float, horizon: int, dt: float) -> np.ndarray:
    """Return an ``(M, 4)`` reference ``[x, y, yaw, v]`` with ``M >= horizon + 1``."""
    step = max(2.0, 0.8 * desired_speed * dt)
    pts = resample_polyline(path, step)
    yaw = heading_from_path(pts)
    vref = desired_speed * curvature_slowdown(yaw)
    xref = np.column_stack((pts[:, 0], pts[:, 1], yaw, vref))
    if len(xref) < horizon + 1:
        xref = np.vstack((xref, np.repeat(xref[-1:], horizon + 1 - len(xref), axis=0)))
    return xref


__all__ = ["build_reference"]
