"""Geometry helpers used to build MPC references (host side, float64 numpy).

Restates ``src/common/geometry.py:9-45`` of the reference (resample, heading,
curvature slowdown).  These run once per ``track`` call (setup, not the hot
loop), so they stay on the host exactly as in the reference.
"""
from __future__ import annotations

import numpy as np


def resample_polyline(path, step: float) -> np.ndarray:
    """Resample ``path`` at ~``step`` spacing (``geometry.py:9-29``)."""
    pts = np.asarray(path, dtype=float)
    if len(pts) < 2:
        return pts
    seg = np.diff(pts, axis=0)
    dist = np.hypot(seg[:, 0], seg[:, 1])
    s = np.insert(np.cumsum(dist), 0, 0.0)
    total = s[-1]
    if total < 1e-9:
        return pts
    samples = np.arange(0.0, total, step)
    if not np.isclose(samples[-1], total):
        samples = np.append(samples, total)
    return np.column_stack((np.interp(samples, s, pts[:, 0]), np.interp(samples, s, pts[:, 1])))


def heading_from_path(points: np.ndarray) -> np.ndarray:
    """Unwrapped yaw of successive differences; first yaw is always 0 (``geometry.py:32-36``)."""
    dirs = np.diff(points, axis=0, prepend=points[0:1])
    return np.unwrap(np.arctan2(dirs[:, 1], dirs[:, 0]))


def curvature_slowdown(yaw: np.ndarray) -> np.ndarray:
    """Slowdown factor in [0.6, 1.0] (``geometry.py:39-45``)."""
    hd = np.abs(np.diff(yaw, prepend=yaw[0]))
    hd = np.minimum(hd, np.pi - hd)
    return 0.6 + 0.4 * (1.0 / (1.0 + 4.0 * hd))


def catmull_rom_spline(points, *, samples_per_segment: int = 20, alpha: float = 0.5,
                       eps: float = 1e-9, dedupe_tol: float = 1e-9) -> np.ndarray:
    """Centripetal Catmull-Rom smoothing (``src/planning/rrt_star.py:93-159``).

    Only used to turn RRT* tree branches into paths for the batched scenarios
    (config 3); the planner itself is out of scope.
    """
    raw = np.asarray(points, dtype=float)
    if len(raw) == 0:
        return raw.copy()
    keep = [raw[0]]
    for p in raw[1:]:
        if np.linalg.norm(p - keep[-1]) > dedupe_tol:
            keep.append(p)
    pts = np.asarray(keep)
    n = len(pts)
    if n == 1:
        return pts.copy()
    if n == 2:
        t = np.linspace(0.0, 1.0, max(2, samples_per_segment + 1))
        return (1 - t)[:, None] * pts[0] + t[:, None] * pts[1]
    ext = np.vstack([pts[0], pts, pts[-1]])

    def knot(ti, pi, pj):
        d = np.linalg.norm(pj - pi)
        return ti + ((d ** alpha) if d > eps else eps)

    out = []
    for i in range(n - 1):
        p0, p1, p2, p3 = ext[i], ext[i + 1], ext[i + 2], ext[i + 3]
        t0 = 0.0
        t1 = knot(t0, p0, p1)
        t2 = knot(t1, p1, p2)
        t3 = knot(t2, p2, p3)
        d01, d12, d23 = max(t1 - t0, eps), max(t2 - t1, eps), max(t3 - t2, eps)
        d02, d13 = max(t2 - t0, eps), max(t3 - t1, eps)
        # all samples of the segment at once: the same IEEE operations in the same order per
        # sample as the reference's scalar loop (numpy does not contract), so bit-identical
        t = np.linspace(t1, t2, max(2, samples_per_segment + 1), endpoint=False)[:, None]
        a1 = (t1 - t) / d01 * p0 + (t - t0) / d01 * p1
        a2 = (t2 - t) / d12 * p1 + (t - t1) / d12 * p2
        a3 = (t3 - t) / d23 * p2 + (t - t2) / d23 * p3
        b1 = (t2 - t) / d02 * a1 + (t - t0) / d02 * a2
        b2 = (t3 - t) / d13 * a2 + (t - t1) / d13 * a3
        out.append((t2 - t) / d12 * b1 + (t - t1) / d12 * b2)
    out.append(pts[-1][None, :])
    return np.concatenate(out)


__all__ = ["resample_polyline", "heading_from_path", "curvature_slowdown", "catmull_rom_spline"]
