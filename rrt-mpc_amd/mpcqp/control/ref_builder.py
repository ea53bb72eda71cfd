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


class PackedPaths:
    """Polylines packed for the device: ``pts`` (P, 2) float64, every path's points in order, and
    ``off`` (V + 1,) int32, path ``v`` in rows ``[off[v], off[v + 1])``.  One pass over the paths,
    shared by ``build_reference_batch`` and the fleet's start states (``fleet.initial_states``)."""

    def __init__(self, paths):
        self.V = V = len(paths)
        pts = None
        if V:  # one C-level concatenation of (k, 2) point arrays / lists (no per-path conversion)
            try:
                counts = np.fromiter(map(len, paths), dtype=np.int64, count=V)
                cat = np.concatenate(paths, axis=0).astype(float, copy=False)
                if cat.ndim == 2 and cat.shape == (int(counts.sum()), 2):
                    pts = cat
            except (ValueError, TypeError):
                pts = None
        if pts is None:  # ragged / empty / unusual element types: per path
            arrs = [np.asarray(q, dtype=float).reshape(-1, 2) for q in paths]
            counts = np.array([len(a) for a in arrs], dtype=np.int64)
            pts = np.concatenate(arrs) if V else np.zeros((0, 2))
        self.counts = counts if V else np.zeros(0, dtype=np.int64)
        self.off = np.zeros(V + 1, dtype=np.int32)
        self.off[1:] = np.cumsum(self.counts)
        self.pts = pts if len(pts) else np.zeros((1, 2))

    @property
    def arrs(self):
        """Path v's points as a view of ``pts``."""
        return [self.pts[self.off[v]:self.off[v + 1]] for v in range(self.V)]


def build_reference_batch(paths, desired_speed: float, horizon: int, dt: float, *, device=None,
                          ref_stride: int | None = None, stream=None, packed: PackedPaths | None = None):
    """``build_reference`` for many paths at once on the GPU (``mpcqp_build_reference``).

    Returns ``(ref, ref_len)`` as device tensors: ``ref`` is ``(V, ref_stride, 4)`` float64 with
    polyline ``v``'s reference in rows ``[0, ref_len[v])`` (identical to ``build_reference`` of that
    path, up to an ulp of ``hypot``/``atan2``), ``ref_len`` is ``(V,)`` int32.  ``ref_stride``
    defaults to an upper bound computed on the host from the path lengths.  ``packed``: the paths
    already packed (``PackedPaths(paths)``), so the caller's pass over them is not repeated.
    """
    import ctypes

    import torch

    from .. import _lib

    if not torch.cuda.is_available():
        raise _lib.LibraryError("build_reference_batch needs a ROCm GPU; there is no CPU fallback")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    pk = packed if packed is not None else PackedPaths(paths)
    V, counts, off = pk.V, pk.counts, pk.off
    max_points = int(counts.max()) if V else 0
    if max_points > _lib.REF_MAX_POINTS:
        raise ValueError(f"a path has {max_points} points; at most {_lib.REF_MAX_POINTS} are supported")
    step = max(2.0, 0.8 * desired_speed * dt)
    if ref_stride is None:  # resampled rows <= ceil(arc length / step) + 1, raw rows = points
        arrs = pk.arrs
        arc = [float(np.hypot(*np.diff(a, axis=0).T).sum()) if len(a) > 1 else 0.0 for a in arrs]
        bound = max([max(int(np.ceil(s / step)) + 2, len(a)) for s, a in zip(arc, arrs)], default=1)
        ref_stride = max(bound, horizon + 1)
    pts = torch.from_numpy(pk.pts).to(dev)
    off_t = torch.from_numpy(off).to(dev)
    ref = torch.empty((max(V, 1), ref_stride, 4), dtype=torch.float64, device=dev)
    ref_len = torch.empty((max(V, 1),), dtype=torch.int32, device=dev)
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    L = _lib.lib()
    with torch.cuda.device(dev):
        _lib.check(L.mpcqp_build_reference(V, pts.data_ptr(), off_t.data_ptr(), max_points, float(desired_speed),
                                           int(horizon), float(dt), int(ref_stride), ref.data_ptr(),
                                           ref_len.data_ptr(), ctypes.c_void_p(stream.cuda_stream)),
                   "mpcqp_build_reference")
    return ref[:V], ref_len[:V]


__all__ = ["build_reference", "build_reference_batch"]
