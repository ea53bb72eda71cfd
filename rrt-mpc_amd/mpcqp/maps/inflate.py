"""Occupancy-grid inflation on the GPU: drop-in for ``src/maps/inflate.py``.

Same functions and results as the reference (``inflate.py:12-66``; without OpenCV the reference
uses its disk-kernel fallback dilation, which ``mpcqp_inflate`` restates on the device).
Accepts numpy arrays (returned as numpy) or CUDA uint8 tensors (returned on the device).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _lib


def inflation_radius_pixels(radius_m: float, resolution_m: float) -> int:
    """``inflate.py:12-15``."""
    return int(np.ceil(radius_m / resolution_m))


def inflate_binary_occupancy(occupancy, radius_px: int, *, device=None):
    """``inflate.py:40-51`` (1 = free, 0 = obstacle); a (B, H, W) stack inflates B grids."""
    import torch

    if not torch.cuda.is_available():
        raise _lib.LibraryError("inflate_binary_occupancy needs a ROCm GPU; there is no CPU fallback")
    on_device = isinstance(occupancy, torch.Tensor)
    dev = occupancy.device if on_device else (torch.device(device) if device is not None else torch.device("cuda"))
    t = occupancy if on_device else torch.from_numpy(np.ascontiguousarray(occupancy, dtype=np.uint8))
    t = t.to(device=dev, dtype=torch.uint8).contiguous()
    shape = tuple(t.shape)
    g = t.reshape((-1,) + shape[-2:])
    out = torch.empty_like(g)
    L = _lib.lib()
    with torch.cuda.device(dev):
        _lib.check(L.mpcqp_inflate(g.shape[0], g.shape[1], g.shape[2], int(radius_px), g.data_ptr(), out.data_ptr(),
                                   ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "mpcqp_inflate")
    out = out.reshape(shape)
    return out if on_device else out.cpu().numpy()


def to_occupancy_grid(img: np.ndarray) -> np.ndarray:
    """``inflate.py:63-66``."""
    return (np.asarray(img) > 200).astype(np.uint8)


def inflate_grayscale_map(img: np.ndarray, radius_m: float, resolution_m: float) -> np.ndarray:
    """``inflate.py:54-60``: white free, black occupied."""
    radius_px = inflation_radius_pixels(radius_m, resolution_m)
    occupancy = to_occupancy_grid(img)
    inflated = inflate_binary_occupancy(occupancy, radius_px)
    return (inflated * 255).astype(np.uint8)


__all__ = ["inflation_radius_pixels", "inflate_binary_occupancy", "inflate_grayscale_map", "to_occupancy_grid"]
