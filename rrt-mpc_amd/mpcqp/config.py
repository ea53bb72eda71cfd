"""MPC configuration (``src/config.py:65-92`` and ``:95-101``), same fields and defaults."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

from .control.mpc_controller import MPCParameters


@dataclass
class MPCConfig:
    wheelbase_m: float = 2.8
    dt: float = 0.1
    horizon: int = 15
    v_px_s: float = 15.0
    sim_steps: int = 300
    q: Tuple[Tuple[float, float, float, float], ...] = (
        (4.0, 0.0, 0.0, 0.0),
        (0.0, 4.0, 0.0, 0.0),
        (0.0, 0.0, 0.6, 0.0),
        (0.0, 0.0, 0.0, 0.1),
    )
    r: Tuple[Tuple[float, float], ...] = ((0.03, 0.0), (0.0, 0.25))
    q_terminal: Tuple[Tuple[float, float, float, float], ...] = (
        (8.0, 0.0, 0.0, 0.0),
        (0.0, 8.0, 0.0, 0.0),
        (0.0, 0.0, 1.0, 0.0),
        (0.0, 0.0, 0.0, 0.2),
    )
    u_bounds: Tuple[Tuple[float, float], Tuple[float, float]] = ((-35.0, 35.0), (-0.6, 0.6))
    v_bounds: Tuple[float, float] = (0.0, 90.0)
    du_bounds: Tuple[Tuple[float, float], Tuple[float, float]] = ((-12.0, 12.0), (-0.15, 0.15))

    def to_parameters(self, map_resolution: float) -> MPCParameters:
        """``config.py:79-92``: the wheelbase is converted from metres to pixels."""
        return MPCParameters(
            wheelbase_px=self.wheelbase_m / map_resolution,
            dt=self.dt,
            horizon=self.horizon,
            q=np.array(self.q, dtype=float),
            r=np.array(self.r, dtype=float),
            q_terminal=np.array(self.q_terminal, dtype=float),
            u_bounds=self.u_bounds,
            v_bounds=self.v_bounds,
            du_bounds=self.du_bounds,
        )


@dataclass
class VizConfig:
    """``config.py:95-101``; visualisation itself is out of scope for this build."""

    backend: str = "auto"
    prediction_pause: float = 0.01
    animate_tree: bool = True
    record_frames: bool = False
    record_dir: str = "frames"


__all__ = ["MPCConfig", "VizConfig"]
