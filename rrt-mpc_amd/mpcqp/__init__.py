"""mpcqp -- MI355X-native batched bicycle-MPC QP solver (hot path of CagriCatik/RRT-MPC).

Public surface mirrors the reference modules it replaces:

* ``mpcqp.control.mpc_controller``  -> ``src/control/mpc_controller.py``
  (``MPCParameters``, ``MPCController``; plus ``BatchedMPCController``)
* ``mpcqp.pipeline.control_stage``  -> ``src/pipeline/control_stage.py``
  (``TrajectoryTracker`` with ``track`` and ``step``)
* ``mpcqp.config``                  -> ``MPCConfig`` / ``VizConfig`` of ``src/config.py``
* ``mpcqp.control.vehicle_model`` / ``ref_builder`` / ``common.geometry``

The numerics run in ``libmpcqp.so`` (``csrc/mpcqp.hip``, C-ABI ``include/mpcqp.h``).
"""
from __future__ import annotations

__version__ = "0.1.0"

from . import _lib  # noqa: F401  (binding; loads lazily)
from .config import MPCConfig, VizConfig  # noqa: E402
from .control.mpc_controller import BatchedMPCController, MPCController, MPCParameters  # noqa: E402
from .pipeline.control_stage import TrackingResult, TrajectoryTracker  # noqa: E402

__all__ = [
    "MPCConfig",
    "VizConfig",
    "MPCParameters",
    "MPCController",
    "BatchedMPCController",
    "TrajectoryTracker",
    "TrackingResult",
]
