"""MPC-based control stage: drop-in for ``src/pipeline/control_stage.py``.

``TrajectoryTracker(mpc, viz)`` is constructed by concrete name by the
reference's ``PipelineOrchestrator`` (``src/pipeline/orchestrator.py:73``) and keeps
``track`` / ``_solve_with_relaxation`` with the reference's arguments, results and
errors (``control_stage.py:26-157``).  ``step`` (named by the north star, absent in
the reference) is one iteration of the loop body (``:101-129``).  Every QP goes
through ``MPCController`` -> ``libmpcqp.so`` on the GPU.
"""
from __future__ import annotations

import logging
from dataclasses import dataclass, field, replace
from typing import Any, Optional, Sequence, Tuple

import numpy as np

from ..control.mpc_controller import MPCController, MPCParameters
from ..control.ref_builder import build_reference
from ..control.vehicle_model import f_discrete

LOG = logging.getLogger(__name__)


def _reference_tracking_result():
    """The reference's own ``TrackingResult`` when this module runs inside the reference tree
    (``src/pipeline/artifacts.py:33-38``), so ``PipelineResult`` holds the class it declares."""
    try:  # pragma: no cover - only inside the reference tree
        from src.pipeline.artifacts import TrackingResult as ref_cls  # type: ignore

        return ref_cls
    except Exception:
        return None


@dataclass
class TrackingResult:
    """``src/pipeline/artifacts.py:33-38`` (returned outside the reference tree; inside it,
    ``track`` returns the reference's own class)."""

    states: Sequence[np.ndarray] = field(default_factory=list)

# MapConfig.map_resolution default (src/config.py:22): the px/m scale step() assumes before any
# track() call has fixed the parameters.
DEFAULT_MAP_RESOLUTION = 0.8


def _viz_hooks():
    """The reference's per-step plotting, when this module runs inside the reference tree."""
    try:  # pragma: no cover - only inside the reference tree
        from src.viz.record import FrameRecorder  # type: ignore
        from src.viz.vehicle_draw import VehicleParams  # type: ignore
        from src.viz.visualization import plot_prediction  # type: ignore

        return plot_prediction, FrameRecorder, VehicleParams
    except Exception:
        return None


def window_at(ref_global: np.ndarray, path_idx: int, horizon: int) -> np.ndarray:
    """Reference window with tail padding (``control_stage.py:101-105``)."""
    end = min(path_idx + horizon + 1, len(ref_global))
    ref_window = ref_global[path_idx:end]
    if len(ref_window) < horizon + 1:
        tail = np.repeat(ref_window[-1:], horizon + 1 - len(ref_window), axis=0)
        ref_window = np.vstack((ref_window, tail))
    return ref_window


@dataclass
class TrajectoryTracker:
    """Run MPC closed-loop tracking over the planned path."""

    mpc: Any  # MPCConfig (reference or mpcqp.config)
    viz: Any  # VizConfig
    # Optional solver settings (mpcqp_params names) of the nominal and the relaxed solve; the
    # reference constructs TrajectoryTracker(mpc, viz) and gets the library defaults.
    solver_settings: dict = field(default_factory=dict)
    relaxed_solver_settings: dict = field(default_factory=dict)
    # parameters of the last track() call; step() without params solves with them
    _params: Optional[MPCParameters] = field(default=None, init=False, repr=False, compare=False)

    def _solve_with_relaxation(
        self,
        state: np.ndarray,
        reference: np.ndarray,
        u_prev: np.ndarray,
        base_params: MPCParameters,
    ) -> Tuple[Optional[np.ndarray], Optional[np.ndarray], Optional[np.ndarray]]:
        """``control_stage.py:33-56``: nominal solve, then one retry with relaxed rates and speed."""
        controller = MPCController(base_params, **self.solver_settings)
        u0, Xp, Up = controller.solve(state, reference, u_prev=u_prev)
        if u0 is not None:
            return u0, Xp, Up
        LOG.warning("MPC infeasible; applying rate relaxation and speed reduction")
        relaxed_reference = np.array(reference, dtype=float, copy=True)
        relaxed_reference[:, 3] *= 0.6
        relaxed_params = replace(
            base_params,
            du_bounds=(
                (base_params.du_bounds[0][0] - 5.0, base_params.du_bounds[0][1] + 5.0),
                (base_params.du_bounds[1][0] - 0.05, base_params.du_bounds[1][1] + 0.05),
            ),
        )
        return MPCController(relaxed_params, **self.relaxed_solver_settings).solve(
            state, relaxed_reference, u_prev=u_prev)

    def step(
        self,
        state: np.ndarray,
        ref_window: np.ndarray,
        u_prev: np.ndarray,
        params: Optional[MPCParameters] = None,
        *,
        map_resolution: Optional[float] = None,
    ) -> Tuple[Optional[np.ndarray], Optional[np.ndarray], Optional[np.ndarray]]:
        """One closed-loop iteration (``control_stage.py:107-129``): solve, then the plant step.

        ``step(state, ref_window, u_prev)`` is the contract of SURVEY.md §8b.  The parameters are,
        in order: ``params`` when given; ``self.mpc.to_parameters(map_resolution)`` when a
        resolution is given; those of the last ``track()`` call; else
        ``self.mpc.to_parameters(0.8)`` (the reference's ``MapConfig.map_resolution`` default).

        Returns ``(next_state, u0, Xp)``, or ``(None, None, None)`` when the QP stays
        unsolved after relaxation (the caller aborts, as ``:108-110`` does).
        """
        if params is None:
            if map_resolution is not None:
                params = self.mpc.to_parameters(map_resolution)
            elif self._params is not None:
                params = self._params
            else:
                LOG.warning("step() before any track() and without params or map_resolution: assuming "
                            "map_resolution=%s (MapConfig's default) for the px/m scaling", DEFAULT_MAP_RESOLUTION)
                params = self._params = self.mpc.to_parameters(DEFAULT_MAP_RESOLUTION)
        u0, Xp, _ = self._solve_with_relaxation(state, ref_window, u_prev, params)
        if u0 is None or Xp is None:
            return None, None, None
        next_state = f_discrete(np.asarray(state, dtype=float), u0, params.dt, params.wheelbase_px)
        return next_state, u0, Xp

    def track(
        self,
        planning,
        maps,
        *,
        map_resolution: float,
        visualize: bool = True,
        occupancy: Optional[np.ndarray] = None,
        axis=None,
    ) -> TrackingResult:
        """``control_stage.py:58-157``."""
        plan = planning.plan
        if not plan.success:
            raise RuntimeError("Planning stage did not succeed; cannot start control stage")
        if not plan.path:
            raise RuntimeError("Planner returned an empty path")

        base_params = self._params = self.mpc.to_parameters(map_resolution)
        horizon = base_params.horizon
        wheelbase_px = base_params.wheelbase_px

        path = plan.path
        if len(path) > 1:
            yaw0 = float(np.arctan2(path[1][1] - path[0][1], path[1][0] - path[0][0]))
        else:
            yaw0 = 0.0
        state = np.array([maps.start[0], maps.start[1], yaw0, 5.0], dtype=float)
        u_prev = np.zeros(2)

        ref_global = build_reference(path, self.mpc.v_px_s, horizon, self.mpc.dt)
        LOG.info(
            "Starting MPC tracking (sim_steps=%d, horizon=%d, reference_points=%d)",
            self.mpc.sim_steps,
            horizon,
            len(ref_global),
        )
        hooks = _viz_hooks() if (visualize and occupancy is not None) else None
        recorder = None
        vehicle_params = None
        if hooks is not None:
            plot_prediction, FrameRecorder, VehicleParams = hooks
            vehicle_params = VehicleParams.from_wheelbase(wheelbase_px)
            if getattr(self.viz, "record_frames", False):
                recorder = FrameRecorder(self.viz.record_dir)

        states: list = []
        path_idx = 0
        goal_reached = False
        progress_interval = max(1, self.mpc.sim_steps // 10)
        for step in range(self.mpc.sim_steps):
            ref_window = window_at(ref_global, path_idx, horizon)
            next_state, u0, Xp = self.step(state, ref_window, u_prev, base_params)
            if next_state is None:
                LOG.error("MPC remained infeasible at step %d; aborting tracking", step)
                break
            if hooks is not None:
                hooks[0](occupancy, path, Xp, state, step, self.viz.prediction_pause, ax=axis,
                         vehicle_params=vehicle_params, control=u0)
                if recorder and axis is not None:
                    recorder.capture(axis.figure)
            state = next_state
            states.append(state.copy())
            u_prev = u0.copy()

            if (step + 1) % progress_interval == 0 or step == 0:
                LOG.info(
                    "Tracking progress: step=%d/%d position=(%.1f, %.1f) speed=%.2f",
                    step + 1,
                    self.mpc.sim_steps,
                    state[0],
                    state[1],
                    state[3],
                )
            if path_idx < len(ref_global) - 2:
                dx = state[0] - ref_global[path_idx][0]
                dy = state[1] - ref_global[path_idx][1]
                if dx * dx + dy * dy > 25.0:
                    path_idx += 1
            if np.hypot(state[0] - maps.goal[0], state[1] - maps.goal[1]) < 8.0:
                LOG.info("Reached goal region at step %d", step)
                goal_reached = True
                break

        LOG.info("MPC tracking finished after %d steps (goal_reached=%s)", len(states), goal_reached)
        return (_reference_tracking_result() or TrackingResult)(states=states)


__all__ = ["TrajectoryTracker", "TrackingResult", "window_at"]
