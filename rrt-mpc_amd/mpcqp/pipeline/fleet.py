"""Closed-loop tracking for a fleet of vehicles, resident on the GPU.

``FleetTracker`` runs the loop body of the reference's ``TrajectoryTracker.track``
(``src/pipeline/control_stage.py:100-150``) for V vehicles at once through
``mpcqp_fleet_run`` (``csrc/mpcqp_fleet.hip``): per step, a masked batched MPC solve
with the reference's relaxation retry (``:33-56``), the plant ``f_discrete`` (``:127``),
the ``path_idx`` advance (``:141-145``) and the goal test (``:147-150``), all on the
device.  The host only checks every ``check_every`` steps whether any vehicle still runs.
``fused=True`` runs the whole loop in ONE launch instead (``mpcqp_fleet_loop``,
``k_fleet_loop`` in ``csrc/mpcqp_solve.h``): each vehicle's wave loops over its own steps, with
no kernel boundary per step, and leaves the loop at its goal -- the same operations, so the
traces are bit-identical to the stepped path.

Each vehicle follows exactly the reference's single-vehicle semantics, so vehicle ``v``
reproduces ``TrajectoryTracker.track`` on its own plan (tests/test_gpu_fleet.py).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, replace
from typing import List, Optional, Sequence

import numpy as np

from .. import _lib
from ..control.ref_builder import PackedPaths, build_reference, build_reference_batch
from .control_stage import TrackingResult

PHASE_NAMES = {
    _lib.FLEET_RUNNING: "running",
    _lib.FLEET_GOAL: "goal_reached",
    _lib.FLEET_ABORTED: "aborted",
    _lib.FLEET_OUT_OF_STEPS: "out_of_steps",
}


def relaxed_parameters(base_params):
    """The retry parameters of ``control_stage.py:50-56`` (du_bounds widened by (5, 0.05))."""
    return replace(
        base_params,
        du_bounds=(
            (base_params.du_bounds[0][0] - 5.0, base_params.du_bounds[0][1] + 5.0),
            (base_params.du_bounds[1][0] - 0.05, base_params.du_bounds[1][1] + 0.05),
        ),
    )


def initial_state(path: Sequence, start) -> np.ndarray:
    """``control_stage.py:74-79``: start position, heading of the first path segment, 5 px/s."""
    if len(path) > 1:
        yaw0 = float(np.arctan2(path[1][1] - path[0][1], path[1][0] - path[0][0]))
    else:
        yaw0 = 0.0
    return np.array([start[0], start[1], yaw0, 5.0], dtype=float)


def initial_states(paths: Sequence, starts, packed: Optional[PackedPaths] = None) -> np.ndarray:
    """``initial_state`` of every vehicle, (V, 4): the first segments' headings by one elementwise
    ``np.arctan2`` over all vehicles (the same float64 differences and ufunc as per path), read
    from the packed polylines (``packed``: the pass ``build_reference_batch`` shares)."""
    pk = packed if packed is not None else PackedPaths(paths)
    V = pk.V
    if V and pk.counts.min() == 0:
        raise RuntimeError("Planner returned an empty path")
    many = pk.counts > 1
    i0 = pk.off[:-1].astype(np.int64)
    i1 = np.where(many, i0 + 1, i0)
    p0, p1 = pk.pts[np.minimum(i0, len(pk.pts) - 1)], pk.pts[np.minimum(i1, len(pk.pts) - 1)]
    out = np.empty((V, 4))
    out[:, :2] = np.asarray(starts, dtype=float).reshape(V, 2)
    out[:, 2] = np.where(many, np.arctan2(p1[:, 1] - p0[:, 1], p1[:, 0] - p0[:, 0]), 0.0)
    out[:, 3] = 5.0
    return out


@dataclass
class FleetResult:
    """Per-vehicle outcome of a fleet run (host copies)."""

    states: List[np.ndarray]  # vehicle v: (steps[v], 4) states after each step (TrackingResult.states)
    inputs: List[np.ndarray]  # vehicle v: (steps[v], 2) applied u0
    phase: np.ndarray  # (V,) int32: 0 running, 1 goal reached, 2 aborted, 3 out of steps
    steps: np.ndarray  # (V,) int32
    path_idx: np.ndarray  # (V,) int32

    def tracking_results(self) -> List[TrackingResult]:
        return [TrackingResult(states=[s.copy() for s in st]) for st in self.states]


def closed_loop_settings(horizon: int) -> dict:
    """Polish schedule of the device closed loops (FleetTracker, Swarm).  A fleet's run is the sum
    of each vehicle's step costs, so an attempt at every termination check pays, where the library
    default (`polish_from` 75) is tuned for a one-shot batch's slowest QP.  Measured with the fused
    loop at N = 15 and the default single Ruiz pass (DESIGN.md §9,
    profiles/r03_s14_schedule_fleets.json): `polish_from` 25 against 75 gives -9 / -7 / -10 % at
    100 / 1024 / 4096 vehicles and -5 % on the config-5 swarm.  Past the one-wave kernel the default
    stays (unmeasured)."""
    return {"polish_from": 25} if horizon <= 32 else {}


class FleetTracker:
    """V vehicles in closed loop on one GPU; every loop step runs on the device.

    ``mpc`` is an ``MPCConfig`` (reference or ``mpcqp.config``); the solver parameters
    are ``mpc.to_parameters(map_resolution)`` as in ``control_stage.py:73``.
    """

    def __init__(self, mpc, *, map_resolution: float, max_vehicles: int, max_ref_len: int,
                 device=None, use_graph: bool = True, fused: bool = False,
                 relaxed_settings: Optional[dict] = None, **settings) -> None:
        import torch

        from ..control.mpc_controller import BatchedMPCController

        self._torch = torch
        self.mpc = mpc
        self.params = mpc.to_parameters(map_resolution)
        self.horizon = int(self.params.horizon)
        self.max_vehicles = int(max_vehicles)
        self.max_ref_len = int(max_ref_len)
        self.use_graph = bool(use_graph)
        self.fused = bool(fused)
        # a closed loop pays every vehicle's step costs, not a batch's slowest QP: the polish schedule
        # defaults to closed_loop_settings (the caller's settings win)
        loop = closed_loop_settings(self.horizon)
        settings = {**loop, **settings}
        self._nominal = BatchedMPCController(self.params, self.max_vehicles, device=device, **settings)
        # the retry's solver settings default to the nominal ones (control_stage.py:50-56 changes
        # only du_bounds and the reference speed)
        rs = settings if relaxed_settings is None else {**loop, **relaxed_settings}
        self._relaxed = BatchedMPCController(relaxed_parameters(self.params), self.max_vehicles,
                                             device=self._nominal.device, **rs)
        self.device = self._nominal.device
        self._L = _lib.lib()
        self._bufs = None
        self._fleet = None
        self.vehicles = 0

    # ------------------------------------------------------------------
    def reset(self, ref_globals: Sequence[np.ndarray], states0: np.ndarray, goals: np.ndarray,
              max_steps: Optional[int] = None) -> None:
        """Load V references (each ``(M_v, 4)``, ``build_reference`` output), start states and goals."""
        V = len(ref_globals)
        if V > self.max_vehicles:
            raise ValueError(f"{V} vehicles exceed max_vehicles {self.max_vehicles}")
        states0 = np.asarray(states0, dtype=float).reshape(V, 4)
        goals = np.asarray(goals, dtype=float).reshape(V, 2)
        max_steps = int(self.mpc.sim_steps if max_steps is None else max_steps)
        if max_steps < 1:
            raise ValueError("max_steps must be >= 1")
        lens = np.array([len(r) for r in ref_globals], dtype=np.int32)
        if V and (lens.min() < 1 or lens.max() > self.max_ref_len):
            raise ValueError(f"reference lengths must be in [1, {self.max_ref_len}]")
        M = self.max_ref_len
        ref = np.zeros((max(V, 1), M, 4))
        for v, r in enumerate(ref_globals):
            r = np.asarray(r, dtype=float)
            if r.ndim != 2 or r.shape[1] != 4:
                raise ValueError("each reference must have shape (M, 4)")
            ref[v, : len(r)] = r
        self._load(V, ref, lens, states0, goals, max_steps)

    def _load(self, V: int, ref: Optional[np.ndarray], lens: np.ndarray, states0: np.ndarray, goals: np.ndarray,
              max_steps: Optional[int]) -> None:
        """The fleet's device buffers for V vehicles; ``ref`` None: the references are copied in on the
        device afterwards (reset_device), so no host copy of them is built or uploaded."""
        torch = self._torch
        states0 = np.asarray(states0, dtype=float).reshape(V, 4)
        goals = np.asarray(goals, dtype=float).reshape(V, 2)
        max_steps = int(self.mpc.sim_steps if max_steps is None else max_steps)
        if max_steps < 1:
            raise ValueError("max_steps must be >= 1")
        M = self.max_ref_len
        N = self.horizon
        dev = dict(device=self.device)
        f64 = torch.float64
        i32 = torch.int32
        b = {
            "ref_global": (torch.from_numpy(ref).to(**dev) if ref is not None
                           else torch.zeros((max(V, 1), M, 4), dtype=f64, **dev)),
            "ref_len": torch.from_numpy(np.maximum(lens, 1) if V else np.ones(1, np.int32)).to(**dev),
            "goal": torch.from_numpy(goals if V else np.zeros((1, 2))).to(**dev),
            "state": torch.from_numpy(states0 if V else np.zeros((1, 4))).to(**dev),
            "u_prev": torch.zeros((max(V, 1), 2), dtype=f64, **dev),
            "path_idx": torch.zeros((max(V, 1),), dtype=i32, **dev),
            "phase": torch.zeros((max(V, 1),), dtype=i32, **dev),
            "steps": torch.zeros((max(V, 1),), dtype=i32, **dev),
            "mask": torch.zeros((2, max(V, 1)), dtype=torch.uint8, **dev),
            "status": torch.zeros((2, max(V, 1)), dtype=i32, **dev),
            "u0": torch.zeros((2, max(V, 1), 2), dtype=f64, **dev),
            "X": torch.zeros((max(V, 1), 4, N + 1), dtype=f64, **dev),
            "trace": torch.zeros((max(V, 1), max_steps, 4), dtype=f64, **dev),
            "u_trace": torch.zeros((max(V, 1), max_steps, 2), dtype=f64, **dev),
        }
        f = _lib.MpcqpFleet()
        f.vehicles = V
        f.ref_stride = M
        f.max_steps = max_steps
        for name, t in b.items():
            setattr(f, name, t.data_ptr())
        self._bufs = b
        self._fleet = f
        self.vehicles = V
        self.max_steps = max_steps

    def reset_from_plans(self, paths: Sequence, starts: np.ndarray, goals: np.ndarray,
                         max_steps: Optional[int] = None, *, device_reference: bool = False):
        """``control_stage.py:69-87`` per vehicle: references from the planned paths, start states.

        ``device_reference=True`` builds the references with the batched GPU ``build_reference``
        (``mpcqp_build_reference``) straight into the fleet's buffers; otherwise on the host.
        Returns the host references (or ``(ref, ref_len)`` device tensors)."""
        packed = PackedPaths(paths)
        states0 = initial_states(paths, starts, packed)
        if device_reference:
            ref, ref_len = build_reference_batch(paths, self.mpc.v_px_s, self.horizon, self.mpc.dt,
                                                 device=self.device, ref_stride=self.max_ref_len, packed=packed)
            self.reset_device(ref, ref_len, states0, goals, max_steps)
            return ref, ref_len
        refs = [build_reference(path, self.mpc.v_px_s, self.horizon, self.mpc.dt) for path in paths]
        self.reset(refs, states0, goals, max_steps)
        return refs

    def reset_device(self, ref, ref_len, states0: np.ndarray, goals: np.ndarray,
                     max_steps: Optional[int] = None) -> None:
        """Load references already on the device: ``ref`` (V, max_ref_len, 4) float64 and
        ``ref_len`` (V,) int32 as produced by ``build_reference_batch``."""
        torch = self._torch
        V = int(ref.shape[0])
        if V > self.max_vehicles:
            raise ValueError(f"{V} vehicles exceed max_vehicles {self.max_vehicles}")
        if int(ref.shape[1]) != self.max_ref_len:
            raise ValueError(f"ref rows {int(ref.shape[1])} != max_ref_len {self.max_ref_len}")
        lens = ref_len.cpu().numpy()
        if V and (lens.min() < 1 or lens.max() > self.max_ref_len):
            raise ValueError(f"reference lengths must be in [1, {self.max_ref_len}] (build_reference_batch "
                             f"reports overflow as negative lengths)")
        self._load(V, None, lens.astype(np.int32), states0, goals, max_steps)
        self._bufs["ref_global"][:V].copy_(ref)
        self._bufs["ref_len"][:V].copy_(ref_len.to(torch.int32))

    # ------------------------------------------------------------------
    def step(self, steps: int = 1, stream=None) -> None:
        """Enqueue ``steps`` closed-loop steps (asynchronous on the current torch stream)."""
        if self._fleet is None:
            raise RuntimeError("reset() the fleet first")
        torch = self._torch
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        s = ctypes.c_void_p(stream.cuda_stream)
        if self.fused:
            _lib.check(self._L.mpcqp_fleet_loop(self._nominal._ws, self._relaxed._ws, ctypes.byref(self._fleet),
                                                int(steps), s), "mpcqp_fleet_loop")
            return
        _lib.check(self._L.mpcqp_fleet_run(self._nominal._ws, self._relaxed._ws, ctypes.byref(self._fleet),
                                           int(steps), int(self.use_graph), s), "mpcqp_fleet_run")

    def running(self) -> int:
        return int((self._bufs["phase"][: self.vehicles] == _lib.FLEET_RUNNING).sum().item())

    def run(self, sim_steps: Optional[int] = None, check_every: int = 16) -> FleetResult:
        """Step until every vehicle has left the RUNNING phase (or ``sim_steps`` steps)."""
        total = self.max_steps if sim_steps is None else min(int(sim_steps), self.max_steps)
        if self.fused:  # one launch: every vehicle leaves the loop by itself
            if self.vehicles:
                self.step(total)
            return self.result()
        done = 0
        while done < total and self.vehicles:
            k = min(check_every, total - done)
            self.step(k)
            done += k
            if self.running() == 0:
                break
        return self.result()

    def result(self) -> FleetResult:
        b = self._bufs
        V = self.vehicles
        self._torch.cuda.synchronize(self.device)
        steps = b["steps"][:V].cpu().numpy().copy()
        trace = b["trace"][:V].cpu().numpy()
        utr = b["u_trace"][:V].cpu().numpy()
        return FleetResult(
            states=[trace[v, : steps[v]].copy() for v in range(V)],
            inputs=[utr[v, : steps[v]].copy() for v in range(V)],
            phase=b["phase"][:V].cpu().numpy().copy(),
            steps=steps,
            path_idx=b["path_idx"][:V].cpu().numpy().copy(),
        )

    def buffers(self) -> dict:
        """The device tensors behind the fleet state (views; for inspection and tests)."""
        return self._bufs

    def close(self) -> None:
        self._nominal.close()
        self._relaxed.close()


__all__ = ["FleetTracker", "FleetResult", "relaxed_parameters", "initial_state", "initial_states", "closed_loop_settings",
           "PHASE_NAMES"]
