"""BASELINE config 5: a swarm of vehicles on one inflated grid, planned and tracked on the GPU.

``Swarm.run`` chains the batched stages for V vehicles:
  1. plan    -- ``BatchedRRTStarPlanner.plan_batch`` (one RRT* tree per vehicle, GPU), then the
               reference's prune + Catmull-Rom post-processing (host);
  2. refs    -- ``build_reference_batch`` (GPU) straight into the fleet's buffers;
  3. track   -- ``FleetTracker`` closed loop (GPU), ``check_every`` steps per host check;
  4. replan  -- the trigger the reference lists as roadmap (``README.md:146-148``): after each
               check, vehicles that aborted (QP unsolved after relaxation) or left their
               reference (distance to ``ref[path_idx]`` above ``replan_distance``) are re-planned
               together from where they stand, their references rebuilt and their loop state
               reset (path_idx 0, phase running), at most ``max_replans`` times each.
Every vehicle between replans follows the reference's single-vehicle loop exactly.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from .. import _lib
from ..control.ref_builder import build_reference_batch
from ..planning.rrt_star import BatchedRRTStarPlanner, PlannerParameters
from .fleet import FleetTracker


@dataclass
class SwarmResult:
    states: List[np.ndarray]  # per vehicle: states after each step, across replans
    phase: np.ndarray  # final MPCQP_FLEET_* phase
    steps: np.ndarray  # closed-loop steps per vehicle
    replans: np.ndarray  # replans per vehicle
    planned: np.ndarray  # initial plan succeeded
    timings: Dict[str, float] = field(default_factory=dict)


class Swarm:
    def __init__(self, occupancy: np.ndarray, mpc, planner: PlannerParameters, *, map_resolution: float,
                 max_vehicles: int, max_ref_len: int = 512, device=None, replan_distance: float = 15.0,
                 max_replans: int = 2) -> None:
        self.occupancy = np.ascontiguousarray(occupancy, dtype=np.uint8)
        self.mpc = mpc
        self.planner = BatchedRRTStarPlanner(self.occupancy, planner, device=device)
        self.fleet = FleetTracker(mpc, map_resolution=map_resolution, max_vehicles=max_vehicles,
                                  max_ref_len=max_ref_len, device=self.planner.device)
        self.device = self.planner.device
        self.replan_distance = float(replan_distance)
        self.max_replans = int(max_replans)

    def _plan(self, starts, goals, seeds):
        """Final paths of every problem (growth, extraction and pruning on the device);
        returns (success mask, paths with the start alone where no plan was found)."""
        found = self.planner.paths_batch(starts, goals, seeds)
        ok = np.array([p is not None for p in found], dtype=bool)
        paths = [p if p is not None else [tuple(s)] for p, s in zip(found, starts)]
        return ok, paths

    def run(self, starts: np.ndarray, goals: np.ndarray, seeds=None, *, sim_steps: Optional[int] = None,
            check_every: int = 10) -> SwarmResult:
        torch = self.fleet._torch
        starts = np.asarray(starts, dtype=float).reshape(-1, 2)
        goals = np.asarray(goals, dtype=float).reshape(-1, 2)
        V = len(starts)
        seeds = np.arange(V) if seeds is None else np.asarray(seeds)
        total = int(self.mpc.sim_steps if sim_steps is None else sim_steps)
        t = {}
        t0 = time.perf_counter()
        planned, paths = self._plan(starts, goals, seeds)
        t["plan_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        self.fleet.reset_from_plans(paths, starts, goals, max_steps=total, device_reference=True)
        b = self.fleet.buffers()
        if (~planned).any():  # no plan: the vehicle never starts (the reference raises, :69-72)
            b["phase"][torch.from_numpy(np.flatnonzero(~planned)).to(self.device)] = _lib.FLEET_ABORTED
        torch.cuda.synchronize(self.device)
        t["refs_s"] = time.perf_counter() - t0
        replans = np.zeros(V, dtype=np.int64)
        t_track = t_replan = 0.0
        done = 0
        while done < total:
            t0 = time.perf_counter()
            k = min(check_every, total - done)
            self.fleet.step(k)
            done += k
            phase = b["phase"][:V].cpu().numpy()
            t_track += time.perf_counter() - t0
            if not (phase == _lib.FLEET_RUNNING).any() and not self._any_replannable(phase, replans, planned):
                break
            t0 = time.perf_counter()
            need = self._replan_candidates(phase, replans, planned)
            if len(need):
                self._replan(need, goals, seeds, replans)
            t_replan += time.perf_counter() - t0
        t["track_s"] = t_track
        t["replan_s"] = t_replan
        r = self.fleet.result()
        return SwarmResult(states=r.states, phase=r.phase, steps=r.steps, replans=replans, planned=planned, timings=t)

    def _any_replannable(self, phase, replans, planned) -> bool:
        return bool(((phase == _lib.FLEET_ABORTED) & planned & (replans < self.max_replans)).any())

    def _replan_candidates(self, phase, replans, planned) -> np.ndarray:
        b = self.fleet.buffers()
        V = len(phase)
        state = b["state"][:V].cpu().numpy()
        pidx = b["path_idx"][:V].long()
        ref_pt = b["ref_global"][:V].gather(1, pidx.view(-1, 1, 1).expand(-1, 1, 4)).squeeze(1).cpu().numpy()
        off = np.hypot(state[:, 0] - ref_pt[:, 0], state[:, 1] - ref_pt[:, 1]) > self.replan_distance
        trig = ((phase == _lib.FLEET_ABORTED) | ((phase == _lib.FLEET_RUNNING) & off))
        return np.flatnonzero(trig & planned & (replans < self.max_replans))

    def _replan(self, idx: np.ndarray, goals, seeds, replans) -> None:
        torch = self.fleet._torch
        b = self.fleet.buffers()
        state = b["state"][:len(replans)].cpu().numpy()
        starts = state[idx, :2]
        ok, paths = self._plan(starts, goals[idx], seeds[idx] + 7919 * (replans[idx] + 1))
        replans[idx] += 1
        if not ok.any():
            return
        sel = idx[ok]
        ref, ref_len = build_reference_batch([paths[i] for i in np.flatnonzero(ok)], self.mpc.v_px_s,
                                             self.fleet.horizon, self.mpc.dt, device=self.device,
                                             ref_stride=self.fleet.max_ref_len)
        if (ref_len < 1).any():
            raise ValueError("replanned reference exceeds max_ref_len")
        si = torch.from_numpy(sel).to(self.device)
        b["ref_global"][si] = ref
        b["ref_len"][si] = ref_len
        b["path_idx"][si] = 0
        b["phase"][si] = _lib.FLEET_RUNNING  # pose, speed and u_prev carry over


__all__ = ["Swarm", "SwarmResult"]
