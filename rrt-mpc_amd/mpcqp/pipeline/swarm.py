"""BASELINE config 5: a swarm of vehicles on one inflated grid, planned, tracked and re-planned
on the GPU with a per-step replan trigger.

``Swarm.run`` chains the batched stages for V vehicles:
  1. plan    -- ``BatchedRRTStarPlanner.paths_batch``: one RRT* tree per vehicle, path extraction,
               shortcut pruning and Catmull-Rom smoothing on the device (``rrt_star.py:201-289``);
  2. refs    -- ``build_reference_batch`` (GPU) straight into the fleet's buffers;
  3. track + replan -- ``mpcqp_swarm_run`` (``csrc/mpcqp_swarm.hip``), every step on the device:
               the fleet closed-loop step (``control_stage.py:100-150``), then the trigger the
               reference lists as roadmap (``README.md:146-148``) -- a vehicle farther than
               ``replan_distance`` from ``ref[path_idx]`` after its step, or one whose QP stayed
               unsolved after relaxation (aborted) -- and, in the same step, its replanning from
               where it stands (RRT* with its next seed ``seed + 7919 (r + 1)``, pruning,
               smoothing, build_reference); pose, speed and u_prev carry over, path_idx restarts at
               0.  At most ``max_replans`` per vehicle.  The whole step is one hipGraph replay; the
               host only polls every ``check_every`` steps whether any vehicle still runs.  With
               ``fused=True``: ``mpcqp_swarm_loop``, the fused fleet loop with the trigger inside
               (max_replans + 1 launches, the replanning kernels between them).
Every vehicle between replans follows the reference's single-vehicle loop exactly.
"""
from __future__ import annotations

import ctypes
import time
from dataclasses import dataclass, field, fields
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import _lib
from ..planning.rrt_star import BatchedRRTStarPlanner, PlannerParameters, pcg64_states
from .fleet import FleetTracker

REPLAN_SEED_STRIDE = 7919  # replan r of vehicle v draws from default_rng(seed_v + 7919 (r + 1))


def replan_seed(seed: int, r: int) -> int:
    return int(seed) + REPLAN_SEED_STRIDE * (int(r) + 1)


@dataclass
class SwarmResult:
    states: List[np.ndarray]  # per vehicle: states after each step, across replans
    phase: np.ndarray  # final MPCQP_FLEET_* phase
    steps: np.ndarray  # closed-loop steps per vehicle
    replans: np.ndarray  # replan attempts per vehicle
    planned: np.ndarray  # initial plan succeeded
    paths: List[Optional[list]] = field(default_factory=list)  # initial plan per vehicle (None: no plan)
    replan_steps: Optional[np.ndarray] = None  # (V, max_replans): steps[v] at replan r, -steps-1 failed, 0 unused
    last_replan_start: Optional[np.ndarray] = None  # (V, 2): where the last replan started
    last_replan_path: List[Optional[np.ndarray]] = field(default_factory=list)  # its final path (None: failed/none)
    # the last replan failed because its smoothed path exceeded path_cap (not an RRT* failure)
    replan_over_capacity: Optional[np.ndarray] = None
    inputs: List[np.ndarray] = field(default_factory=list)  # per vehicle: applied u0 per step
    timings: Dict[str, float] = field(default_factory=dict)


class Swarm:
    def __init__(self, occupancy: np.ndarray, mpc, planner: PlannerParameters, *, map_resolution: float,
                 max_vehicles: int, max_ref_len: int = 512, device=None, replan_distance: float = 15.0,
                 max_replans: int = 2, path_cap: int = 6144, use_graph: bool = True, fused: bool = False,
                 **settings) -> None:
        # path_cap: smoothed points a replan may produce.  The default is the most that the device
        # reference builder stages (kRefCap, csrc/mpcqp_swarm.hip), so a replanned path is never cut
        # shorter than a reference could be built from; capacity failures are reported apart from
        # RRT* failures (SwarmResult.replan_over_capacity).
        self.occupancy = np.ascontiguousarray(occupancy, dtype=np.uint8)
        self.mpc = mpc
        self.planner = BatchedRRTStarPlanner(self.occupancy, planner, device=device)
        # settings: solver settings of the vehicles' QPs (mpcqp_params names), as FleetTracker's
        self.fleet = FleetTracker(mpc, map_resolution=map_resolution, max_vehicles=max_vehicles,
                                  max_ref_len=max_ref_len, device=self.planner.device, **settings)
        self.device = self.planner.device
        self.replan_distance = float(replan_distance)
        self.max_replans = int(max_replans)
        self.path_cap = int(path_cap)
        self.use_graph = bool(use_graph)
        # fused: the run as max_replans + 1 launches of the fused fleet loop with the trigger inside
        # (mpcqp_swarm_loop) instead of one graph-replayed launch sequence per step
        self.fused = bool(fused)
        self._L = _lib.lib()

    def _plan(self, starts, goals, seeds):
        """Final paths of every problem (growth, extraction, pruning and smoothing on the device);
        returns (success mask, paths with the start alone where no plan was found)."""
        found = self.planner.paths_batch(starts, goals, seeds, smoothing="device")
        ok = np.array([p is not None for p in found], dtype=bool)
        paths = [p if p is not None else [tuple(s)] for p, s in zip(found, starts)]
        return ok, paths, found

    def _swarm_struct(self, V: int, seeds, planned) -> tuple:
        torch = self.fleet._torch
        dev = dict(device=self.device)
        R = max(self.max_replans, 1)
        M = int(self.planner.params.max_iterations) + 2
        S = self.fleet.max_ref_len
        table = np.zeros((max(V, 1), R, 4), dtype=np.uint64)
        if self.max_replans:
            for v in range(V):
                table[v] = pcg64_states([replan_seed(seeds[v], r) for r in range(self.max_replans)])
        f64, i32 = torch.float64, torch.int32
        n = max(V, 1)
        b = {
            "rng_table": torch.from_numpy(table).to(**dev),
            # vehicles without an initial plan never replan (the reference raises, control_stage.py:69-72)
            "replans": torch.from_numpy(np.where(planned, 0, self.max_replans).astype(np.int32)
                                        if V else np.zeros(1, np.int32)).to(**dev),
            "replan_step": torch.zeros((n, R), dtype=i32, **dev),
            "start_goal": torch.zeros((n, 4), dtype=f64, **dev),
            "nodes": torch.zeros((n, M, 4), dtype=f64, **dev),
            "count": torch.zeros((n,), dtype=i32, **dev),
            "meta": torch.zeros((n, 2), dtype=i32, **dev),
            "raw": torch.zeros((n, M, 2), dtype=f64, **dev),
            "raw_len": torch.zeros((n,), dtype=i32, **dev),
            "pruned": torch.zeros((n, M, 2), dtype=f64, **dev),
            "pruned_len": torch.zeros((n,), dtype=i32, **dev),
            "smooth": torch.zeros((n, self.path_cap, 2), dtype=f64, **dev),
            "smooth_len": torch.zeros((n,), dtype=i32, **dev),
            "new_ref": torch.zeros((n, S, 4), dtype=f64, **dev),
            "new_len": torch.zeros((n,), dtype=i32, **dev),
        }
        occ = torch.from_numpy(self.occupancy).to(**dev)
        s = _lib.MpcqpSwarm()
        s.rrt = self.planner._c
        s.occupancy = occ.data_ptr()
        pp = self.planner.params
        s.prune = int(bool(pp.prune_path))
        s.spline_samples = int(pp.spline_samples)
        s.spline_alpha = float(pp.spline_alpha)
        s.dedupe_tol = float(pp.dedupe_tolerance)
        s.desired_speed = float(self.mpc.v_px_s)
        s.dt = float(self.mpc.dt)
        s.horizon = int(self.fleet.horizon)
        s.max_replans = self.max_replans
        s.replan_distance = self.replan_distance
        s.path_cap = self.path_cap
        for k, t in b.items():
            setattr(s, k, t.data_ptr())
        b["occupancy"] = occ
        return s, b

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
        planned, paths, found = self._plan(starts, goals, seeds)
        t["plan_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        self.fleet.reset_from_plans(paths, starts, goals, max_steps=total, device_reference=True)
        fb = self.fleet.buffers()
        if (~planned).any():  # no plan: the vehicle never starts (the reference raises, :69-72)
            fb["phase"][torch.from_numpy(np.flatnonzero(~planned)).to(self.device)] = _lib.FLEET_ABORTED
        sw, sb = self._swarm_struct(V, seeds, planned)
        torch.cuda.synchronize(self.device)
        t["refs_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        stream = torch.cuda.current_stream(self.device)
        done = 0
        if self.fused and V:
            _lib.check(self._L.mpcqp_swarm_loop(self.fleet._nominal._ws, self.fleet._relaxed._ws,
                                                ctypes.byref(self.fleet._fleet), ctypes.byref(sw),
                                                ctypes.c_void_p(stream.cuda_stream)), "mpcqp_swarm_loop")
            done = total
        while done < total and V:
            k = min(check_every, total - done)
            _lib.check(self._L.mpcqp_swarm_run(self.fleet._nominal._ws, self.fleet._relaxed._ws,
                                               ctypes.byref(self.fleet._fleet), ctypes.byref(sw), int(k),
                                               int(self.use_graph), ctypes.c_void_p(stream.cuda_stream)),
                       "mpcqp_swarm_run")
            done += k
            if not bool((fb["phase"][:V] == _lib.FLEET_RUNNING).any().item()):
                break
        torch.cuda.synchronize(self.device)
        t["track_replan_s"] = time.perf_counter() - t0
        r = self.fleet.result()
        replans = sb["replans"][:V].cpu().numpy().astype(np.int64)
        replans = np.where(planned, replans, 0)
        rsteps = sb["replan_step"][:V, : max(self.max_replans, 1)].cpu().numpy()
        sg = sb["start_goal"][:V].cpu().numpy()
        sl = sb["smooth_len"][:V].cpu().numpy()
        smooth = sb["smooth"][:V].cpu().numpy()
        last_paths = []
        over_cap = np.zeros(V, dtype=bool)
        for v in range(V):
            over_cap[v] = bool(replans[v] and rsteps[v, replans[v] - 1] < 0 and sl[v] == -1)
            if replans[v] and rsteps[v, replans[v] - 1] >= 0 and sl[v] >= 1:
                last_paths.append(smooth[v, : sl[v]].copy())
            else:
                last_paths.append(None)
        return SwarmResult(states=r.states, phase=r.phase, steps=r.steps, replans=replans, planned=planned,
                           paths=found, replan_steps=rsteps, last_replan_start=sg[:, :2].copy(),
                           last_replan_path=last_paths, inputs=r.inputs, timings=t,
                           replan_over_capacity=over_cap)


# ------------------------------------------------------------------ multi-GPU: vehicles sharded over ranks
# The vehicles of the swarm are independent (the reference tracks each one alone,
# control_stage.py:100-150; nothing couples two vehicles), so config 5 on G GPUs gives each rank a
# contiguous block of vehicles -- with the vehicles' own seeds, so every vehicle does exactly what it
# does in a one-GPU run -- and the only collective is the gather of the per-vehicle results at the end
# (no data-path exchange: weak scaling in the vehicles, strong scaling of a fixed swarm).

def shard_vehicles(V: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of rank's contiguous block; block sizes differ by at most one (bench.shard_bounds)."""
    base, extra = divmod(int(V), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


_PER_VEHICLE_ARRAYS = ("phase", "steps", "replans", "planned", "replan_steps", "last_replan_start",
                       "replan_over_capacity")
_PER_VEHICLE_LISTS = ("states", "paths", "last_replan_path", "inputs")


def merge_swarm_results(parts: Sequence[SwarmResult]) -> SwarmResult:
    """Rank-ordered shard results -> the swarm's result in vehicle order; timings: max over ranks
    (the ranks run concurrently, the slowest one sets the swarm's wall time)."""
    parts = [p for p in parts if p is not None]
    kw = {}
    for f in fields(SwarmResult):
        vals = [getattr(p, f.name) for p in parts]
        if f.name in _PER_VEHICLE_ARRAYS:
            vals = [v for v in vals if v is not None and len(v)]
            kw[f.name] = np.concatenate(vals) if vals else None
        elif f.name in _PER_VEHICLE_LISTS:
            kw[f.name] = [x for v in vals for x in v]
        elif f.name == "timings":
            keys = sorted({k for v in vals for k in v})
            kw[f.name] = {k: max(v.get(k, 0.0) for v in vals) for k in keys}
    return SwarmResult(**kw)


def run_swarm_sharded(run: Callable[..., SwarmResult], starts, goals, seeds, *, rank: int, world: int,
                      all_gather_object: Callable[[list, object], None], **kwargs) -> SwarmResult:
    """Run rank's block of the swarm with ``run`` (``Swarm.run`` of this rank's device) and gather
    every rank's result: each rank returns the whole swarm's result, in vehicle order."""
    starts = np.asarray(starts, dtype=float).reshape(-1, 2)
    goals = np.asarray(goals, dtype=float).reshape(-1, 2)
    V = len(starts)
    seeds = np.arange(V) if seeds is None else np.asarray(seeds)
    lo, hi = shard_vehicles(V, world, rank)
    local = run(starts[lo:hi], goals[lo:hi], seeds=seeds[lo:hi], **kwargs) if hi > lo else None
    parts: list = [None] * world
    all_gather_object(parts, local)
    return merge_swarm_results(parts)


__all__ = ["Swarm", "SwarmResult", "replan_seed", "REPLAN_SEED_STRIDE", "shard_vehicles", "merge_swarm_results",
           "run_swarm_sharded"]
