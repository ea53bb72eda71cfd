"""RRT* planning with the tree grown on the GPU: drop-in for ``src/planning/rrt_star.py``.

``RRTStarPlanner(occupancy, params).plan(start, goal) -> PlanResult`` keeps the reference's
names, arguments and results (``rrt_star.py:192-357``, ``plan_result.py``).  The expensive part,
the tree growth loop (nearest / steer / segment checks / choose parent / rewire / goal,
``:213-243``), runs in ``mpcqp_rrt_plan`` (``csrc/mpcqp_rrt.hip``), one workgroup per planning
problem; ``BatchedRRTStarPlanner.plan_batch`` grows many trees at once (config 5: a fleet
replanning).  The random stream of each problem is drawn here with the reference's own numpy
calls (``_sample``, ``:320-325``) so every seed replays exactly; path extraction, shortcut
pruning and Catmull-Rom smoothing (``:250-283``) are the reference's cheap host
post-processing, restated below.
"""
from __future__ import annotations

import copy
import ctypes
import logging
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .. import _lib
from ..common.geometry import catmull_rom_spline

LOG = logging.getLogger(__name__)


@dataclass
class PlannerParameters:
    """``rrt_star.py:26-38``."""

    step: float
    goal_radius: float
    max_iterations: int
    rewire_radius: float
    goal_sample_rate: float
    random_seed: int
    prune_path: bool = True
    spline_samples: int = 20
    spline_alpha: float = 0.5
    dedupe_tolerance: float = 1e-9
    collision_step: float = 1.0


def default_planner_parameters(**overrides) -> PlannerParameters:
    """``PlannerConfig().to_parameters()`` (``src/config.py:35-62``)."""
    p = dict(step=3.0, goal_radius=10.0, max_iterations=2000, rewire_radius=20.0, goal_sample_rate=0.1,
             random_seed=13, prune_path=True, spline_samples=20, spline_alpha=0.5, dedupe_tolerance=1e-9,
             collision_step=0.75)
    p.update(overrides)
    return PlannerParameters(**p)


@dataclass
class RRTStarNode:
    """``plan_result.py:8-15``."""

    x: float
    y: float
    cost: float
    parent: Optional[int]


@dataclass
class PlanResult:
    """``plan_result.py:18-29``."""

    success: bool
    path: List[Tuple[float, float]]
    nodes: List[RRTStarNode]
    iterations: int
    goal_index: Optional[int]
    raw_path: Sequence[Tuple[float, float]] = field(default_factory=list)
    pruned_path: Optional[Sequence[Tuple[float, float]]] = None
    smoothed_path: Optional[Sequence[Tuple[float, float]]] = None


def draw_samples(seed, goal, shape, goal_sample_rate: float, max_iterations: int) -> np.ndarray:
    """The planner's sample of every iteration (``_sample``, ``rrt_star.py:296-301``): the same
    ``numpy.random.default_rng(seed)`` calls in the same order (one per iteration, whether or
    not the iteration then adds a node).  ``seed`` may also be a live ``numpy.random.Generator``,
    which is advanced by the draws."""
    rng = seed if isinstance(seed, np.random.Generator) else np.random.default_rng(seed)
    out = np.empty((max_iterations, 2))
    h, w = int(shape[0]), int(shape[1])
    gx, gy = float(goal[0]), float(goal[1])
    for k in range(max_iterations):
        if rng.random() < goal_sample_rate:
            out[k] = (gx, gy)
        else:
            y = rng.integers(0, h)
            x = rng.integers(0, w)
            out[k] = (float(x), float(y))
    return out


def pcg64_states(seeds) -> np.ndarray:
    """``numpy.random.default_rng(seed).bit_generator.state`` per seed as (V, 4) uint64
    {state lo, state hi, inc lo, inc hi}: the device draws _sample's stream from it."""
    m = (1 << 64) - 1
    out = np.empty((len(seeds), 4), dtype=np.uint64)
    for i, sd in enumerate(seeds):
        st = np.random.default_rng(int(sd)).bit_generator.state
        if st["bit_generator"] != "PCG64":
            raise RuntimeError("numpy's default generator is no longer PCG64")
        s, inc = st["state"]["state"], st["state"]["inc"]
        out[i] = (s & m, s >> 64, inc & m, inc >> 64)
    return out


def segment_is_free(occupancy: np.ndarray, start, end, collision_step: float) -> bool:
    """``_segment_is_free`` (``rrt_star.py:339-352``), used by the host shortcut pruning."""
    dx = end[0] - start[0]
    dy = end[1] - start[1]
    distance = math.hypot(dx, dy)
    step = max(collision_step, 1e-3)
    samples = max(1, int(math.ceil(distance / step)))
    xs = np.linspace(start[0], end[0], samples + 1)
    ys = np.linspace(start[1], end[1], samples + 1)
    h, w = occupancy.shape
    # vectorised: np.rint rounds half to even like Python's round(); same clip, same lookups
    xi = np.clip(np.rint(xs), 0, w - 1).astype(np.intp)
    yi = np.clip(np.rint(ys), 0, h - 1).astype(np.intp)
    return not bool((occupancy[yi, xi] == 0).any())


def _finish(occupancy, params: PlannerParameters, nodes: List[RRTStarNode], iterations: int,
            goal_index: Optional[int]) -> PlanResult:
    """``rrt_star.py:245-294``: extract, shortcut-prune and smooth the path."""
    success = goal_index is not None
    raw_path: List[Tuple[float, float]] = []
    pruned_path = None
    smoothed_path = None
    final_path: List[Tuple[float, float]] = []
    if success:
        idx = goal_index
        while idx is not None:
            raw_path.append((nodes[idx].x, nodes[idx].y))
            idx = nodes[idx].parent
        raw_path.reverse()
        working = list(raw_path)
        if params.prune_path and len(working) >= 2:
            pruned = _shortcut_prune(occupancy, working, params.collision_step)
            if len(pruned) >= 2:
                pruned_path = pruned
                working = pruned
        if len(working) >= 2 and params.spline_samples > 1:
            spline = catmull_rom_spline(working, samples_per_segment=params.spline_samples,
                                        alpha=params.spline_alpha, dedupe_tol=params.dedupe_tolerance)
            if len(spline) >= 2:
                smoothed_path = [tuple(map(float, pt)) for pt in spline]
                working = smoothed_path
        final_path = [tuple(map(float, pt)) for pt in working]
    else:
        LOG.warning("Failed to find a path within %d iterations", params.max_iterations)
    return PlanResult(
        success=success,
        path=final_path,
        nodes=nodes,
        iterations=iterations,
        goal_index=goal_index,
        raw_path=[tuple(map(float, pt)) for pt in raw_path],
        pruned_path=None if pruned_path is None else [tuple(map(float, pt)) for pt in pruned_path],
        smoothed_path=smoothed_path,
    )


def _shortcut_prune(occupancy, path, collision_step) -> List[Tuple[float, float]]:
    """``rrt_star.py:376-389``."""
    if len(path) <= 2:
        return list(path)
    pts = [tuple(map(float, pt)) for pt in path]
    pruned = [pts[0]]
    i = 0
    while i < len(pts) - 1:
        j = len(pts) - 1
        while j > i + 1 and not segment_is_free(occupancy, pts[i], pts[j], collision_step):
            j -= 1
        pruned.append(pts[j])
        i = j
    return pruned


class BatchedRRTStarPlanner:
    """Grow V RRT* trees on one occupancy grid at once on the GPU."""

    def __init__(self, occupancy: np.ndarray, params: PlannerParameters, *, device=None) -> None:
        import torch

        if not torch.cuda.is_available():
            raise _lib.LibraryError("BatchedRRTStarPlanner needs a ROCm GPU; there is no CPU fallback")
        if not 1 <= int(params.max_iterations) <= _lib.RRT_MAX_ITERATIONS:
            raise ValueError(f"max_iterations must be in [1, {_lib.RRT_MAX_ITERATIONS}]")
        self._torch = torch
        self.occupancy = np.ascontiguousarray(occupancy, dtype=np.uint8)
        self.params = params
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._occ = torch.from_numpy(self.occupancy).to(self.device)
        c = _lib.MpcqpRrtParams()
        c.step = float(params.step)
        c.goal_radius = float(params.goal_radius)
        c.rewire_radius = float(params.rewire_radius)
        c.collision_step = float(params.collision_step)
        c.goal_sample_rate = float(params.goal_sample_rate)
        c.max_iterations = int(params.max_iterations)
        c.height, c.width = (int(v) for v in self.occupancy.shape)
        self._c = c

    def grow(self, starts, goals, seeds, stream=None, *, host_samples: bool = False, samples=None):
        """Launch the tree growth; returns device tensors (nodes (V, M, 4), count (V,), meta (V, 2)).

        The samples replay ``numpy.random.default_rng(seed)``: drawn on the device from the
        generator's PCG64 state (default), or with ``host_samples=True`` by numpy itself, or
        given as ``samples`` (V, max_iterations, 2)."""
        torch = self._torch
        starts = np.asarray(starts, dtype=float).reshape(-1, 2)
        goals = np.asarray(goals, dtype=float).reshape(-1, 2)
        V = len(starts)
        T = int(self.params.max_iterations)
        dev = self.device
        sg = torch.from_numpy(np.hstack([starts, goals]) if V else np.zeros((1, 4))).to(dev)
        smp = rs = None
        if samples is not None:
            smp = torch.from_numpy(np.ascontiguousarray(samples, dtype=np.float64).reshape(V, T, 2)).to(dev)
        elif host_samples:
            samples = np.stack([draw_samples(int(s), g, self.occupancy.shape, self.params.goal_sample_rate, T)
                                for s, g in zip(seeds, goals)]) if V else np.zeros((1, T, 2))
            smp = torch.from_numpy(samples).to(dev)
        else:
            rs = torch.from_numpy(pcg64_states(seeds) if V else np.zeros((1, 4), np.uint64)).to(dev)
        nodes = torch.empty((max(V, 1), T + 2, 4), dtype=torch.float64, device=dev)
        count = torch.empty((max(V, 1),), dtype=torch.int32, device=dev)
        meta = torch.empty((max(V, 1), 2), dtype=torch.int32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        L = _lib.lib()
        with torch.cuda.device(dev):
            _lib.check(L.mpcqp_rrt_plan(ctypes.byref(self._c), V, self._occ.data_ptr(), sg.data_ptr(),
                                        None if smp is None else smp.data_ptr(),
                                        None if rs is None else rs.data_ptr(), nodes.data_ptr(), count.data_ptr(),
                                        meta.data_ptr(), ctypes.c_void_p(stream.cuda_stream)), "mpcqp_rrt_plan")
        return nodes[:V], count[:V], meta[:V]

    def extract(self, nodes, count, meta, stream=None):
        """Raw and shortcut-pruned paths of grown trees on the device (``mpcqp_rrt_paths``,
        ``rrt_star.py:245-262,376-389``): device tensors raw (V, M, 2), raw_len (V,),
        pruned (V, M, 2), pruned_len (V,)."""
        torch = self._torch
        V = int(nodes.shape[0])
        M = int(self.params.max_iterations) + 2
        dev = self.device
        raw = torch.empty((max(V, 1), M, 2), dtype=torch.float64, device=dev)
        pruned = torch.empty_like(raw)
        raw_len = torch.empty((max(V, 1),), dtype=torch.int32, device=dev)
        pruned_len = torch.empty_like(raw_len)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().mpcqp_rrt_paths(ctypes.byref(self._c), V, int(bool(self.params.prune_path)),
                                                  self._occ.data_ptr(), nodes.data_ptr(), count.data_ptr(),
                                                  meta.data_ptr(), raw.data_ptr(), raw_len.data_ptr(),
                                                  pruned.data_ptr(), pruned_len.data_ptr(),
                                                  ctypes.c_void_p(stream.cuda_stream)), "mpcqp_rrt_paths")
        return raw[:V], raw_len[:V], pruned[:V], pruned_len[:V]

    def smooth(self, paths, lens, stream=None, *, out_stride: int = 4096):
        """Centripetal Catmull-Rom of device paths ``paths`` (V, stride, 2) with ``lens`` (V,) points on
        the device (``mpcqp_catmull_rom``, ``rrt_star.py:104-159``); returns (out (V, out_stride, 2),
        out_len (V,)) device tensors (out_len -1: over capacity)."""
        torch = self._torch
        V = int(paths.shape[0])
        out = torch.empty((max(V, 1), out_stride, 2), dtype=torch.float64, device=self.device)
        out_len = torch.empty((max(V, 1),), dtype=torch.int32, device=self.device)
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        paths = paths.contiguous()
        lens = lens.to(torch.int32).contiguous()
        with torch.cuda.device(self.device):
            _lib.check(_lib.lib().mpcqp_catmull_rom(V, paths.data_ptr(), lens.data_ptr(), int(paths.shape[1]),
                                                    int(self.params.spline_samples), float(self.params.spline_alpha),
                                                    float(self.params.dedupe_tolerance), out.data_ptr(),
                                                    out_len.data_ptr(), int(out_stride),
                                                    ctypes.c_void_p(stream.cuda_stream)), "mpcqp_catmull_rom")
        return out[:V], out_len[:V]

    def paths_batch(self, starts, goals, seeds=None, *, smoothing: str = "host"
                    ) -> List[Optional[List[Tuple[float, float]]]]:
        """The final path of ``plan(start, goal)`` for every problem (None where no goal was
        reached), without building the tree on the host: growth, extraction and pruning run on
        the device; the Catmull-Rom smoothing (``rrt_star.py:264-283``) on the host from the
        pruned paths (``smoothing="host"``: equal to ``plan_batch(...)[v].path`` bit for bit) or on
        the device (``smoothing="device"``: within the ~1e-5 px that the reference's duplicated
        end points amplify an ulp to)."""
        starts = np.asarray(starts, dtype=float).reshape(-1, 2)
        V = len(starts)
        if seeds is None:
            seeds = [self.params.random_seed] * V
        nodes, count, meta = self.grow(starts, goals, seeds)
        _, _, pruned, plen_t = self.extract(nodes, count, meta)
        if smoothing == "device" and V:
            return self._device_final_paths(pruned, plen_t)
        plen = plen_t.cpu().numpy()
        L = int(plen.max()) if V else 0
        pts = pruned[:, :L].cpu().numpy()
        out: List[Optional[List[Tuple[float, float]]]] = []
        for v in range(V):
            n = int(plen[v])
            if n == 0:
                out.append(None)
                continue
            working = [tuple(map(float, pt)) for pt in pts[v, :n]]
            if n >= 2 and self.params.spline_samples > 1:
                spline = catmull_rom_spline(working, samples_per_segment=self.params.spline_samples,
                                            alpha=self.params.spline_alpha, dedupe_tol=self.params.dedupe_tolerance)
                if len(spline) >= 2:
                    working = [tuple(map(float, pt)) for pt in spline]
            out.append(working)
        return out

    def _device_final_paths(self, pruned, plen_t) -> List[Optional[List[Tuple[float, float]]]]:
        """rrt_star.py:264-283 with the smoothing on the device: the smoothed path when
        spline_samples > 1 and it has >= 2 points, else the pruned path."""
        plen = plen_t.cpu().numpy()
        smooth = self.params.spline_samples > 1
        if smooth:
            Lp = int(plen.max())
            sm, sl = self.smooth(pruned[:, :max(Lp, 1)], plen_t,
                                 out_stride=max(2, (max(Lp, 1) - 1) * max(2, self.params.spline_samples + 1) + 1))
            sl = sl.cpu().numpy()
            Ls = int(max(sl.max(), 1))
            sm = sm[:, :Ls].cpu().numpy()
        pts = pruned[:, :max(int(plen.max()), 1)].cpu().numpy()
        out: List[Optional[List[Tuple[float, float]]]] = []
        for v in range(len(plen)):
            n = int(plen[v])
            if n == 0:
                out.append(None)
            elif smooth and n >= 2 and sl[v] == -1:
                # the device smoothing's capacity (deduplicated points in LDS) is exceeded: the
                # reference would smooth this path (rrt_star.py:264-273), so do not hand back the
                # pruned one in its place
                raise RuntimeError(f"problem {v}: pruned path of {n} points exceeds the device "
                                   "Catmull-Rom capacity (mpcqp_catmull_rom returned -1)")
            elif smooth and n >= 2 and sl[v] >= 2:
                out.append([tuple(map(float, q)) for q in sm[v, : sl[v]]])
            else:
                out.append([tuple(map(float, q)) for q in pts[v, :n]])
        return out

    def plan_batch(self, starts, goals, seeds=None, *, samples=None) -> List[PlanResult]:
        """``plan(start, goal)`` for every problem (seed defaults to ``params.random_seed``;
        ``samples`` (V, max_iterations, 2) replaces the seeds' streams)."""
        starts = np.asarray(starts, dtype=float).reshape(-1, 2)
        V = len(starts)
        if seeds is None:
            seeds = [self.params.random_seed] * V
        nodes, count, meta = self.grow(starts, goals, seeds, samples=samples)
        nodes = nodes.cpu().numpy()
        count = count.cpu().numpy()
        meta = meta.cpu().numpy()
        out = []
        for v in range(V):
            tree = [RRTStarNode(float(x), float(y), float(c), None if p < 0 else int(p))
                    for x, y, c, p in nodes[v, : count[v]]]
            gi = int(meta[v, 1])
            out.append(_finish(self.occupancy, self.params, tree, int(meta[v, 0]), None if gi < 0 else gi))
        return out


class RRTStarPlanner:
    """Compute paths on an inflated occupancy grid (``rrt_star.py:192-357``); the tree grows
    on the GPU."""

    def __init__(self, occupancy: np.ndarray, params: PlannerParameters) -> None:
        self.occupancy = occupancy
        self.params = params
        # one generator per planner, advanced across plan() calls (rrt_star.py:199,296-301)
        self.rng = np.random.default_rng(params.random_seed)
        self._batched = None

    def plan(self, start: Tuple[float, float], goal: Tuple[float, float]) -> PlanResult:
        LOG.info("Running RRT* planner from %s to %s (max_iterations=%d)", start, goal, self.params.max_iterations)
        if self._batched is None:
            self._batched = BatchedRRTStarPlanner(self.occupancy, self.params)
        T = int(self.params.max_iterations)
        shape = np.asarray(self.occupancy).shape
        before = copy.deepcopy(self.rng.bit_generator.state)
        samples = draw_samples(self.rng, goal, shape, self.params.goal_sample_rate, T)
        result = self._batched.plan_batch([start], [goal], samples=samples[None])[0]
        # the reference draws one sample per iteration it runs (the loop breaks at the goal):
        # rewind and consume exactly that many, so the next plan() continues the same stream
        self.rng.bit_generator.state = before
        draw_samples(self.rng, goal, shape, self.params.goal_sample_rate, int(result.iterations))
        return result


__all__ = ["PlannerParameters", "RRTStarNode", "PlanResult", "RRTStarPlanner", "BatchedRRTStarPlanner",
           "draw_samples", "pcg64_states", "segment_is_free", "default_planner_parameters"]
