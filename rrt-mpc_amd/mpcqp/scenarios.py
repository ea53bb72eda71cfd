"""Synthetic batched MPC workloads (BASELINE.json configs 2-4).

All inputs derive from the reference's default pipeline run (map seed 4, RRT*
seed 13), captured once by ``tests/golden/gen_golden.py`` into
``mpcqp/data/default_plan.npz`` (plan path, start/goal, the 117-node RRT* tree).

* config 2 -- B identical QPs at N=20: the reference's first closed-loop QP
  (x0 = [start, yaw0, 5], window = ref_global[0:N+1], u_prev = 0;
  ``control_stage.py:80-105``) replicated.
* config 3 -- B randomised QPs at N=20 from RRT* tree branches: branch ->
  Catmull-Rom -> build_reference -> random window offset (tail-padded) ->
  perturbed x0 / u_prev.  ``numpy.random.default_rng(20240)``.
* config 4 -- B Monte-Carlo start poses at N=30 on the default window.
  ``numpy.random.default_rng(7)``.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Dict

import numpy as np

from .common.geometry import catmull_rom_spline
from .control.ref_builder import build_reference

DATA = Path(__file__).resolve().parent / "data" / "default_plan.npz"


@dataclass
class Batch:
    """Row-major float64 host arrays in the C-ABI layout (include/mpcqp.h)."""

    x0: np.ndarray  # (B, 4)
    ref: np.ndarray  # (B, N+1, 4)
    u_prev: np.ndarray  # (B, 2)
    horizon: int
    name: str

    @property
    def size(self) -> int:
        return int(self.x0.shape[0])


def load_default_plan() -> Dict[str, np.ndarray]:
    with np.load(DATA, allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def window(ref_global: np.ndarray, offset: int, horizon: int) -> np.ndarray:
    """``control_stage.py:101-105`` window gather with tail padding."""
    end = min(offset + horizon + 1, len(ref_global))
    w = ref_global[offset:end]
    if len(w) < horizon + 1:
        w = np.vstack((w, np.repeat(w[-1:], horizon + 1 - len(w), axis=0)))
    return w


def config2(batch: int = 1024, horizon: int = 20) -> Batch:
    plan = load_default_plan()
    ref_g = build_reference(plan["path"], 15.0, horizon, 0.1)
    x0 = np.array([plan["start"][0], plan["start"][1], float(plan["yaw0"]), 5.0])
    w = window(ref_g, 0, horizon)
    return Batch(
        x0=np.tile(x0, (batch, 1)),
        ref=np.tile(w, (batch, 1, 1)),
        u_prev=np.zeros((batch, 2)),
        horizon=horizon,
        name=f"config2_identical_B{batch}_N{horizon}",
    )


def _tree_depth(parent: np.ndarray) -> np.ndarray:
    depth = np.zeros(len(parent), dtype=int)
    for i in range(len(parent)):
        d, j = 0, i
        while parent[j] >= 0:
            d += 1
            j = parent[j]
        depth[i] = d
    return depth


def config3(batch: int = 4096, horizon: int = 20, seed: int = 20240) -> Batch:
    plan = load_default_plan()
    nodes = plan["nodes"]
    parent = nodes[:, 3].astype(int)
    eligible = np.flatnonzero(_tree_depth(parent) >= 3)
    rng = np.random.default_rng(seed)
    cache: Dict[int, np.ndarray] = {}
    x0 = np.zeros((batch, 4))
    ref = np.zeros((batch, horizon + 1, 4))
    u_prev = np.zeros((batch, 2))
    sd_x = np.array([2.0, 2.0, 0.3, 2.0])
    sd_u = np.array([3.0, 0.05])
    for b in range(batch):
        node = int(eligible[rng.integers(0, len(eligible))])
        if node not in cache:
            pts, j = [], node
            while j >= 0:
                pts.append(nodes[j, :2])
                j = parent[j]
            spline = catmull_rom_spline(pts[::-1], samples_per_segment=20, alpha=0.5)
            cache[node] = build_reference(spline, 15.0, horizon, 0.1)
        ref_g = cache[node]
        w = window(ref_g, int(rng.integers(0, len(ref_g))), horizon)
        ref[b] = w
        x0[b] = w[0] + rng.normal(0.0, 1.0, 4) * sd_x
        u_prev[b] = rng.normal(0.0, 1.0, 2) * sd_u
    return Batch(x0, ref, u_prev, horizon, f"config3_rrt_branches_B{batch}_N{horizon}")


def config4(batch: int = 16384, horizon: int = 30, seed: int = 7) -> Batch:
    plan = load_default_plan()
    ref_g = build_reference(plan["path"], 15.0, horizon, 0.1)
    w = window(ref_g, 0, horizon)
    rng = np.random.default_rng(seed)
    yaw0 = float(plan["yaw0"])
    x0 = np.column_stack(
        [
            plan["start"][0] + rng.uniform(-5, 5, batch),
            plan["start"][1] + rng.uniform(-5, 5, batch),
            yaw0 + rng.uniform(-0.5, 0.5, batch),
            rng.uniform(0, 15, batch),
        ]
    )
    return Batch(x0, np.tile(w, (batch, 1, 1)), np.zeros((batch, 2)), horizon,
                 f"config4_montecarlo_B{batch}_N{horizon}")


def fleet5(vehicles: int = 100, seed: int = 5):
    """Config-5-style fleet: V vehicles on RRT* tree branches of the default plan
    (root -> random node of depth >= 3, Catmull-Rom smoothed as the planner does), start = branch
    start + U(-3, 3) px, goal = branch end.  Returns (paths, starts (V, 2), goals (V, 2))."""
    plan = load_default_plan()
    nodes = plan["nodes"]
    parent = nodes[:, 3].astype(int)
    eligible = np.flatnonzero(_tree_depth(parent) >= 3)
    rng = np.random.default_rng(seed)
    cache: Dict[int, np.ndarray] = {}
    paths = []
    for _ in range(vehicles):
        node = int(eligible[rng.integers(0, len(eligible))])
        if node not in cache:
            pts, j = [], node
            while j >= 0:
                pts.append(nodes[j, :2])
                j = parent[j]
            cache[node] = catmull_rom_spline(pts[::-1], samples_per_segment=20, alpha=0.5)
        paths.append(cache[node])
    starts = np.array([p[0] for p in paths]) + rng.uniform(-3, 3, size=(vehicles, 2))
    goals = np.array([p[-1] for p in paths])
    return paths, starts, goals


CONFIGS = {"config2": config2, "config3": config3, "config4": config4}

__all__ = ["Batch", "config2", "config3", "config4", "fleet5", "CONFIGS", "load_default_plan", "window"]
