"""Generate planning.npz (occupancy inflation + RRT* goldens) by importing the reference's Python.

Run in the build container only (``/root/reference`` does not exist on the GPU box):

    python tests/golden/gen_golden_planning.py

Same import-only ``cvxpy`` stub as gen_golden.py (the planner and map modules never call it).
Outputs (numpy ``.npz``, no pickled objects):
  inflate_*   src/maps/inflate.py:18-51  _fallback_dilation / inflate_binary_occupancy (cv2 is
              absent, so the reference itself takes the fallback) on the default raw map at the
              configured radius and on seeded random grids at radii 0..5
  rrt_*       src/planning/rrt_star.py:201-357  RRTStarPlanner.plan on the default inflated map
              for several (start, goal, seed) cases: the tree (x, y, cost, parent), iterations,
              goal index, raw / pruned / final path
"""
from __future__ import annotations

import os
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REFERENCE = Path(os.environ.get("RRT_MPC_REFERENCE", "/root/reference"))
sys.path.insert(0, str(HERE))

from gen_golden import _install_cvxpy_stub  # noqa: E402

# (start, goal, seed, max_iterations): the default case first, then other corners of the map
# (start None = the map's start (70, 70); goal None = the map's goal (10, 10))
RRT_CASES = [
    (None, None, 13, 2000),  # the default pipeline's plan (default_plan.npz)
    (None, None, 7, 2000),
    ((70.0, 10.0), (10.0, 70.0), 21, 2000),
    ((40.0, 5.0), (40.0, 75.0), 3, 2000),
    (None, None, 99, 60),  # iteration cap before the goal: success=False
]


def main() -> None:
    _install_cvxpy_stub()
    sys.path.insert(0, str(REFERENCE))
    import matplotlib

    matplotlib.use("Agg")
    from src.config import default_config
    from src.maps.inflate import inflate_binary_occupancy, inflation_radius_pixels, to_occupancy_grid
    from src.pipeline.map_stage import MapStage
    from src.planning.rrt_star import RRTStarPlanner

    tmp = Path(tempfile.mkdtemp(prefix="rrtmpc_golden_"))
    cfg = default_config()
    cfg.map.map_file = str(tmp / "base.png")
    cfg.map.inflated_map_file = str(tmp / "inflated.png")
    cfg.map.generate = True
    cfg.viz.backend = "Agg"
    stage = MapStage(cfg.map)
    raw = stage.ensure_base_map()
    maps = stage.build()
    out = {}
    # ---------------- inflation ----------------
    radius = inflation_radius_pixels(cfg.map.inflation_radius_m, cfg.map.map_resolution)
    occ = to_occupancy_grid(raw)
    out["inflate_default_in"] = occ.astype(np.uint8)
    out["inflate_default_radius"] = np.int64(radius)
    out["inflate_default_out"] = inflate_binary_occupancy(occ, radius).astype(np.uint8)
    rng = np.random.default_rng(11)
    grids, radii, results = [], [], []
    for r in range(0, 6):
        g = (rng.random((37, 53)) > 0.04).astype(np.uint8)  # sparse obstacles, odd sizes
        grids.append(g)
        radii.append(r)
        results.append(inflate_binary_occupancy(g, r).astype(np.uint8))
    out["inflate_random_in"] = np.stack(grids)
    out["inflate_random_radius"] = np.array(radii)
    out["inflate_random_out"] = np.stack(results)
    # ---------------- RRT* ----------------
    occupancy = maps.occupancy
    out["rrt_occupancy"] = occupancy.astype(np.uint8)
    base = cfg.planner.to_parameters()
    for k, (start, goal, seed, iters) in enumerate(RRT_CASES):
        start = start if start is not None else tuple(map(float, maps.start))
        goal = goal if goal is not None else tuple(map(float, maps.goal))
        params = type(base)(**{**base.__dict__, "random_seed": seed, "max_iterations": iters})
        res = RRTStarPlanner(occupancy, params).plan(start, goal)
        nodes = np.array([[n.x, n.y, n.cost, -1 if n.parent is None else n.parent] for n in res.nodes])
        out[f"rrt{k}_case"] = np.array([start[0], start[1], goal[0], goal[1], seed, iters], dtype=float)
        out[f"rrt{k}_nodes"] = nodes
        out[f"rrt{k}_meta"] = np.array([int(res.success), res.iterations,
                                        -1 if res.goal_index is None else res.goal_index])
        out[f"rrt{k}_raw_path"] = np.asarray(res.raw_path, dtype=float).reshape(-1, 2)
        out[f"rrt{k}_pruned_path"] = np.asarray(res.pruned_path or [], dtype=float).reshape(-1, 2)
        out[f"rrt{k}_path"] = np.asarray(res.path, dtype=float).reshape(-1, 2)
    out["rrt_params"] = np.array([base.step, base.goal_radius, base.rewire_radius, base.goal_sample_rate,
                                  base.collision_step, base.spline_samples, base.spline_alpha,
                                  base.dedupe_tolerance, float(base.prune_path)])
    np.savez_compressed(HERE / "planning.npz", **out)
    print("wrote", HERE / "planning.npz", {k: np.asarray(v).shape for k, v in out.items() if k.endswith("nodes")})


if __name__ == "__main__":
    main()
