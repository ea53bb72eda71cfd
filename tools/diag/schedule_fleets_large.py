#!/usr/bin/env python3
"""Polish schedule on the fused fleets and swarm at scale: fused fleet loop (N = 15, 100 steps) at
100 / 1024 / 4096 vehicles and the fused config-5 swarm at 100 / 1024 vehicles, polish_from 75 / 50 / 25, interleaved, best of three each.

    python tools/diag/schedule_fleets_large.py
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "rrt-mpc_amd"), str(ROOT / "tools")]
SCHEDULES = [{"polish_from": 75}, {"polish_from": 50}, {"polish_from": 25}]


def fleet_time(V, settings, dev):
    import torch
    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.pipeline.fleet import FleetTracker

    paths, starts, goals = scenarios.fleet5(V)
    ft = FleetTracker(MPCConfig(horizon=15, sim_steps=100), map_resolution=0.8, max_vehicles=V, max_ref_len=160,
                      device=dev, fused=True, **settings)
    best = None
    for _ in range(4):
        ft.reset_from_plans(paths, starts, goals, device_reference=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ft.step(100)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    ft.close()
    return best


def swarm_time(V, settings, dev):
    import torch
    from swarm_bench import pairs
    from mpcqp.config import MPCConfig
    from mpcqp.pipeline.swarm import Swarm
    from mpcqp.planning.rrt_star import default_planner_parameters

    occ = np.load(ROOT / "rrt-mpc_amd" / "mpcqp" / "data" / "default_plan.npz")["occupancy"]
    starts, goals = pairs(occ, V, 5)
    sw = Swarm(occ, MPCConfig(horizon=15, sim_steps=300), default_planner_parameters(), map_resolution=0.8,
               max_vehicles=V, device=dev, replan_distance=5.5, max_replans=2, fused=True, **settings)
    sw.run(starts[:4], goals[:4], seeds=np.arange(4), sim_steps=5)
    best = None
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sw.run(starts, goals, seeds=np.arange(V), check_every=50)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best


def main() -> None:
    import torch

    dev = torch.device("cuda:0")
    out = {"what": __doc__.split("\n\n")[0], "fleet_s": {}, "swarm_s": {}}
    for rep in range(2):
        for settings in SCHEDULES:
            key = json.dumps(settings)
            for V in (100, 1024, 4096):
                out["fleet_s"].setdefault(key, {}).setdefault(str(V), []).append(fleet_time(V, settings, dev))
            for V in (100, 1024):
                out["swarm_s"].setdefault(key, {}).setdefault(str(V), []).append(swarm_time(V, settings, dev))
            print(key, json.dumps({k: out[k][key] for k in ("fleet_s", "swarm_s")}), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
