#!/usr/bin/env python3
"""Closed-loop fleet benchmark (BASELINE config 5 style): V vehicles on
RRT*-branch plans, references built on the device, `sim_steps` closed-loop MPC steps each, every
step on the GPU (mpcqp_fleet_run, hipGraph replay per step; --fused: mpcqp_fleet_loop, the whole
loop in one launch).  Reports vehicle-steps/s (one vehicle-step =
window + nominal QP (+ relaxed retry) + plant + path_idx/goal update) and, for scale, the
reference-style host loop (TrajectoryTracker.track, one B=1 solve per step) on one vehicle.

    python tools/fleet_bench.py [--vehicles 100 1024 4096] [--steps 100] [--horizon 15] [--fused]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path
from types import SimpleNamespace

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--vehicles", type=int, nargs="+", default=[100, 1024, 4096])
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--horizon", type=int, default=15)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fused", action="store_true", help="mpcqp_fleet_loop: one launch for the whole loop")
    ap.add_argument("--pairing", default="auto", choices=["auto", "on", "off"],
                    help="two vehicles per wave for N <= 15 (mpcqp_set_pairing)")
    a = ap.parse_args()
    import torch

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker
    from mpcqp.pipeline.fleet import FleetTracker

    dev = torch.device("cuda:0")
    out = {"metric": "closed-loop vehicle-steps/s", "horizon": a.horizon, "sim_steps": a.steps,
           "mode": "fused loop (mpcqp_fleet_loop)" if a.fused else "graph-replayed steps (mpcqp_fleet_run)", "runs": []}
    for V in a.vehicles:
        paths, starts, goals = scenarios.fleet5(V)
        mpc = MPCConfig(horizon=a.horizon, sim_steps=a.steps)
        ft = FleetTracker(mpc, map_resolution=0.8, max_vehicles=V, max_ref_len=160, device=dev, fused=a.fused,
                          pairing=a.pairing)
        best = None
        for r in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ft.reset_from_plans(paths, starts, goals, device_reference=True)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ft.step(a.steps)  # masked vehicles cost an exiting wave; no host check inside the run
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            dt = t2 - t0
            res = ft.result()
            if r and (best is None or dt < best[0]):
                best = (dt, res, t2 - t1, t1 - t0)
        dt, res, loop_dt, reset_dt = best
        vsteps = int(res.steps.sum())
        out["runs"].append({
            "vehicles": V, "seconds": dt, "vehicle_steps": vsteps, "value": vsteps / dt,
            "goal_reached": int((res.phase == 1).sum()), "aborted": int((res.phase == 2).sum()),
            "ms_per_step": 1e3 * dt / a.steps,
            # the loop alone (ft.step after the references are built and loaded): the fused kernel
            "loop_seconds": loop_dt, "loop_value": vsteps / loop_dt, "reset_seconds": reset_dt,
        })
        ft.close()
        print(json.dumps(out["runs"][-1]), flush=True)
    # reference-style host loop: one vehicle, one solve (B=1 kernel launch + sync) per step
    paths, starts, goals = scenarios.fleet5(1)
    tr = TrajectoryTracker(MPCConfig(horizon=a.horizon, sim_steps=a.steps), VizConfig())
    planning = SimpleNamespace(plan=SimpleNamespace(success=True, path=[tuple(map(float, q)) for q in paths[0]]))
    maps = SimpleNamespace(start=tuple(starts[0]), goal=tuple(goals[0]))
    tr.track(planning, maps, map_resolution=0.8, visualize=False)
    t0 = time.perf_counter()
    st = tr.track(planning, maps, map_resolution=0.8, visualize=False).states
    dt = time.perf_counter() - t0
    out["host_loop_one_vehicle"] = {"vehicle_steps": len(st), "seconds": dt, "value": len(st) / dt}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
