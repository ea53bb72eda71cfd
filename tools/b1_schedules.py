#!/usr/bin/env python3
"""Config 1 (the reference's single-vehicle loop, N = 10, 65 solves) through the drop-in
TrajectoryTracker under several B=1 solver schedules: ms per step (best of 5) and the kernel's own
per-QP time (HIP events over the 65 windows from device memory).  Every schedule ends at the exact
optimum; the states must agree with the reference loop (closed_loop.npz) to 1e-7 px.

    python tools/b1_schedules.py > profiles/<round>_b1_schedules.json
"""
from __future__ import annotations

import ctypes
import json
import sys
import time
from pathlib import Path
from types import SimpleNamespace

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "rrt-mpc_amd"), str(ROOT)]

SCHEDULES = [
    {"polish_from": 25},
    {"polish_from": 10, "check_termination": 10, "adaptive_rho_interval": 10},
    {"polish_from": 15, "check_termination": 15, "adaptive_rho_interval": 15},
    {"polish_from": 5, "check_termination": 5, "adaptive_rho_interval": 25},
    {"polish_from": 10, "check_termination": 10, "adaptive_rho_interval": 20},
]


def main() -> None:
    import torch

    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.control.mpc_controller import BatchedMPCController
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    g = np.load(ROOT / "tests" / "golden" / "closed_loop.npz")
    ref_states = g["N10_states"]
    wins, x0s, ups = g["N10_window"], g["N10_x0"], g["N10_u_prev"]
    plan = scenarios.load_default_plan()
    path = [tuple(map(float, q)) for q in plan["path"]]
    planning = SimpleNamespace(plan=SimpleNamespace(success=True, path=path))
    maps = SimpleNamespace(start=tuple(plan["start"]), goal=tuple(plan["goal"]))
    params = MPCConfig(horizon=10).to_parameters(0.8)
    dev = torch.device("cuda:0")
    x0_t, w_t, up_t = (torch.from_numpy(a).to(dev) for a in (x0s, wins, ups))
    L = _lib.lib()
    out = []
    for sched in SCHEDULES:
        tr = TrajectoryTracker(MPCConfig(horizon=10, sim_steps=100), VizConfig(), solver_settings=dict(sched),
                               relaxed_solver_settings=dict(sched))
        st = tr.track(planning, maps, map_resolution=0.8, visualize=False).states
        best = None
        for _ in range(5):
            t0 = time.perf_counter()
            st = tr.track(planning, maps, map_resolution=0.8, visualize=False).states
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        dev_px = float(np.abs(np.asarray(st) - ref_states).max()) if len(st) == len(ref_states) else None
        ctrl = BatchedMPCController(params, 1, device=dev, **sched)
        stream = torch.cuda.current_stream(dev)
        s = ctypes.c_void_p(stream.cuda_stream)
        ks, its = [], []
        for rep in range(2):
            for q in range(len(wins)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                _lib.check(L.mpcqp_build(ctrl._ws, 1, x0_t[q].data_ptr(), w_t[q].data_ptr(), up_t[q].data_ptr(), s), "b")
                _lib.check(L.mpcqp_solve(ctrl._ws, 1, ctrl._u0.data_ptr(), ctrl._X.data_ptr(), ctrl._U.data_ptr(),
                                         ctrl._status.data_ptr(), ctrl._iters.data_ptr(), ctrl._active.data_ptr(), s), "s")
                e1.record(stream)
                torch.cuda.synchronize(dev)
                if rep:
                    ks.append(e0.elapsed_time(e1) * 1e3)
                    its.append(ctrl._iters[0].cpu().numpy().tolist())
        ctrl.close()
        its = np.asarray(its, float)
        out.append({"settings": sched, "track_ms_per_step": 1e3 * best / len(st), "steps": len(st),
                    "max_state_diff_vs_reference_px": dev_px, "kernel_us_mean": float(np.mean(ks)),
                    "kernel_us_max": float(np.max(ks)), "iters_mean": its.mean(axis=0).round(2).tolist()})
        print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
