#!/usr/bin/env python3
"""Where a B=1 drop-in step's time goes (config 1: one QP per closed-loop step, N = 10).

    python tools/b1_latency.py [--horizon 10] [--calls 400] > profiles/<round>_b1_latency.json

Each figure is the best of 5 repeats of `calls` calls on the config-1 windows (the reference loop's
own 65 windows of closed_loop.npz, cycled):
  * staged_c          mpcqp_solve_staged alone (inputs already in the mapped block): launch + kernel +
                      stream sync, the library's floor for one QP from the host;
  * solve_one         BatchedMPCController.solve_one (write the inputs, the staged call, copy outputs);
  * mpc_controller    MPCController(params).solve as the tracker calls it (+ argument handling and
                      the controller cache lookup);
  * device_inputs     the same QP from device memory with the caller's torch stream: mpcqp_build +
                      mpcqp_solve + torch.cuda.synchronize (no mapped memory);
  * kernel_event_us   HIP events around the device-input solve (the kernel alone, on its stream);
  * track_ms_per_step the whole drop-in TrajectoryTracker.track loop (bench.py's config1 figure).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path
from types import SimpleNamespace

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "rrt-mpc_amd"), str(ROOT)]


def best_of(fn, calls: int, reps: int = 5) -> float:
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        for k in range(calls):
            fn(k)
        dt = (time.perf_counter() - t0) / calls * 1e6
        best = dt if best is None else min(best, dt)
    return best


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--calls", type=int, default=400)
    a = ap.parse_args()
    import torch

    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.control.mpc_controller import MPCController, _single_controller
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    N = a.horizon
    g = np.load(ROOT / "tests" / "golden" / "closed_loop.npz")
    key = f"N{N}_window" if f"N{N}_window" in g.files else None
    if key is None:
        raise SystemExit(f"closed_loop.npz has no N={N} windows ({g.files})")
    wins, x0s, ups = g[f"N{N}_window"], g[f"N{N}_x0"], g[f"N{N}_u_prev"]
    n = len(wins)
    params = MPCConfig(horizon=N).to_parameters(0.8)
    ctrl = _single_controller(params)
    L = _lib.lib()
    out = {"horizon": N, "calls": a.calls, "windows": n, "settings": dict(ctrl.settings)}

    ctrl.solve_one(x0s[0], wins[0], ups[0])  # warm: staging blocks, code objects
    io = ctrl._one

    def staged(k):
        q = k % n
        io["x0"][:] = x0s[q]
        io["ref"][:] = wins[q]
        io["up"][:] = ups[q]
        L.mpcqp_solve_staged(ctrl._ws)

    # the C call alone: the inputs written once, then the call repeated on them
    staged(0)
    out["staged_c_us"] = best_of(lambda k: L.mpcqp_solve_staged(ctrl._ws), a.calls)
    out["staged_with_input_writes_us"] = best_of(staged, a.calls)
    out["solve_one_us"] = best_of(lambda k: ctrl.solve_one(x0s[k % n], wins[k % n], ups[k % n]), a.calls)
    out["mpc_controller_us"] = best_of(
        lambda k: MPCController(params).solve(x0s[k % n], wins[k % n], u_prev=ups[k % n]), a.calls)

    dev = torch.device("cuda:0")
    x0_t = torch.from_numpy(x0s).to(dev)
    w_t = torch.from_numpy(wins).to(dev)
    up_t = torch.from_numpy(ups).to(dev)
    stream = torch.cuda.current_stream(dev)
    s = ctypes.c_void_p(stream.cuda_stream)

    def device_call(k):
        q = k % n
        _lib.check(L.mpcqp_build(ctrl._ws, 1, x0_t[q].data_ptr(), w_t[q].data_ptr(), up_t[q].data_ptr(), s), "build")
        _lib.check(L.mpcqp_solve(ctrl._ws, 1, ctrl._u0.data_ptr(), ctrl._X.data_ptr(), ctrl._U.data_ptr(),
                                 ctrl._status.data_ptr(), ctrl._iters.data_ptr(), ctrl._active.data_ptr(), s), "solve")
        torch.cuda.synchronize(dev)

    out["device_inputs_us"] = best_of(device_call, a.calls)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for q in range(n):
        ev[q][0].record(stream)
        _lib.check(L.mpcqp_build(ctrl._ws, 1, x0_t[q].data_ptr(), w_t[q].data_ptr(), up_t[q].data_ptr(), s), "build")
        _lib.check(L.mpcqp_solve(ctrl._ws, 1, ctrl._u0.data_ptr(), ctrl._X.data_ptr(), ctrl._U.data_ptr(),
                                 ctrl._status.data_ptr(), ctrl._iters.data_ptr(), ctrl._active.data_ptr(), s), "solve")
        ev[q][1].record(stream)
        torch.cuda.synchronize(dev)
    ks = np.array([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev])
    out["kernel_event_us"] = {"mean": float(ks.mean()), "min": float(ks.min()), "max": float(ks.max())}

    plan = scenarios.load_default_plan()
    path = [tuple(map(float, q)) for q in plan["path"]]
    tracker = TrajectoryTracker(MPCConfig(horizon=N, sim_steps=100), VizConfig())
    planning = SimpleNamespace(plan=SimpleNamespace(success=True, path=path))
    maps = SimpleNamespace(start=tuple(plan["start"]), goal=tuple(plan["goal"]))
    tracker.track(planning, maps, map_resolution=0.8, visualize=False)
    best = None
    for _ in range(5):
        t0 = time.perf_counter()
        st = tracker.track(planning, maps, map_resolution=0.8, visualize=False).states
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    out["track_ms_per_step"] = 1e3 * best / len(st)
    out["track_steps"] = len(st)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
