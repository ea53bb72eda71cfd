#!/usr/bin/env python3
"""Development tool: split k_solve time into phases by timing solver-setting variants.

    python tools/phase_timing.py [--config config3] [--batch 4096]

Each variant runs the same batch; differences isolate setup (condense + Ruiz),
KKT factorizations, ADMM iterations and polish iterations.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = getattr(scenarios, args.config)(args.batch)
    N = b.horizon
    params = MPCConfig(horizon=N).to_parameters(0.8)
    dev = torch.device("cuda:0")
    x0 = torch.from_numpy(b.x0).to(dev)
    ref = torch.from_numpy(b.ref).to(dev)
    up = torch.from_numpy(b.u_prev).to(dev)
    variants = {
        "default": dict(),
        "admm_only": dict(polish=0),
        "setup+1it": dict(max_iter=1, polish=0),
        "setup+1it_noscale": dict(max_iter=1, polish=0, scaling=0),
        "setup+51it_fixed_rho": dict(max_iter=51, polish=0, adaptive_rho=0, check_termination=1000),
        "setup+101it_fixed_rho": dict(max_iter=101, polish=0, adaptive_rho=0, check_termination=1000),
        "newton": dict(method="newton"),
    }
    res = {}
    for name, kw in variants.items():
        kw = dict(kw)
        method = kw.pop("method", "admm")
        ctrl = BatchedMPCController(params, args.batch, device=dev, method=method, **kw)
        L = _lib.lib()
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        times = []
        for r in range(args.reps + 1):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            _lib.check(L.mpcqp_build(ctrl._ws, args.batch, x0.data_ptr(), ref.data_ptr(), up.data_ptr(), s), "b")
            e1.record()
            _lib.check(L.mpcqp_solve(ctrl._ws, args.batch, ctrl._u0.data_ptr(), ctrl._X.data_ptr(),
                                     ctrl._U.data_ptr(), ctrl._status.data_ptr(), ctrl._iters.data_ptr(),
                                     ctrl._active.data_ptr(), s), "s")
            e2.record()
            torch.cuda.synchronize()
            if r:
                times.append(e1.elapsed_time(e2))
        it = ctrl._iters[: args.batch].cpu().numpy()
        res[name] = dict(k_solve_ms=float(np.median(times)), iters_mean=it.mean(axis=0).round(2).tolist(),
                         iters_max=it.max(axis=0).tolist())
        ctrl.close()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
