#!/usr/bin/env python3
"""Development check: the B=1 server kernel (k_serve<N>) against a launch per call (k_solve<N>) on the
same QPs: statuses, counters and the largest output difference per horizon and schedule."""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "rrt-mpc_amd")]


def run(N, settings, mode, b):
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    os.environ["MPCQP_B1_SERVER"] = mode
    ctrl = BatchedMPCController(MPCConfig(horizon=N).to_parameters(0.8), 1, device="cuda:0", **settings)
    out = []
    for q in range(b.size):
        st, u0, X, U = ctrl.solve_one(b.x0[q], b.ref[q], b.u_prev[q])
        out.append((st, U.copy(), X.copy(), ctrl._one["iters"].copy()))
    ctrl.close()
    return out


def main():
    from mpcqp import scenarios

    res = []
    for N in (10, 15, 20, 31):
        for settings in ({}, {"max_iter": 50, "polish_from": 0, "polish_near": 0.0}):
            b = scenarios.config3(64, horizon=N, seed=41 + N)
            a, c = run(N, settings, "0", b), run(N, settings, "1", b)
            dU = max(float(np.abs(x[1] - y[1]).max()) for x, y in zip(a, c))
            same_bits = sum(np.array_equal(x[1], y[1]) and np.array_equal(x[2], y[2]) for x, y in zip(a, c))
            res.append({"N": N, "settings": settings, "status_equal": all(x[0] == y[0] for x, y in zip(a, c)),
                        "iters_equal": all(np.array_equal(x[3], y[3]) for x, y in zip(a, c)),
                        "bitwise_equal_qps": same_bits, "qps": b.size, "max_abs_dU": dU})
            print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
