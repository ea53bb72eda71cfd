#!/usr/bin/env python3
"""Iteration indexing of the product path: the fraction of QPs whose four counters (ADMM
iterations, polish passes, factorizations, line-search trials), status and active set equal the C
restatement's (oracle/mpcqp_cpu.c), over the BASELINE configs at full size, config 3 at the
one-wave horizons and at mid horizons.  Writes one JSON object (profiles/r03_*_iters_agreement.json).

    python tools/iters_agreement.py [--quick]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "rrt-mpc_amd"), str(ROOT / "oracle")]


def agreement(params, batch, **settings) -> dict:
    import cpu_solver
    import torch
    from mpcqp.control.mpc_controller import BatchedMPCController

    B = batch.size
    ctrl = BatchedMPCController(params, B, device="cuda:0", **settings)
    sol = ctrl.solve_batch(batch.x0, batch.ref, batch.u_prev)
    torch.cuda.synchronize()
    g = {k: getattr(sol, k).cpu().numpy() for k in ("iters", "status", "active", "U")}
    ctrl.close()
    ref = cpu_solver.cpu_solve(params, batch.x0, batch.ref, batch.u_prev, nthreads=16, **settings)
    same = g["iters"] == ref["iters"]
    bad = np.flatnonzero(~same.all(axis=1))
    return {
        "qps": int(B),
        "iters_agreement": float(same.all(axis=1).mean()),
        "per_counter": {k: float(same[:, i].mean()) for i, k in enumerate(("admm", "polish", "fact", "ls"))},
        "status_equal": bool(np.array_equal(g["status"], ref["status"])),
        "active_equal": bool(np.array_equal(g["active"], ref["active"])),
        "max_rel_U": float(np.abs(g["U"] - ref["U"]).max() / max(1.0, np.abs(ref["U"]).max())),
        "disagreeing_qps": bad[:20].tolist(),
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    from mpcqp import scenarios
    from mpcqp.config import MPCConfig

    P = lambda N: MPCConfig(horizon=N).to_parameters(0.8)  # noqa: E731
    out = {"what": "GPU product path (fast kernel) vs C restatement: counters / status / active set", "runs": {}}
    t0 = time.time()
    runs = [("config2_B1024_N20", lambda: scenarios.config2(), {}),
            ("config3_B4096_N20", lambda: scenarios.config3(), {}),
            ("config3_B4096_N20_polish_near0", lambda: scenarios.config3(), {"polish_near": 0.0}),
            ("config3_B4096_N20_osqp_order", lambda: scenarios.config3(), {"polish_from": 0, "polish_near": 0.0}),
            ("config4_B16384_N30", lambda: scenarios.config4(2048 if a.quick else 16384), {})]
    for N in ([5, 10, 31] if a.quick else [1, 2, 3, 5, 8, 10, 12, 15, 18, 21, 24, 26, 28, 29, 30, 31]):
        runs.append((f"config3_B1024_N{N}", (lambda N=N: scenarios.config3(1024, horizon=N, seed=5000 + N)), {}))
    # the mid-horizon kernel (N = 32..63, k_solve_mid)
    for N in ([40] if a.quick else [32, 36, 40, 48, 56, 63]):
        runs.append((f"config3_B1024_N{N}_mid", (lambda N=N: scenarios.config3(1024, horizon=N, seed=5000 + N)), {}))
    for name, mk, settings in runs:
        b = mk()
        out["runs"][name] = agreement(P(b.horizon), b, **settings)
        print(name, json.dumps(out["runs"][name]), file=sys.stderr, flush=True)
    tot = sum(r["qps"] for r in out["runs"].values())
    agree = sum(r["qps"] * r["iters_agreement"] for r in out["runs"].values())
    out["total_qps"] = tot
    out["overall_iters_agreement"] = agree / tot
    out["seconds"] = time.time() - t0
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
