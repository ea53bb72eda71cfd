#!/usr/bin/env python3
"""Development A/B: every output of the batched solve on fixed workloads, saved for a bitwise
comparison between two kernel builds (a kernel change that claims the same arithmetic must
reproduce these arrays bit for bit).

    python tools/dump_outputs.py gpurun_out/outputs_<tag>.npz
    python tools/dump_outputs.py --compare a.npz b.npz
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "rrt-mpc_amd")]

WORKLOADS = [("config2", 20, 1024), ("config3", 20, 4096), ("config4", 30, 4096), ("config3", 10, 1024),
             ("config3", 15, 1024), ("config3", 32, 512), ("config3", 40, 256), ("config3", 4, 1024),
             ("config3", 8, 1024), ("config3", 16, 1024), ("config3", 10, 4096), ("config3", 15, 4096)]


def dump(path: str) -> None:
    import torch

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    out = {}
    for cfg, N, B in WORKLOADS:
        b = (scenarios.config2(B, horizon=N) if cfg == "config2" else
             scenarios.config4(B) if cfg == "config4" else scenarios.config3(B, horizon=N))
        ctrl = BatchedMPCController(MPCConfig(horizon=b.horizon).to_parameters(0.8), B, device="cuda:0")
        sol = ctrl.solve_batch(b.x0, b.ref, b.u_prev)
        torch.cuda.synchronize()
        for k in sol._fields:
            out[f"{cfg}_N{N}_{k}"] = getattr(sol, k).cpu().numpy().copy()
        ctrl.close()
    np.savez(path, **out)
    print(f"wrote {path}: {len(out)} arrays")


def compare(a: str, b: str) -> int:
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in sorted(set(A.files) | set(B.files)):
        if k not in A.files or k not in B.files:
            print(f"{k}: missing in one file")
            bad += 1
            continue
        x, y = A[k], B[k]
        if x.shape != y.shape or not np.array_equal(x.view(np.uint8), y.view(np.uint8)):
            diff = np.abs(x.astype(float) - y.astype(float))
            print(f"{k}: differs ({int((diff > 0).sum())} entries, max {diff.max():.3e})")
            bad += 1
    print("bitwise identical" if not bad else f"{bad} arrays differ")
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    dump(sys.argv[1])
