#!/usr/bin/env python3
"""Development tool: per-phase cycle attribution from the -DMPCQP_STAMPS diagnostic build.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DMPCQP_STAMPS -DMPCQP_ONLY_N=20 \
        -o build/libmpcqp_stamps.so rrt-mpc_amd/csrc/mpcqp.hip
    MPCQP_LIB=build/libmpcqp_stamps.so python tools/stamps.py

Stamps serialize around each phase, so read the SHARES, never the absolute run time.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
os.environ.setdefault("MPCQP_LIB", str(ROOT / "build" / "libmpcqp_stamps.so"))
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))

NAMES = {0: "admm.form", 1: "admm.sweep", 2: "admm.iteration", 3: "admm.check", 4: "admm.total",
         8: "polish.form", 9: "polish.sweep", 10: "polish.solve", 11: "polish.linesearch", 12: "polish.total"}


def main() -> None:
    import torch

    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
    b = getattr(scenarios, cfg)()
    B = b.size
    ctrl = BatchedMPCController(MPCConfig(horizon=b.horizon).to_parameters(0.8), B, device="cuda:0")
    L = _lib.lib()
    buf = (ctypes.c_ulonglong * 16)()
    ctrl.solve_batch(b.x0, b.ref, b.u_prev)
    torch.cuda.synchronize()
    _lib.check(L.mpcqp_debug_stamps(buf, 1), "stamps reset")
    ctrl.solve_batch(b.x0, b.ref, b.u_prev)
    torch.cuda.synchronize()
    _lib.check(L.mpcqp_debug_stamps(buf, 0), "stamps read")
    it = ctrl._iters[:B].cpu().numpy()
    out = {NAMES[k]: int(buf[k]) / B for k in NAMES}
    out["per_call"] = {
        "admm.form": out["admm.form"] / max(1e-9, it[:, 2].mean() - it[:, 1].mean()),
        "admm.iteration": out["admm.iteration"] / max(1e-9, it[:, 0].mean()),
        "polish.sweep": out["polish.sweep"] / max(1e-9, it[:, 1].mean()),
        "admm.sweep": out["admm.sweep"] / max(1e-9, it[:, 2].mean() - it[:, 1].mean()),
    }
    out["iters_mean"] = it.mean(axis=0).round(2).tolist()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
