#!/usr/bin/env python3
"""Development tool: per-phase cycle attribution from the -DMPCQP_STAMPS diagnostic build.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DMPCQP_STAMPS -DMPCQP_ONLY_N=20 \
        -o tools/diag/libmpcqp_stamps.so rrt-mpc_amd/csrc/mpcqp.hip rrt-mpc_amd/csrc/mpcqp_fleet.hip
    python tools/stamps.py [config] [--worst K]

--worst K: replicate the K-th slowest QP (by ADMM iterations) over the batch, so the per-QP
averages are that QP's own breakdown (the tail that sets the kernel's latency).

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
os.environ.setdefault("MPCQP_LIB", str(ROOT / "tools" / "diag" / "libmpcqp_stamps.so"))
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))

NAMES = {0: "admm.form", 1: "admm.sweep", 2: "admm.iteration", 3: "admm.check", 4: "admm.total",
         8: "polish.form", 9: "polish.sweep", 10: "polish.solve", 11: "polish.linesearch", 12: "polish.total",
         13: "finish.outputs", 22: "qp.total",
         16: "setup.load_prefix", 17: "setup.condense", 18: "setup.unscaled", 19: "setup.ruiz", 20: "setup.write",
         21: "setup.total", 26: "setup.write.finite_model", 27: "setup.write.pbar", 28: "setup.write.context"}


def main() -> None:
    import torch

    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="config3")
    ap.add_argument("--worst", type=int, default=-1)
    ap.add_argument("--by", type=int, default=0, help="iteration counter ranking --worst (0 ADMM, 1 polish)")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--horizon", type=int, default=0, help="the config's generator at another horizon")
    ap.add_argument("--polish-from", type=int, default=None, help="solver setting polish_from (default: library's)")
    a = ap.parse_args()
    b = getattr(scenarios, a.config)(**({"horizon": a.horizon} if a.horizon else {}))
    x0, ref, up = b.x0, b.ref, b.u_prev
    B = a.batch or b.size
    extra = {} if a.polish_from is None else {"polish_from": a.polish_from}
    ctrl = BatchedMPCController(MPCConfig(horizon=b.horizon).to_parameters(0.8), max(B, b.size), device="cuda:0",
                                **extra)
    L = _lib.lib()
    buf = (ctypes.c_ulonglong * 32)()
    ctrl.solve_batch(x0, ref, up)
    torch.cuda.synchronize()
    if a.worst >= 0:
        order = np.argsort(-ctrl._iters[: b.size, a.by].cpu().numpy(), kind="stable")
        q = int(order[a.worst])
        x0, ref, up = (np.repeat(v[q:q + 1], B, axis=0) for v in (x0, ref, up))
    else:
        x0, ref, up = x0[:B], ref[:B], up[:B]
    ctrl.solve_batch(x0, ref, up)
    torch.cuda.synchronize()
    _lib.check(L.mpcqp_debug_stamps(buf, 1), "stamps reset")
    ctrl.solve_batch(x0, ref, up)
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
