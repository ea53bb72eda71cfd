#!/usr/bin/env python3
"""Development check for kernel rewrites meant to be bit-identical: solves the same batches with
each library (tools/ablibs/<name>.so, one subprocess each) and compares every output bit for bit.

    python tools/ab_bitwise.py --libs base new --out gpurun_out/bitwise.json
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
CASES = [  # (config, horizon, batch, pairing, settings)
    ("config3", 20, 4096, "auto", {}),
    ("config2", 20, 1024, "auto", {}),
    ("config4", 30, 2048, "auto", {}),
    ("config3", 15, 4096, "on", {}),
    ("config3", 10, 1024, "off", {"polish_from": 25}),
    ("config3", 20, 1024, "auto", {"max_iter": 40, "polish": 0}),
]
MID_CASES = [  # the mid-horizon kernel (N = 33..64)
    ("config3", 33, 1024, "auto", {}),
    ("config3", 40, 1024, "auto", {}),
    ("config3", 48, 512, "auto", {}),
    ("config3", 56, 512, "auto", {}),
    ("config3", 64, 512, "auto", {}),
    ("config3", 40, 512, "auto", {"max_iter": 40, "polish": 0}),
    ("config3", 37, 512, "auto", {}),  # N < NT: padding steps in every bucket
    ("config3", 45, 512, "auto", {}),
    ("config3", 53, 256, "auto", {}),
    ("config3", 61, 256, "auto", {}),
]
if os.environ.get("MPCQP_AB_MID") == "1":
    CASES = MID_CASES


def child(out: str) -> None:
    sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))
    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    res = {}
    for i, (cfg, N, B, pairing, sett) in enumerate(CASES):
        b = getattr(scenarios, cfg)(B, horizon=N)
        ctrl = BatchedMPCController(MPCConfig(horizon=N).to_parameters(0.8), B, device="cuda:0", pairing=pairing,
                                    **sett)
        sol = ctrl.solve_batch(b.x0[:B], b.ref[:B], b.u_prev[:B])
        for k in ("u0", "X", "U", "status", "iters", "active"):
            res[f"{i}_{k}"] = getattr(sol, k).cpu().numpy()
        ctrl.close()
    np.savez(out, **res)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs=2, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--child", default=None)
    ap.add_argument("--mid", action="store_true", help="the mid-horizon cases (N = 33..64) instead")
    a = ap.parse_args()
    if a.mid:
        os.environ["MPCQP_AB_MID"] = "1"
    if a.child:
        child(a.child)
        return
    outs = []
    with tempfile.TemporaryDirectory() as d:
        for lib in a.libs:
            f = os.path.join(d, f"{lib}.npz")
            env = dict(os.environ, MPCQP_LIB=str(ROOT / "tools" / "ablibs" / f"{lib}.so"), MPCQP_ABI_ANY="1")
            subprocess.run([sys.executable, __file__, "--libs", *a.libs, "--out", a.out, "--child", f], env=env,
                           check=True, timeout=300)
            outs.append(dict(np.load(f)))
    rep = {}
    for k in outs[0]:
        x, y = outs[0][k], outs[1][k]
        same = x.shape == y.shape and np.array_equal(x.view(np.uint8), y.view(np.uint8))
        rep[k] = {"bitwise_equal": bool(same)}
        if not same and x.dtype.kind == "f":
            rep[k]["max_abs_diff"] = float(np.nanmax(np.abs(x - y)))
    summary = {"cases": [list(map(str, c)) for c in CASES], "all_equal": all(v["bitwise_equal"] for v in rep.values()),
               "fields": rep}
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(summary, indent=1))
    print(json.dumps({"all_equal": summary["all_equal"],
                      "differ": [k for k, v in rep.items() if not v["bitwise_equal"]]}))


if __name__ == "__main__":
    main()
