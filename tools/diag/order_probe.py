#!/usr/bin/env python3
"""Development probe: how much of k_solve's time is dispatch packing (the tail), not work.

Times k_solve (HIP events, median of 9) on config 3 at several batch sizes and in three orders of
the same 4096 QPs: as generated, sorted by the QP's own cost (longest first, from the kernel's
iteration counters of a first solve: an oracle ordering, not something the product can know) and
shortest first.  gpurun -- 'python tools/diag/order_probe.py > gpurun_out/order_probe.json'
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))


def main() -> None:
    import torch

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = scenarios.config3(4096)
    ctrl = BatchedMPCController(MPCConfig(horizon=20).to_parameters(0.8), 4096, device="cuda:0")
    dev = torch.device("cuda:0")
    x0 = torch.from_numpy(b.x0).to(dev)
    ref = torch.from_numpy(b.ref).to(dev)
    up = torch.from_numpy(b.u_prev).to(dev)

    def timed(x, r, u, reps=9):
        ts = []
        for _ in range(reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ctrl.solve_batch(x, r, u)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts[2:]))

    out = {}
    sol = ctrl.solve_batch(x0, ref, up)
    torch.cuda.synchronize()
    it = sol.iters.cpu().numpy().astype(float)
    # per-QP lone-cycle model of tools/qp_cycles.py (profiles/r01_s9_qp_cycles.txt)
    cost = 79334 + 1087 * it[:, 0] + 23912 * it[:, 2] - 19049 * it[:, 1] + 1494 * it[:, 3]
    for B in (256, 512, 1024, 1536, 2048, 2560, 3072, 4096):
        out[f"B{B}"] = timed(x0[:B], ref[:B], up[:B])
    for name, idx in (("longest_first", np.argsort(-cost, kind="stable")),
                      ("shortest_first", np.argsort(cost, kind="stable")),
                      ("interleaved", np.argsort(-cost, kind="stable").reshape(2, -1).T.reshape(-1))):
        t = torch.from_numpy(idx).to(dev)
        out[f"B4096_{name}"] = timed(x0[t].contiguous(), ref[t].contiguous(), up[t].contiguous())
    out["B4096_asis"] = timed(x0, ref, up)
    out["cost_model"] = {"mean": float(cost.mean()), "max": float(cost.max())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
