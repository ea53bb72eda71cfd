#!/usr/bin/env python3
"""Consecutive batches overlapped on S streams (each stream its own workspace and output buffers):
the headline batch (config 3, B = 4096, N = 20) solved K times with step k on stream k % S, so a
batch's dispatch tail (its slowest QPs) overlaps the next batch's start.  Reported
beside the bench line, not as it: each step is still one whole batch, but S batches are in flight.

    python tools/pipelined.py [--streams 1 2 3] [--steps 40]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "rrt-mpc_amd"), str(ROOT)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--config", default="config3")
    ap.add_argument("--batch", type=int, default=4096)
    a = ap.parse_args()
    import torch

    import bench
    from mpcqp import _lib
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = bench.make_global_batch(a.config, a.batch)
    dev = torch.device("cuda:0")
    params = MPCConfig(horizon=b.horizon).to_parameters(0.8)
    x0_t, ref_t, up_t = (torch.from_numpy(v).to(dev) for v in (b.x0, b.ref, b.u_prev))
    L = _lib.lib()
    out = []
    for S in a.streams:
        ctrls = [BatchedMPCController(params, a.batch, device=dev) for _ in range(S)]
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        B = a.batch

        def step(k):
            c, st = ctrls[k % S], streams[k % S]
            s = ctypes.c_void_p(st.cuda_stream)
            _lib.check(L.mpcqp_build(c._ws, B, x0_t.data_ptr(), ref_t.data_ptr(), up_t.data_ptr(), s), "build")
            _lib.check(L.mpcqp_solve(c._ws, B, c._u0.data_ptr(), c._X.data_ptr(), c._U.data_ptr(), c._status.data_ptr(),
                                     c._iters.data_ptr(), c._active.data_ptr(), s), "solve")

        for k in range(3 * S):
            step(k)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(a.steps):
            step(k)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        solved = sum(int((c._status[:B] == 1).sum().item()) for c in ctrls) / S
        same = all(torch.equal(ctrls[0]._U[:B], c._U[:B]) for c in ctrls[1:])
        out.append({"streams": S, "steps": a.steps, "batch": B, "QP_per_s": solved * a.steps / dt,
                    "ms_per_step": 1e3 * dt / a.steps, "identical_results_across_streams": bool(same)})
        print(json.dumps(out[-1]), file=sys.stderr, flush=True)
        for c in ctrls:
            c.close()
    print(json.dumps({"workload": f"{a.config} B={a.batch}", "runs": out}, indent=1))


if __name__ == "__main__":
    main()
