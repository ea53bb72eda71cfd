"""The headline kernel's time per step from a cold process: how many steps (and how many ms of
GPU work) the MI355X takes to reach its sustained clock.  Every step is bracketed by its own
event pair; prints the per-step times binned by 10 steps, and the same after 2 s idle."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "rrt-mpc_amd"))
import bench  # noqa: E402
from mpcqp import _lib  # noqa: E402
from mpcqp.config import MPCConfig  # noqa: E402
from mpcqp.control.mpc_controller import BatchedMPCController  # noqa: E402


def run(ctrl, B, x0, ref, up, steps):
    L = _lib.lib()
    st = torch.cuda.current_stream()
    s = ctypes.c_void_p(st.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for k in range(steps):
        ev[k][0].record(st)
        _lib.check(L.mpcqp_build(ctrl._ws, B, x0.data_ptr(), ref.data_ptr(), up.data_ptr(), s), "build")
        _lib.check(L.mpcqp_solve(ctrl._ws, B, ctrl._u0.data_ptr(), ctrl._X.data_ptr(), ctrl._U.data_ptr(),
                                 ctrl._status.data_ptr(), ctrl._iters.data_ptr(), ctrl._active.data_ptr(), s),
                   "solve")
        ev[k][1].record(st)
    torch.cuda.synchronize()
    t = np.array([a.elapsed_time(b) for a, b in ev]) * 1e3
    return [round(float(x), 1) for x in t.reshape(-1, 10).mean(axis=1)]


def main():
    B = 4096
    batch = bench.make_global_batch("config3", B, 0)
    params = MPCConfig(horizon=batch.horizon).to_parameters(0.8)
    ctrl = BatchedMPCController(params, B, device="cuda:0")
    x0 = torch.from_numpy(batch.x0).cuda()
    ref = torch.from_numpy(batch.ref).cuda()
    up = torch.from_numpy(batch.u_prev).cuda()
    out = {"cold_us_per_10": run(ctrl, B, x0, ref, up, 400)}
    time.sleep(2.0)
    out["after_2s_idle_us_per_10"] = run(ctrl, B, x0, ref, up, 200)
    time.sleep(0.2)
    out["after_200ms_idle_us_per_10"] = run(ctrl, B, x0, ref, up, 100)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
