#!/usr/bin/env python3
"""Diagnostic: does a resident B=1 server wave (mpcqp_solve_served) hold up work on other streams?
Times how long ops on fresh default-priority torch streams take to complete (a) with no server, (b)
with a live idle server, (c) while the closed loop keeps the server busy; streams created before or
after the server starts."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))


def main():
    import torch

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = scenarios.config3(8, horizon=10, seed=3)
    out = {"priority_range": torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else None}
    x = torch.zeros(64, device="cuda:0")
    torch.cuda.synchronize()

    def enqueue(streams, base):
        evs = []
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                x[base + i].add_(1.0)
                e = torch.cuda.Event()
                e.record(s)
                evs.append(e)
        return evs

    def wait(evs, ctrl=None, busy=False, limit=0.1):
        t0 = time.perf_counter()
        done = {}
        q = 0
        while time.perf_counter() - t0 < limit and len(done) < len(evs):
            if busy:
                ctrl.solve_one(b.x0[q % 8], b.ref[q % 8], b.u_prev[q % 8])
                q += 1
            for i, e in enumerate(evs):
                if i not in done and e.query():
                    done[i] = round((time.perf_counter() - t0) * 1e3, 3)
        return {"done_ms": done, "n_done": len(done), "requests": q}

    os.environ["MPCQP_B1_SERVER"] = "1"
    ctrl = BatchedMPCController(MPCConfig(horizon=10).to_parameters(0.8), 1, device="cuda:0")
    pre = [torch.cuda.Stream() for _ in range(8)]
    enqueue(pre, 0)
    torch.cuda.synchronize()
    out["a_no_server"] = wait(enqueue(pre, 0))
    ctrl.solve_one(b.x0[0], b.ref[0], b.u_prev[0])
    out["b_idle_server_pre_streams"] = wait(enqueue(pre, 0))
    ctrl.solve_one(b.x0[0], b.ref[0], b.u_prev[0])
    out["c_busy_server_pre_streams"] = wait(enqueue(pre, 0), ctrl, busy=True)
    ctrl.solve_one(b.x0[0], b.ref[0], b.u_prev[0])
    t = time.perf_counter()
    post = [torch.cuda.Stream() for _ in range(8)]
    out["stream_create_ms"] = round((time.perf_counter() - t) * 1e3, 3)
    out["d_busy_server_new_streams"] = wait(enqueue(post, 8), ctrl, busy=True)
    ctrl.solve_one(b.x0[0], b.ref[0], b.u_prev[0])
    with torch.cuda.stream(torch.cuda.current_stream()):
        out["e_busy_server_default_stream"] = wait(enqueue([torch.cuda.current_stream()], 16), ctrl, busy=True)
    torch.cuda.synchronize()
    ctrl.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
