#!/usr/bin/env python3
"""Development probe: the shader clock a lone QP runs at.  One QP per launch (B = 1) and a
one-wave-per-SIMD batch (config 2, B = 1024), each with debug_state, so the wave writes its own
s_memtime cycles start to finish (qp_cycles.py); the launch is timed with HIP events on its stream.
cycles / event time is a lower bound of the clock (the event pair also holds the launch).

    python tools/diag/b1_clock.py > gpurun_out/b1_clock.json
"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))


def probe(N: int, B: int, reps: int, polish_from: int | None) -> dict:
    import torch

    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = scenarios.config2(B, horizon=N) if B > 1 else scenarios.config3(64, horizon=N)
    x0, ref, up = b.x0[:B], b.ref[:B], b.u_prev[:B]
    extra = {} if polish_from is None else {"polish_from": polish_from}
    ctrl = BatchedMPCController(MPCConfig(horizon=N).to_parameters(0.8), B, device="cuda:0", debug_state=1, **extra)
    L = _lib.lib()
    SS = L.mpcqp_state_stride(N)
    off = (4 * N * N + 7) // 8 * 8 + 15 * 64 + 4
    st = torch.empty((B, SS), dtype=torch.float64, device="cuda:0")
    hip = ctypes.CDLL("libamdhip64.so")
    for _ in range(20):
        ctrl.solve_batch(x0, ref, up)
    torch.cuda.synchronize()
    ms, cyc = [], []
    s = torch.cuda.current_stream()
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        ctrl.solve_batch(x0, ref, up)
        e1.record(s)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
        hip.hipMemcpy(ctypes.c_void_p(st.data_ptr()), ctypes.c_void_p(L.mpcqp_state_buffer(ctrl._ws)),
                      ctypes.c_size_t(B * SS * 8), 3)
        torch.cuda.synchronize()
        cyc.append(float(st[:, off].max().item()))
    ms, cyc = np.array(ms), np.array(cyc)
    ctrl.close()
    return {"N": N, "B": B, "polish_from": polish_from, "event_us_median": float(np.median(ms) * 1e3),
            "cycles_max_wave_median": float(np.median(cyc)),
            "clock_ghz_lower_bound": float(np.median(cyc / (ms * 1e-3)) / 1e9)}


def main() -> None:
    out = [probe(10, 1, 100, 25), probe(10, 1, 100, None), probe(20, 1, 100, None), probe(20, 1024, 50, None)]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
