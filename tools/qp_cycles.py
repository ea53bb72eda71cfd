#!/usr/bin/env python3
"""Development tool: per-QP wave cycles (s_memtime, start to finish, written with debug_state)
against the QP's own work counters, fitted as cycles ~ c0 + c1*ADMM its + c2*factorizations +
c3*checks + ... (polish factorizations, rank-1 updates, passes, line-search trials).  The marginal cost of each unit of work on the
critical path of one wave, at the batch's real occupancy.

    python tools/qp_cycles.py [--batch 4096] [--lone 256]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))


def run(B, stride_pick=1):
    import torch
    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = scenarios.config3(4096)
    idx = np.arange(0, 4096, stride_pick)[:B]
    ctrl = BatchedMPCController(MPCConfig(horizon=20).to_parameters(0.8), B, device="cuda:0", debug_state=1)
    for _ in range(2):
        ctrl.solve_batch(b.x0[idx], b.ref[idx], b.u_prev[idx])
    torch.cuda.synchronize()
    L = _lib.lib()
    SS = L.mpcqp_state_stride(20)
    st = torch.empty((B, SS), dtype=torch.float64, device="cuda:0")
    ptr = L.mpcqp_state_buffer(ctrl._ws)
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy(ctypes.c_void_p(st.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(B * SS * 8), 3)
    cyc = st[:, L.mpcqp_state_stride(20) - 8 + 4].cpu().numpy() if False else None
    off = (4 * 20 * 20 + 7) // 8 * 8 + 15 * 64 + 4
    sc = st[:, off:off + 4].cpu().numpy()  # cycles, polish full factorizations, rank-1 updates, start time
    it = ctrl._iters[:B].cpu().numpy().astype(float)
    return sc, it


def fit(sc, it):
    cyc, full, r1 = sc[:, 0], sc[:, 1], sc[:, 2]
    checks = np.floor(it[:, 0] / 25) + (it[:, 0] % 25 > 0)
    admm_fact = it[:, 2] - it[:, 1]  # nfact counts the ADMM factorizations and every polish pass
    A = np.column_stack([np.ones(len(cyc)), it[:, 0], checks, admm_fact, full, r1, it[:, 1], it[:, 3]])
    coef, *_ = np.linalg.lstsq(A, cyc, rcond=None)
    pred = A @ coef
    names = ["const", "admm_it", "check", "admm_factorization", "polish_full_factorization", "rank1_update",
             "polish_pass", "ls_trial"]
    means = dict(zip(names[1:], A[:, 1:].mean(axis=0).round(3).tolist()))
    share = {n: round(float(c * A[:, i].mean() / cyc.mean()), 3) for i, (n, c) in enumerate(zip(names, coef))}
    return {n: round(float(c)) for n, c in zip(names, coef)}, float(np.corrcoef(pred, cyc)[0, 1]), means, share


def timeline(sc):
    """Occupancy of the batch's waves over the kernel: the span from the first start to the last end
    against the summed wave lifetimes (s_memtime is one clock per XCD; good to a few hundred cycles)."""
    start = sc[:, 3] - sc[:, 3].min()
    end = start + sc[:, 0]
    span = end.max()
    return {"span_cycles": float(span), "sum_wave_cycles": float(sc[:, 0].sum()),
            "last_start": float(start.max()), "end_p50": float(np.percentile(end, 50)),
            "end_p90": float(np.percentile(end, 90)), "end_p99": float(np.percentile(end, 99))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--lone", type=int, default=256)
    a = ap.parse_args()
    out = {}
    for name, B, stride in (("full", a.batch, 1), ("lone", a.lone, 4096 // a.lone)):
        sc, it = run(B, stride)
        cyc = sc[:, 0]
        coef, r, means, share = fit(sc, it)
        w = int(np.argmax(cyc))
        out[name] = {"batch": B, "cycles_mean": float(cyc.mean()), "cycles_max": float(cyc.max()),
                     "p99": float(np.percentile(cyc, 99)), "fit": coef, "fit_r": r, "work_means": means,
                     "cycle_share": share, "timeline": timeline(sc),
                     "slowest_qp_iters": it[w].tolist(), "slowest_qp_work": sc[w, 1:3].tolist(),
                     "slowest_qp_cycles": float(cyc[w])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
