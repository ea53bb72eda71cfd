"""Dispatch-tail simulation of k_solve on config 3.

Per-QP cycles come from the linear model tools/qp_cycles.py fitted on the kernel's own counters
(mean 245k, max 444k cycles at N=20), evaluated on the C restatement's (oracle/mpcqp_cpu.c)
iteration counters of the same 4096 QPs.  2048 wave slots, two per SIMD; a slot whose SIMD
partner is busy runs at `share` of a lone wave's speed.  `tau`: preemption -- a fresh QP still
running after tau cycles is parked (its remaining work + `ovh` cycles of state write / re-read)
and resumed after every fresh QP has started.

    python tools/tail_sim.py          # host only, ~1 min
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "rrt-mpc_amd"), str(ROOT / "oracle")]
CLOCK_CYCLES_PER_US = 2.4e3


def qp_costs(B=4096, N=20):
    import cpu_solver
    import mpc_oracle as mo
    from mpcqp import scenarios

    b = scenarios.config3(B)
    out = cpu_solver.cpu_solve(mo.default_params(N), b.x0, b.ref, b.u_prev, nthreads=8)
    it = out["iters"].astype(float)
    checks = np.ceil(it[:, 0] / 25)
    return 79334 + 1087 * it[:, 0] + 23912 * it[:, 2] - 19049 * it[:, 1] + 1494 * it[:, 3] + 43 * checks


def simulate(cost, order, slots=2048, share=0.82, tau=None, ovh=70000):
    queue = list(order)[::-1]
    parked = []
    job = [None] * slots
    rem = np.zeros(slots)
    spent = np.zeros(slots)

    def assign(s):
        if queue:
            j = queue.pop()
            job[s], rem[s] = ("fresh", j), cost[j]
        elif parked:
            j, r = parked.pop(0)
            job[s], rem[s] = ("parked", j), r + ovh
        else:
            job[s] = None

    for s in range(slots):
        assign(s)
    t = 0.0
    while any(j is not None for j in job):
        act = np.array([j is not None for j in job])
        pair = act.reshape(-1, 2).sum(1)
        sp = np.where(np.repeat(pair, 2) == 2, share, 1.0) * act
        dt_fin = np.where(act, rem / np.maximum(sp, 1e-9), np.inf)
        dt_park = np.full(slots, np.inf)
        if tau is not None:
            fresh = np.array([j is not None and j[0] == "fresh" for j in job])
            dt_park = np.where(fresh & (rem > 0), np.maximum((tau - spent) / np.maximum(sp, 1e-9), 0), np.inf)
        dt = min(dt_fin.min(), dt_park.min())
        t += dt
        rem -= sp * dt
        spent += sp * dt
        for s in range(slots):
            if job[s] is None:
                continue
            if rem[s] <= 1e-6:
                spent[s] = 0
                assign(s)
            elif tau is not None and job[s][0] == "fresh" and spent[s] >= tau - 1e-6:
                parked.append((job[s][1], rem[s]))
                spent[s] = 0
                assign(s)
    return t / CLOCK_CYCLES_PER_US


def main():
    cost = qp_costs()
    idx = np.arange(len(cost))
    print(f"per-QP cycles: mean {cost.mean():.0f} max {cost.max():.0f} p99 {np.percentile(cost, 99):.0f}")
    print(f"as generated {simulate(cost, idx):.0f} us; longest-first {simulate(cost, np.argsort(-cost)):.0f} us; "
          f"B=2048 {simulate(cost, idx[:2048]):.0f} us")
    for tau in (150e3, 200e3, 250e3, 300e3):
        print(f"preemption tau={tau:.0f}: {simulate(cost, idx, tau=tau):.0f} us")


if __name__ == "__main__":
    main()
