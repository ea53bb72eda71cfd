#!/usr/bin/env python3
"""Split a bench.py run's rocprofv3 kernel trace into its legs.  bench.py launches the headline
kernel (k_solve<N>) W + K times, then the pipelined leg (W' + K, two streams), then the OSQP-settings
leg (W + K), all under the same kernel name, so the stats summary's average mixes them; this takes
the dispatches in order and reports each leg's mean, min and max duration.

    python tools/prof_legs.py gpurun_out/f_prof/run_kernel_trace.csv --N 20 --steps 10 --warmup 2
"""
import argparse
import csv
import json

import numpy as np


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if f"k_solve<{a.N}>" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    us = np.array([int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]) / 1e3
    n1 = a.warmup + a.steps
    n2 = max(a.warmup, 2) + a.steps
    legs = {"headline": us[:n1], "pipelined (two streams: overlapping dispatches)": us[n1:n1 + n2],
            "osqp_settings": us[n1 + n2:n1 + n2 + n1]}
    out = {"kernel": f"k_solve<{a.N}>", "dispatches": int(len(us)),
           "legs": {k: {"dispatches": int(len(v)), "mean_us": round(float(v.mean()), 2),
                        "min_us": round(float(v.min()), 2), "max_us": round(float(v.max()), 2)}
                    for k, v in legs.items() if len(v)},
           "vgpr": int(rows[0]["VGPR_Count"]) if rows else None,
           "scratch_bytes": int(rows[0]["Scratch_Size"]) if rows else None,
           "lds_bytes": int(rows[0]["LDS_Block_Size"]) if rows else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
