#!/usr/bin/env python3
"""Fold rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, TCC_EA0_*REQ, SQ_*) into profiles/pmc_traffic.json.

    python tools/pmc_traffic.py gpurun_out --N 20 --B 4096 > profiles/pmc_traffic.json

Units and corrections (MI355X_MICROARCH.md, HBM section):
  * FETCH_SIZE / WRITE_SIZE are in KiB (FETCH_SIZE = TCC_EA0_RDREQ x 64 B / 1024, checked
    against the TCC_EA0_RDREQ_sum pass);
  * gfx950 FETCH_SIZE reports 1/2 of the bytes of wide streaming reads: the read side is
    doubled (an upper bound for this kernel's 8-byte-per-lane reads; k_build, whose read
    bytes are known exactly, calibrates that access width and is reported beside it);
  * WRITE_SIZE is taken as is.
k_solve = the fused solve kernel (one dispatch per mpcqp_solve call).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import sys
from pathlib import Path

SOLVE = ("k_solve",)


def per_kernel(path: Path, N: int) -> dict:
    """Mean counter value per (kernel, counter); k_solve = k_solve<N> only (bench.py also runs the
    config-1 loop's B=1 k_solve<10> launches, which must not dilute the averages)."""
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        short = "k_solve" if f"k_solve<{N}>" in name else ("k_build" if "k_build" in name else None)
        if short:
            acc[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def measurement_keys(N: int, sets: list) -> dict:
    """bench.settings_key / bench.lib_key of the measured run (run this with the .so the passes ran)."""
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "rrt-mpc_amd")]
    import bench
    from mpcqp import _lib
    from mpcqp.config import MPCConfig

    extra = {}
    for kv in sets:
        k, v = kv.split("=", 1)
        extra[k] = float(v) if "." in v or "e" in v else int(v)
    cp = _lib.to_c_params(MPCConfig(horizon=N).to_parameters(0.8), **extra)
    return {"settings_key": bench.settings_key(cp), "lib_key": bench.lib_key(),
            "solver_settings": bench.solver_settings(cp)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("out_dir")
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="solver settings the passes ran with (bench.py --set), default: the library's")
    a = ap.parse_args()
    d = Path(a.out_dir)
    c = {}
    for p in ("pmc_fetch", "pmc_write", "pmc_req", "pmc_sq", "pmc_f64"):
        f = d / p / "run_counter_collection.csv"
        if f.exists():
            c.update(per_kernel(f, a.N))
    kib = 1024.0
    kernels = [k for k in (*SOLVE, "k_build") if (k, "FETCH_SIZE") in c]  # k_build: absent when K1 is fused
    fetch = {k: c[(k, "FETCH_SIZE")] * kib for k in kernels}
    write = {k: c[(k, "WRITE_SIZE")] * kib for k in kernels}
    rdreq = {k: c.get((k, "TCC_EA0_RDREQ_sum")) for k in kernels}
    N, B = a.N, a.B
    build_read_alg = 8.0 * B * (4 * (N + 1) + 6)  # K1's inputs: x0, ref window, u_prev
    out_alg = 8.0 * B * (2 + 4 * (N + 1) + 2 * N) + B * (4 + 16 + 5 * N + 1)  # u0, X, U, status, iters, active
    read = 2.0 * sum(fetch[k] for k in SOLVE)
    wr = sum(write[k] for k in SOLVE)
    out = {
        f"N{N}_B{B}": {
            "k_solve_hbm_bytes_per_launch": read + wr,
            "k_solve_read_bytes_corrected": read,
            "k_solve_write_bytes": wr,
            "per_kernel_fetch_bytes_raw": fetch,
            "per_kernel_write_bytes": write,
            "per_kernel_tcc_ea0_rdreq": rdreq,
            "algorithmic_bytes_per_launch": {"read": build_read_alg, "write": out_alg,
                                             "total": build_read_alg + out_alg},
            "hbm_over_algorithmic": (read + wr) / (build_read_alg + out_alg),
            "per_qp_bytes": (read + wr) / B,
            "note": "FETCH doubled per the gfx950 correction (8-byte-per-lane loads: an upper bound); "
                    + ("K1 separate: k_solve reads the model block per QP; " if "k_build" in fetch else
                       "K1 fused: k_solve reads the inputs (x0, ref window, u_prev) itself; ")
                    + "it writes the outputs; the scaled problem stays on chip",
        }
    }
    sq = {name: v for (k, name), v in c.items() if k == "k_solve" and name.startswith("SQ_")}
    if sq:
        # SQ_WAVE_CYCLES / WAIT_* / ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md constants)
        cyc = sq.get("SQ_WAVE_CYCLES")
        out[f"N{N}_B{B}"]["k_solve_sq"] = {
            "counters_per_launch": sq,
            # SQ_INSTS_VALU_FLOPS_FP64 counts per wave instruction (FMA 2, ADD/MUL/TRANS 1: it equals
            # 2*FMA+ADD+MUL+TRANS below); x64 lanes = executed flops, masked lanes included
            "hw_fp64_flops_per_launch": 64.0 * sq["SQ_INSTS_VALU_FLOPS_FP64"] if "SQ_INSTS_VALU_FLOPS_FP64" in sq else None,
            "wave_cycles_per_wave": 4.0 * cyc / sq["SQ_WAVES"] if cyc and sq.get("SQ_WAVES") else None,
            "frac_wait_any": sq["SQ_WAIT_ANY"] / cyc if cyc and "SQ_WAIT_ANY" in sq else None,
            "frac_wait_inst_any": sq["SQ_WAIT_INST_ANY"] / cyc if cyc and "SQ_WAIT_INST_ANY" in sq else None,
            "frac_active_inst_any": sq["SQ_ACTIVE_INST_ANY"] / cyc if cyc and "SQ_ACTIVE_INST_ANY" in sq else None,
            "f64_valu_insts_per_wave": (sum(sq.get(f"SQ_INSTS_VALU_{o}_F64", 0.0) for o in ("FMA", "ADD", "MUL", "TRANS"))
                                        / sq["SQ_WAVES"]) if sq.get("SQ_WAVES") else None,
            "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / sq["SQ_WAVES"] if sq.get("SQ_WAVES") and "SQ_INSTS_VALU" in sq else None,
        }
    # bench.py attaches this entry to its line only when the run's settings and kernel library match
    out[f"N{N}_B{B}"].update(measurement_keys(N, a.set))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
