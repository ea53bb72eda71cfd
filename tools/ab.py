#!/usr/bin/env python3
"""Interleaved A/B of kernel libraries on one GPU box (development; tools/ab_lib.py builds them):
each repeat runs every library on config 3 (the headline batch), config 2, the config-4 8-GPU shard
(B = 2048, N = 30) and, with --b1, the B = 1 kernel latency (tools/b1_latency.py), then prints the
per-library means.

    python tools/ab.py --libs base new --reps 2 --out gpurun_out/ab
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HEAD = ["--cpu-seconds", "0", "--no-config1", "--no-config5", "--no-osqp-settings", "--no-pipelined", "--no-strong"]
LEGS = {
    "c3": ["--check-sample", "128"],
    "c2": ["--config", "config2", "--check-sample", "64"],
    "c4_2048": ["--config", "config4", "--batch", "2048", "--check-sample", "64"],
    # lone waves: one QP per CU (256) and a single QP (the kernel event time is the QP's latency)
    "c3_b256": ["--batch", "256", "--check-sample", "64"],
    "c3_b1": ["--batch", "1", "--check-sample", "1"],
    # two QPs per wave (N = 15)
    "pair15": ["--horizon", "15", "--batch", "16384", "--pairing", "on", "--check-sample", "128"],
    "n10_b1": ["--horizon", "10", "--batch", "1", "--polish-from", "25", "--check-sample", "1"],
    "n15_b1024": ["--horizon", "15", "--batch", "1024", "--pairing", "off", "--check-sample", "64"],
    "n10_b1024": ["--horizon", "10", "--batch", "1024", "--pairing", "off", "--check-sample", "64"],
    # a fixed schedule (150 ADMM iterations, no termination check, no polish): per-iteration costs
    # of variants whose iterates differ
    "c3_fixed": ["--set", "max_iter=150", "--set", "polish=0", "--set", "check_termination=1000",
                 "--set", "adaptive_rho=0", "--check-sample", "0"],
    "c3_b1_fixed": ["--batch", "1", "--set", "max_iter=150", "--set", "polish=0", "--set",
                    "check_termination=1000", "--set", "adaptive_rho=0", "--check-sample", "0"],
}


def run(lib: str, args: list, timeout: int = 240) -> dict:
    env = dict(os.environ, MPCQP_LIB=str(ROOT / "tools" / "ablibs" / f"{lib}.so"), MPCQP_ABI_ANY="1")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *HEAD, *args], env=env, capture_output=True,
                       text=True, timeout=timeout)
    if r.returncode:
        raise SystemExit(f"{lib} {args}: rc {r.returncode}\n{r.stderr[-3000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--legs", nargs="*", default=list(LEGS))
    ap.add_argument("--b1", action="store_true")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    res: dict = {}
    for r in range(a.reps):
        for lib in a.libs:
            for leg in a.legs:
                d = run(lib, LEGS[leg])
                re_ = d.get("rel_err") or {"max_rel_err_U": 0.0, "active_set_mismatches": 0, "status_mismatches": 0}
                rec = {"value": d["value"], "k_solve_ms": d["kernel_ms"]["k_solve"], "ms_per_step": d["ms_per_step"],
                       "rel_err": re_["max_rel_err_U"], "iters_agreement": re_.get("iters_agreement"),
                       "mism": re_["active_set_mismatches"] + re_["status_mismatches"],
                       "admm_iters": d["iters_mean"]["admm"], "polish_iters": d["iters_mean"]["polish"]}
                res.setdefault(lib, {}).setdefault(leg, []).append(rec)
                print(lib, leg, r, json.dumps(rec), flush=True)
            if a.b1:
                env = dict(os.environ, MPCQP_LIB=str(ROOT / "tools" / "ablibs" / f"{lib}.so"), MPCQP_ABI_ANY="1")
                p = subprocess.run([sys.executable, str(ROOT / "tools" / "b1_latency.py"), "--calls", "200"], env=env,
                                   capture_output=True, text=True, timeout=240)
                if p.returncode:
                    raise SystemExit(p.stderr[-3000:])
                b = json.loads(p.stdout)
                res.setdefault(lib, {}).setdefault("b1", []).append(b)
                print(lib, "b1", r, json.dumps({k: b[k] for k in b if "us" in k or "ms" in k}), flush=True)
    summary = {}
    for lib, legs in res.items():
        summary[lib] = {}
        for leg, recs in legs.items():
            if leg == "b1":
                summary[lib][leg] = {k: sum(x[k] for x in recs) / len(recs) for k in recs[0] if isinstance(recs[0][k], (int, float))}
            else:
                summary[lib][leg] = {k: sum(x[k] for x in recs) / len(recs) for k in ("value", "k_solve_ms", "ms_per_step", "admm_iters", "polish_iters")}
                summary[lib][leg]["worst_rel_err"] = max(x["rel_err"] for x in recs)
                summary[lib][leg]["mismatches"] = sum(x["mism"] for x in recs)
                summary[lib][leg]["iters_agreement_min"] = min((x["iters_agreement"] or 0) for x in recs)
    (out / "ab.json").write_text(json.dumps({"runs": res, "summary": summary}, indent=1))
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
