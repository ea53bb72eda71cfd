#!/usr/bin/env python3
"""Static + dynamic instruction-class breakdown of k_solve<N> by solver phase.

The solver marks where each phase begins (MPCQP_MARK, compiled in only with -DMPCQP_PHASE_MARKS):

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on --cuda-device-only -S -DMPCQP_PHASE_MARKS \\
        -DMPCQP_PART_LO=20 -DMPCQP_PART_HI=20 -o /tmp/p20m.s rrt-mpc_amd/csrc/mpcqp_part.hip
    python tools/isa_breakdown.py /tmp/p20m.s --work profiles/r04_s2_qp_cycles.json [--pmc profiles/pmc_traffic.json]

Every instruction of the kernel's assembly is attributed to the last mark before it in the text (the
compiler lays the blocks out in source order here; the marks are empty asm statements, so the code
generated between them is the product kernel's).  Each phase's static counts are then weighted by how
often the phase runs per QP (the kernel's own counters: ADMM iterations, termination checks, ADMM
factorizations, polish passes, full polish factorizations, rank-1 updates, line-search trials), which
gives the dynamic instruction mix per QP; the total is checked against the PMC pass's per-wave VALU count.
"""
from __future__ import annotations

import argparse
import collections
import json
import re


def classify(op: str) -> str:
    if op.startswith("v_"):
        if "f64" in op:
            return "f64"
        if op.startswith("v_permlane"):
            return "v_permlane"
        if "_dpp" in op and op.startswith("v_mov"):
            return "v_mov_dpp"
        if op.startswith("v_mov"):
            return "v_mov"
        if op.startswith("v_cndmask"):
            return "v_cndmask"
        if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            return "v_readlane"
        if op.startswith("v_cmp"):
            return "v_cmp"
        return "v_other"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    return "vmem"


VALU_NON_F64 = ("v_permlane", "v_mov_dpp", "v_mov", "v_cndmask", "v_readlane", "v_cmp", "v_other")


def parse(path: str, kernel: str) -> dict:
    text = open(path).read().split("\n")
    start = next(i for i, l in enumerate(text) if re.match(rf"^_ZN12_GLOBAL__N_1{kernel}", l))
    end = next(i for i in range(start + 1, len(text)) if text[i].startswith(".Lfunc_end"))
    phase = "entry"
    out: dict = collections.defaultdict(collections.Counter)
    for l in text[start:end]:
        m = re.search(r";@phase (\S+)", l)
        if m:
            phase = m.group(1)
            continue
        t = l.split(";")[0].strip()
        if not t or t.endswith(":") or t.startswith("."):
            continue
        out[phase][classify(t.split()[0])] += 1
    return out


def weights(work: dict, N: int) -> dict:
    """Executions per QP of each phase, from the kernel's mean work counters.  A rank-1 update reads
    three columns of the inverse through pick<>'s tree of uniform branches."""
    w = work["work_means"]
    passes = w["polish_pass"]
    return {
        "entry": 1.0, "ctl": 1.0, "outputs": 1.0,
        "setup.k1": 1.0, "setup.prefix": 1.0, "setup.condense": 1.0, "setup.band": 1.0, "setup.unscaled": 1.0,
        # the full-Q condensing runs only for non-diagonal Q / Q_N (the default parameters are diagonal)
        "setup.condense_full_q": 0.0, "setup.gcol": 1.0,
        "setup.ruiz": 1.0, "setup.write": 1.0,
        "admm.form": w["admm_factorization"], "admm.sweep": w["admm_factorization"],
        "admm.fctl": w["admm_factorization"],
        "admm.iter": w["admm_it"], "admm.check": w["check"],
        # the rank-1 update is inlined once per soft-row slot (3 copies, one runs per update); each
        # copy reads three inverse columns through pick<>'s uniform branch tree, one leaf of ceil(n/2)
        "pol.ctl": passes, "pol.rank1": w["rank1_update"] / 3.0,
        "pol.pick_leaf": w["rank1_update"] / (3.0 * ((2 * N + 1) // 2)),
        "pol.form": w["polish_full_factorization"], "pol.sweep": w["polish_full_factorization"],
        "pol.solve": passes, "pol.refine": w["polish_full_factorization"],
        "pol.ls": max(0.0, passes - w["polish_full_factorization"]), "pol.lstrial": w["ls_trial"],
        "pol.lsend": max(0.0, passes - w["polish_full_factorization"]),
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="7k_solveILi20E")
    ap.add_argument("--work", required=True, help="qp_cycles.py output (work_means of the batch)")
    ap.add_argument("--which", default="full")
    ap.add_argument("--pmc", default=None, help="pmc_traffic.json: compare with SQ_INSTS_VALU per wave")
    ap.add_argument("--pmc-key", default="N20_B4096")
    a = ap.parse_args()
    stat = parse(a.asm, a.kernel)
    N = int(re.search(r"ILi(\d+)E", a.kernel).group(1))
    W = weights(json.load(open(a.work))[a.which], N)
    classes = ["f64", *VALU_NON_F64, "salu", "s_nop", "s_waitcnt", "lds", "vmem"]
    rows = {}
    tot = collections.Counter()
    for ph, c in sorted(stat.items()):
        wgt = W.get(ph, 1.0)
        dyn = {k: c[k] * wgt for k in classes}
        rows[ph] = {"per_qp_executions": round(wgt, 3), "static": {k: c[k] for k in classes if c[k]},
                    "dynamic": {k: round(v, 1) for k, v in dyn.items() if v}}
        tot.update(dyn)
    valu = sum(tot[k] for k in ("f64", *VALU_NON_F64))
    out = {"phases": rows,
           "dynamic_per_qp": {k: round(tot[k], 1) for k in classes},
           "valu_per_qp": round(valu, 1), "non_f64_valu_per_qp": round(valu - tot["f64"], 1)}
    if a.pmc:
        sq = json.load(open(a.pmc))[a.pmc_key]["k_solve_sq"]
        out["pmc"] = {"valu_insts_per_wave": sq["valu_insts_per_wave"], "f64_valu_insts_per_wave": sq["f64_valu_insts_per_wave"],
                      "non_f64": sq["valu_insts_per_wave"] - sq["f64_valu_insts_per_wave"],
                      "model_over_pmc_valu": round(valu / sq["valu_insts_per_wave"], 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
