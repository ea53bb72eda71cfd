#!/usr/bin/env python3
"""Development check: scan device assembly for DPP reads of a VGPR written by a VALU
instruction fewer than two wait states earlier (the inline-asm v_fmac_f64_dpp broadcasts
are invisible to the compiler's hazard recognizer).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -o /tmp/m.s rrt-mpc_amd/csrc/mpcqp.hip
    python tools/check_dpp_hazards.py /tmp/m.s
"""
import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(tok: str) -> set[int]:
    out = set()
    for m in REG.finditer(tok):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def main(path: str) -> int:
    insts = []
    for line in open(path):
        t = line.split(";")[0].strip()
        if not t or t.endswith(":") or t.startswith("."):
            if t.endswith(":"):
                insts.append(("LABEL", ""))
            continue
        op, _, rest = t.partition(" ")
        insts.append((op, rest))
    bad = 0
    for i, (op, rest) in enumerate(insts):
        if "_dpp" not in op:
            continue
        ops = [o.strip() for o in rest.split(",")]
        src0 = regs(ops[1]) if len(ops) > 1 else set()
        waits = 0
        j = i - 1
        while j >= 0 and waits < 2:
            pop, prest = insts[j]
            if pop == "LABEL":
                break  # conservative: stop at block boundaries
            if pop.startswith("s_nop"):
                waits += int(prest.split()[0]) + 1 if prest else 1
                j -= 1
                continue
            if pop.startswith("v_"):
                dst = regs(prest.split(",")[0])
                if dst & src0:
                    bad += 1
                    print(f"hazard: inst {i} {op} {rest} <- {pop} {prest} ({waits} waits)")
                    break
            waits += 1
            j -= 1
    print(f"{sum(1 for o, _ in insts if '_dpp' in o)} dpp instructions, {bad} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
