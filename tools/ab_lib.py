#!/usr/bin/env python3
"""Development A/B libraries: the library of the last full build (build/obj) with the solver objects of a
few horizon groups recompiled from the current sources, so a kernel change can be timed against the
previous code on the same GPU box without a full rebuild.

    python tools/ab_lib.py base               # tools/ablibs/base.so: build/obj as it is
    python tools/ab_lib.py new --parts 20 30  # tools/ablibs/new.so: part_20_20, part_30_30 recompiled
    MPCQP_LIB=tools/ablibs/new.so MPCQP_ABI_ANY=1 python bench.py ...
"""
from __future__ import annotations

import argparse
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    import __graft_entry__ as g

    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--parts", type=int, nargs="*", default=[], help="horizons whose part objects to recompile")
    ap.add_argument("--define", action="append", default=[], help="extra -D for the recompiled objects")
    ap.add_argument("--sources", nargs="*", default=[],
                    help="also recompile the objects of these source files (e.g. mpcqp.hip for a stamps build)")
    a = ap.parse_args()
    hipcc = "/opt/rocm/bin/hipcc"
    cmds = g._compile_jobs(hipcc)
    odir = ROOT / "tools" / "ablibs" / f"obj_{a.name}"
    odir.mkdir(parents=True, exist_ok=True)
    objs, jobs = [], []
    for c in cmds:
        obj = c[c.index("-o") + 1]
        lo = next((int(x.split("=")[1]) for x in c if x.startswith("-DMPCQP_PART_LO=")), None)
        hi = next((int(x.split("=")[1]) for x in c if x.startswith("-DMPCQP_PART_HI=")), None)
        src = any(x.endswith(tuple("/" + f for f in a.sources)) for x in c) if a.sources else False
        if src or (lo is not None and any(lo <= n <= hi for n in a.parts)):
            new = odir / Path(obj).name
            c2 = list(c)
            c2[c2.index("-o") + 1] = str(new)
            c2 = c2[:1] + [f"-D{d}" for d in a.define] + c2[1:]
            jobs.append(c2)
            objs.append(str(new))
        else:
            objs.append(obj)
    with ThreadPoolExecutor(8) as ex:
        for r in ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs):
            if r.returncode:
                raise SystemExit(r.stderr)
    objs.append(str(ROOT / "build" / "obj" / "build_id.o"))
    out = ROOT / "tools" / "ablibs" / f"{a.name}.so"
    subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(out), *objs], check=True)
    print(out)


if __name__ == "__main__":
    main()
