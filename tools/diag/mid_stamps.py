"""Development tool: per-phase cycles of the mid-horizon kernel (-DMPCQP_MID_STAMPS build).

    python tools/diag/mid_stamps.py build          # here, on the CPU: tools/diag/libmpcqp_midstamps.so
    python tools/diag/mid_stamps.py run 32 40 63   # on the GPU box

Thread 0 of each QP stamps s_memtime around the phases; the sums are per-QP averages (cycles).
"""
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
DIAG = ROOT / "tools" / "diag"
LIB = DIAG / "libmpcqp_midstamps.so"
PHASES = ["setup", "admm_fact", "admm_iter", "admm_check", "polish_fact", "polish_total", "outputs", "qp_total"]
# the setup's sub-phases (slots 9..14 of the stamp buffer)
SETUP = {9: "s_prefix_free_response", 10: "s_condense", 11: "s_input_band_rowmax", 12: "s_ruiz",
         13: "s_pbar_store", 14: "s_rest",
         16: "p_ballot_rank1", 17: "p_solve", 18: "p_refine", 19: "p_line_search", 20: "p_step"}


def build():
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as g

    g.HIPCC_FLAGS = g.HIPCC_FLAGS + ["-DMPCQP_MID_STAMPS"]
    g.OBJ_DIR = DIAG / "obj_midstamps"
    g.LIB = LIB
    g.library_build_id.__defaults__ = (LIB,)  # its default was bound to the product library
    g.RESOURCES = DIAG / "obj_midstamps" / "resources.json"
    g.build_library()
    print("built", LIB)


def run(Ns):
    os.environ.setdefault("MPCQP_LIB", str(LIB))
    sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))
    import torch
    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    L = ctypes.CDLL(os.environ["MPCQP_LIB"])
    out = {}
    for N in Ns:
        b = scenarios.config3(4096, horizon=N)
        ctrl = BatchedMPCController(MPCConfig(horizon=N).to_parameters(0.8), 4096, device="cuda:0")
        buf = (ctypes.c_ulonglong * 24)()
        nt = 32 if N <= 32 else (40 if N <= 40 else (48 if N <= 48 else (56 if N <= 56 else 64)))
        fn = getattr(L, f"mpcqp_debug_mid_stamps_{nt}")
        ctrl.solve_batch(b.x0, b.ref, b.u_prev)
        torch.cuda.synchronize()
        fn(buf, 1)
        ctrl.solve_batch(b.x0, b.ref, b.u_prev)
        torch.cuda.synchronize()
        fn(buf, 1)
        q = max(1, buf[8])
        it = ctrl._iters[:4096].cpu().numpy().mean(axis=0).tolist()
        out[f"N{N}"] = {"qps": q, **{k: buf[i] / q for i, k in enumerate(PHASES)},
                        **{k: buf[i] / q for i, k in SETUP.items()}, "iters_mean": it}
        ctrl.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run([int(a) for a in sys.argv[2:]])
