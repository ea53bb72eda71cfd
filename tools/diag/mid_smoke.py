"""Development: a few QPs through the mid-horizon kernel (N = 32..63) against the exact oracle."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "rrt-mpc_amd"), str(ROOT / "oracle")]


def main():
    import torch
    import mpc_oracle as mo
    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    for N in [int(a) for a in sys.argv[1:]] or [40]:
        b = scenarios.config3(8, horizon=N, seed=300 + N)
        p = MPCConfig(horizon=N).to_parameters(0.8)
        ctrl = BatchedMPCController(p, 8, device="cuda:0")
        t = time.time()
        sol = ctrl.solve_batch(b.x0, b.ref, b.u_prev)
        torch.cuda.synchronize()
        st = sol.status.cpu().numpy()
        U = sol.U.cpu().numpy()
        it = sol.iters.cpu().numpy()
        errs = []
        for q in range(8):
            ex = mo.solve_exact(p, b.x0[q], b.ref[q], b.u_prev[q])
            errs.append(float(np.abs(U[q] - ex.Umat).max() / max(1.0, np.abs(ex.Umat).max())))
        print(f"N={N} status={st.tolist()} iters={it[:, :2].tolist()} max_rel_err={max(errs):.3e} "
              f"t={time.time() - t:.2f}s", flush=True)
        ctrl.close()


if __name__ == "__main__":
    main()
