"""Development: per-row X error of the mid-horizon kernel against the exact oracle."""
import sys
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

    N = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    b = scenarios.config3(4, horizon=N, seed=300 + N)
    p = MPCConfig(horizon=N).to_parameters(0.8)
    ctrl = BatchedMPCController(p, 4, device="cuda:0")
    sol = ctrl.solve_batch(b.x0, b.ref, b.u_prev)
    torch.cuda.synchronize()
    X = sol.X.cpu().numpy()
    for q in range(4):
        ex = mo.solve_exact(p, b.x0[q], b.ref[q], b.u_prev[q])
        d = np.abs(X[q] - ex.X)
        print(q, "row max err", d.max(axis=1), "first bad col per row", [int(np.argmax(r > 1e-6)) for r in d])
        print("  gpu psi", X[q][2, :6], "\n  ref psi", ex.X[2, :6])
        print("  gpu x", X[q][0, :6], "\n  ref x", ex.X[0, :6])


if __name__ == "__main__":
    main()
