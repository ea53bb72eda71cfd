"""Development: one QP at very long horizons through MPCController.solve, timed, checked against
the exact oracle.  python tools/diag/huge_horizon.py N [N ...]"""
import json, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rrt-mpc_amd")); sys.path.insert(0, str(ROOT / "oracle"))
import numpy as np
from mpcqp import scenarios
from mpcqp.config import MPCConfig
from mpcqp.control.mpc_controller import MPCController
import mpc_oracle as mo
for N in [int(a) for a in sys.argv[1:]]:
    b = scenarios.config3(1, horizon=N, seed=5)
    params = MPCConfig(horizon=N).to_parameters(0.8)
    ctrl = MPCController(params)
    ctrl.solve(b.x0[0], b.ref[0], u_prev=b.u_prev[0])  # workspace + first launch
    t = time.perf_counter()
    u0, X, U = ctrl.solve(b.x0[0], b.ref[0], u_prev=b.u_prev[0])
    dt = time.perf_counter() - t
    t = time.perf_counter()
    ex = mo.solve_exact(params, b.x0[0], b.ref[0], b.u_prev[0])
    dto = time.perf_counter() - t
    err = float(np.abs(U - ex.Umat).max() / max(1.0, np.abs(ex.Umat).max())) if U is not None else None
    print(json.dumps({"N": N, "gpu_s": dt, "oracle_numpy_s": dto, "rel_err_U": err}), flush=True)
