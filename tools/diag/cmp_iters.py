import sys, numpy as np
sys.path.insert(0, "rrt-mpc_amd"); sys.path.insert(0, "oracle")
import torch, cpu_solver
from mpcqp import scenarios
from mpcqp.config import MPCConfig
from mpcqp.control.mpc_controller import BatchedMPCController
b = scenarios.config3(512)
p = MPCConfig(horizon=20).to_parameters(0.8)
c = BatchedMPCController(p, 512, device="cuda:0")
s = c.solve_batch(b.x0, b.ref, b.u_prev); torch.cuda.synchronize()
g = s.iters.cpu().numpy()
r = cpu_solver.cpu_solve(p, b.x0, b.ref, b.u_prev)["iters"]
for k in range(4): print(k, (g[:, k] == r[:, k]).mean())
bad = np.flatnonzero((g != r).any(axis=1))[:10]
print(np.column_stack([g[bad], r[bad]]))
