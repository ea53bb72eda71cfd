import sys, numpy as np
sys.path.insert(0, "rrt-mpc_amd")
from mpcqp.planning.rrt_star import BatchedRRTStarPlanner, default_planner_parameters
g = np.load("tests/golden/planning.npz")
k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
sx, sy, gx, gy, seed, iters = g[f"rrt{k}_case"]
pl = BatchedRRTStarPlanner(g["rrt_occupancy"], default_planner_parameters(max_iterations=int(iters)), device="cuda:0")
nodes, count, meta = (t.cpu().numpy() for t in pl.grow([(sx, sy)], [(gx, gy)], [int(seed)]))
np.savez("gpurun_out/dbg_rrt.npz", nodes=nodes[0, :count[0]], meta=meta[0])
