set -o pipefail
mkdir -p gpurun_out
for B in 512 1024 2048 4096 8192 16384; do
  timeout -k 10 120 python bench.py --batch $B --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/sweep_$B.json || exit 1
done
timeout -k 10 120 python - > gpurun_out/iters_hist.json <<'PY'
import sys, json, numpy as np, torch
sys.path.insert(0, "rrt-mpc_amd")
from mpcqp import scenarios
from mpcqp.config import MPCConfig
from mpcqp.control.mpc_controller import BatchedMPCController
b = scenarios.config3(4096)
c = BatchedMPCController(MPCConfig(horizon=20).to_parameters(0.8), 4096, device="cuda:0")
s = c.solve_batch(b.x0, b.ref, b.u_prev); torch.cuda.synchronize()
it = s.iters.cpu().numpy()
out = {}
for i, nm in enumerate(["admm", "polish", "fact", "ls"]):
    out[nm] = {"pct": np.percentile(it[:, i], [50, 90, 99, 99.9, 100]).tolist(), "hist": np.bincount(it[:, i]).tolist() if nm != "ls" else None}
print(json.dumps(out))
PY
