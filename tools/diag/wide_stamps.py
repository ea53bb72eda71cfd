"""Development: per-phase cycles of the long-horizon kernel (tools/diag/libmpcqp_wstamps.so,
-DMPCQP_WIDE_STAMPS): python tools/diag/wide_stamps.py [N] [B]"""
import ctypes, json, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
os.environ.setdefault("MPCQP_LIB", str(ROOT / "tools" / "diag" / "libmpcqp_wstamps.so"))
os.environ.setdefault("MPCQP_ABI_ANY", "1")
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))
import numpy as np
import torch
from mpcqp import _lib, scenarios
from mpcqp.config import MPCConfig
from mpcqp.control.mpc_controller import BatchedMPCController
N = int(sys.argv[1]) if len(sys.argv) > 1 else 32
B = int(sys.argv[2]) if len(sys.argv) > 2 else 512
b = scenarios.config3(B, horizon=N)
ctrl = BatchedMPCController(MPCConfig(horizon=N).to_parameters(0.8), B, device="cuda:0")
ctrl.solve_batch(b.x0, b.ref, b.u_prev)
torch.cuda.synchronize()
L = _lib.lib()
SS = L.mpcqp_state_stride(N)
st = np.zeros((B, SS))
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
assert hip.hipMemcpy(st.ctypes.data, L.mpcqp_state_buffer(ctrl._ws), st.nbytes, 2) == 0
n = 2 * N
off = n * (n + 1)
names = ["setup", "admm.factor", "admm.iteration", "admm.check", "polish.form", "polish.sweep", "polish.solve",
         "polish.linesearch"]
S = st[:, off:off + 8].mean(axis=0)
it = ctrl._iters[:B].cpu().numpy().mean(axis=0)
print(json.dumps({"N": N, "B": B, "cycles_per_qp": dict(zip(names, S.round().tolist())), "iters_mean": it.tolist(),
                  "total": float(S.sum())}))
