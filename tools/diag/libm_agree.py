"""Development tool: how often the device's double-precision cos / sin / atan2 / hypot (torch's
kernels call the ROCm device library) equal the host's (Python's math: glibc, and CPython's own
hypot) bit for bit -- the RRT* steer and the segment-sample counts depend on the last ulp.

    python tools/diag/libm_agree.py     # on the GPU box
"""
import json
import math

import numpy as np
import torch


def main():
    rng = np.random.default_rng(5)
    n = 200000
    th = rng.uniform(-math.pi, math.pi, n)
    y = rng.uniform(-80, 80, n)
    x = rng.uniform(-80, 80, n)
    # the steer's own pattern: nx = X + 3 cos(atan2(sy - Y, sx - X)), then hypot(nx - X, ny - Y)
    X = rng.uniform(0, 80, n)
    Y = rng.uniform(0, 80, n)
    d = torch.device("cuda:0")
    tt, ty, tx = (torch.from_numpy(a).to(d) for a in (th, y, x))
    out = {}
    out["cos"] = int((torch.cos(tt).cpu().numpy() != np.array([math.cos(v) for v in th])).sum())
    out["sin"] = int((torch.sin(tt).cpu().numpy() != np.array([math.sin(v) for v in th])).sum())
    out["atan2"] = int((torch.atan2(ty, tx).cpu().numpy() != np.array([math.atan2(a, b) for a, b in zip(y, x)])).sum())
    out["hypot"] = int((torch.hypot(tx, ty).cpu().numpy() != np.array([math.hypot(b, a) for a, b in zip(y, x)])).sum())
    a = np.arctan2(y, x)
    nx = X + 3.0 * np.cos(a)
    ny = Y + 3.0 * np.sin(a)
    host = np.array([math.hypot(p - q, r - s) for p, q, r, s in zip(nx, X, ny, Y)])
    dev = torch.hypot(torch.from_numpy(nx - X).to(d), torch.from_numpy(ny - Y).to(d)).cpu().numpy()
    out["hypot_steer"] = int((dev != host).sum())
    out["n"] = n
    print(json.dumps(out))


if __name__ == "__main__":
    main()
