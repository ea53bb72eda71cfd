"""Maximum sizes on the device: batches whose output and workspace buffers pass 2**31 bytes.

A QP's solve reads only its own inputs, so a batch made of R copies of a base batch must give every
copy the base batch's outputs bit for bit (solution, trajectory, status, the four iteration
counters, active set).  That size-independent property checks the 64-bit indexing of every
per-QP buffer at batch sizes the oracle cannot follow: the one-wave kernel at 4.2M QPs (X and the
reference window 2.8 GB each; before the workspace buffers were allocated at first use its
workspace alone held 87 GiB of unused model / state), the mid kernel with a 4.9 GiB state buffer
(its Pbar slots) and the long-horizon kernel with a 5.4 GiB one (its per-QP arenas).  The base batches themselves are held to the
oracle by the parity tests (test_gpu_parity.py, test_gpu_wide.py).
"""
from __future__ import annotations

import pytest

pytestmark = pytest.mark.gpu


def _tiled_equal(cuda, horizon: int, base_batch: int, copies: int, min_bytes: int) -> None:
    import torch
    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = scenarios.config3(base_batch, horizon=horizon, seed=9100 + horizon)
    params = MPCConfig(horizon=horizon).to_parameters(0.8)
    x0 = torch.as_tensor(b.x0, device=cuda)
    ref = torch.as_tensor(b.ref, device=cuda)
    up = torch.as_tensor(b.u_prev, device=cuda)

    ctrl = BatchedMPCController(params, base_batch, device=cuda)
    s = ctrl.solve_batch(x0, ref, up)
    base = {k: getattr(s, k).clone() for k in ("U", "X", "status", "iters", "active")}
    ctrl.close()
    assert bool(((base["status"] == 1) | (base["status"] == 2)).all())  # every base QP solved

    B = base_batch * copies
    big = BatchedMPCController(params, B, device=cuda)
    sol = big.solve_batch(x0.repeat(copies, 1), ref.repeat(copies, 1, 1), up.repeat(copies, 1))
    torch.cuda.synchronize()
    assert sol.X.numel() * sol.X.element_size() >= min_bytes
    for k, v in base.items():
        got = getattr(sol, k).reshape(copies, base_batch, *v.shape[1:])
        same = (got == v.unsqueeze(0)).reshape(copies, -1).all(dim=1)
        bad = torch.nonzero(~same).flatten()[:8].tolist()
        assert not bad, f"{k}: copies {bad} differ from the base batch (B={B}, N={horizon})"
    del sol
    big.close()
    torch.cuda.empty_cache()


def test_workspace_buffers_allocated_at_first_use(cuda):
    """A workspace that runs only the fused one-wave solve holds no model / state buffers (22 KB
    per QP at N = 20); a debug build allocates both, the long-horizon kernels have them from
    mpcqp_create, and the stepped fleet allocates the models before its graph capture."""
    import numpy as np
    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController
    from mpcqp.pipeline.fleet import FleetTracker

    L = _lib.lib()
    b = scenarios.config3(64)
    params = MPCConfig(horizon=20).to_parameters(0.8)
    ctrl = BatchedMPCController(params, 64, device=cuda)
    ctrl.solve_batch(b.x0, b.ref, b.u_prev)
    assert not L.mpcqp_model_buffer(ctrl._ws) and not L.mpcqp_state_buffer(ctrl._ws)
    ctrl.close()
    dbg = BatchedMPCController(params, 64, device=cuda, debug_state=1)
    assert not L.mpcqp_model_buffer(dbg._ws)
    s = dbg.solve_batch(b.x0, b.ref, b.u_prev)
    assert L.mpcqp_model_buffer(dbg._ws) and L.mpcqp_state_buffer(dbg._ws)
    assert int((s.status == 1).sum()) == 64
    dbg.close()
    wide = BatchedMPCController(MPCConfig(horizon=40).to_parameters(0.8), 8, device=cuda)
    assert L.mpcqp_model_buffer(wide._ws) and L.mpcqp_state_buffer(wide._ws)
    wide.close()

    plan = scenarios.load_default_plan()
    mpc = MPCConfig(horizon=10, sim_steps=100)
    ref = {}
    for fused in (False, True):
        ft = FleetTracker(mpc, map_resolution=0.8, max_vehicles=1, max_ref_len=len(plan["path"]) * 8 + 64,
                          device=cuda, fused=fused)
        ft.reset_from_plans([plan["path"]], np.asarray(plan["start"])[None], np.asarray(plan["goal"])[None])
        ref[fused] = np.asarray(ft.run().states[0])
        held = bool(L.mpcqp_model_buffer(ft._nominal._ws))
        assert held == (not fused), fused
        ft.close()
    assert np.array_equal(ref[False], ref[True])


def test_one_wave_kernel_4m_qps(cuda):
    """k_solve<20>: 4,194,304 QPs (1024 copies of a 4096 batch); X is 2.8 GB."""
    _tiled_equal(cuda, 20, 4096, 1024, 2**31)


def test_mid_kernel_past_2gb_workspace(cuda):
    """k_solve_mid (N = 40): 32,768 QPs, a 4.9 GiB state buffer (19,858 doubles per QP)."""
    _tiled_equal(cuda, 40, 1024, 32, 0)


def test_long_horizon_kernel_past_2gb_workspace(cuda):
    """k_solve_wide (N = 64): 16,384 QPs, a 5.4 GiB state buffer (43,954 doubles per QP)."""
    _tiled_equal(cuda, 64, 256, 64, 0)
