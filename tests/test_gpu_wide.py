"""Long horizons (N >= 32): the workgroup-per-QP kernel (csrc/mpcqp_wide.hip).

The reference builds its QP for any horizon (src/control/mpc_controller.py:47-57).  Horizons
32..63 run one 256-thread workgroup per QP (the arena in LDS up to N ~ 48, in the workspace
beyond).  Two modes: reproducible = 1 is the C restatement parallelised without changing a
floating-point operation; the default (fast) mode's polish updates the inverse by rank-1 changes
and sums its line search in tree order.  Checks:
  * the exact oracle (mpc_oracle.solve_exact): U / X / u0 to 1e-8 relative, identical active sets;
  * reproducible = 1 against the C restatement fed the GPU's own LTV model (K1 output): U, X,
    statuses AND iteration counts identical bit for bit;
  * the fast mode against the same: statuses, active sets and all four counters identical on
    every QP, U to 1e-8;
  * the drop-in surface: MPCController(MPCConfig(horizon=40)) and a fleet at N = 40;
  * horizons past a wave (N = 64..127): K1 in chunks of 64 rows, the sweep in memory past 2N = 128.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_TOL = 1e-8


def _params(N):
    from mpcqp.config import MPCConfig

    return MPCConfig(horizon=N).to_parameters(0.8)


def _rel(a, b):
    return float(np.abs(a - b).max() / max(1.0, np.abs(b).max()))


def _solve_with_model(params, x0, ref, u_prev, **settings):
    import torch
    from mpcqp import _lib
    from mpcqp.control.mpc_controller import BatchedMPCController

    N = int(params.horizon)
    B = len(x0)
    ctrl = BatchedMPCController(params, B, device="cuda:0", **settings)
    sol = ctrl.solve_batch(x0, ref, u_prev)
    torch.cuda.synchronize()
    out = {k: getattr(sol, k).cpu().numpy().copy() for k in sol._fields}
    L = _lib.lib()
    ptr = L.mpcqp_model_buffer(ctrl._ws)
    model = None  # the fused one-wave solve builds its model on chip: no model buffer
    if ptr:
        model = np.zeros((B, L.mpcqp_model_stride(N)))
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        assert hip.hipMemcpy(model.ctypes.data, ptr, model.nbytes, 2) == 0
    ctrl.close()
    return out, model


@pytest.mark.parametrize("N", [32, 40, 48, 63, 64, 80, 127])
def test_long_horizons_match_exact_oracle(cuda, N):
    import mpc_oracle as mo
    from mpcqp import scenarios

    batch = scenarios.config3(24 if N < 64 else 8, horizon=N, seed=300 + N)
    params = _params(N)
    out, _ = _solve_with_model(params, batch.x0, batch.ref, batch.u_prev)
    assert (out["status"] == 1).all(), np.unique(out["status"], return_counts=True)
    for b in range(batch.size):
        ex = mo.solve_exact(params, batch.x0[b], batch.ref[b], batch.u_prev[b])
        assert ex.converged
        e = max(_rel(out["U"][b], ex.Umat), _rel(out["X"][b], ex.X), _rel(out["u0"][b], ex.Umat[:, 0]))
        assert e <= REL_TOL, f"N={N} QP {b}: rel err {e:.3e}"
        assert np.array_equal(out["active"][b], ex.active), f"N={N} QP {b}: active set differs"


@pytest.mark.parametrize("N,settings", [(32, {}), (40, {}), (40, {"polish_near": 0.0}),
                                        (48, {"polish_from": 0, "polish_near": 0.0}), (63, {}), (64, {}),
                                        (90, {})])
def test_long_horizons_bit_exact_with_c_restatement(cuda, N, settings):
    """Same model in -> same bits out: solutions, statuses, ADMM/polish/factorization/line-search
    counts all identical to oracle/mpcqp_cpu.c (100 % of QPs, not a majority)."""
    import cpu_solver
    from mpcqp import scenarios

    batch = scenarios.config3(48 if N < 64 else 16, horizon=N, seed=700 + N)
    params = _params(N)
    out, model = _solve_with_model(params, batch.x0, batch.ref, batch.u_prev, reproducible=1, **settings)
    ref = cpu_solver.cpu_solve_models(params, model, **settings)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["iters"], ref["iters"]), np.argwhere((out["iters"] != ref["iters"]).any(axis=1))
    assert np.array_equal(out["U"], ref["U"])
    assert np.array_equal(out["X"], ref["X"])
    assert np.array_equal(out["active"], ref["active"])


@pytest.mark.parametrize("N,settings", [(32, {}), (33, {}), (40, {}), (41, {}),
                                        (48, {"polish_from": 0, "polish_near": 0.0}), (52, {}), (56, {}), (63, {}),
                                        (64, {})])
def test_long_horizons_fast_mode_against_c_restatement(cuda, N, settings):
    """The default (fast) long-horizon mode (the mid kernel from N = 33, the one-wave kernel at N = 32): the
    same optimum, statuses, active sets
    and all four counters as the C restatement on every QP (its tree-order sums round differently,
    but no counter decision flips: profiles/r03_s16_iters_agreement.json, 6 x 1024 QPs at N = 32..63)."""
    import cpu_solver
    from mpcqp import scenarios

    batch = scenarios.config3(64, horizon=N, seed=900 + N)
    params = _params(N)
    out, model = _solve_with_model(params, batch.x0, batch.ref, batch.u_prev, **settings)
    # N = 32 runs the one-wave kernel with K1 fused (no model buffer): the C code from the inputs
    ref = (cpu_solver.cpu_solve_models(params, model, **settings) if model is not None else
           cpu_solver.cpu_solve(params, batch.x0, batch.ref, batch.u_prev, **settings))
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["active"], ref["active"])
    assert _rel(out["U"], ref["U"]) <= REL_TOL and _rel(out["X"], ref["X"]) <= REL_TOL
    same = (out["iters"] == ref["iters"]).all(axis=1)
    assert same.all(), f"QPs {np.flatnonzero(~same)[:10]} disagree on iteration counts"


@pytest.mark.parametrize("N", [33, 45, 53, 61])
def test_mid_kernel_deterministic_below_the_bucket(cuda, N):
    """The mid kernel at N < NT (padding steps in every bucket) is deterministic: the same batch solved
    twice gives the same bits.  (A round-6 setup rewrite once left the row registers of the steps past N
    unset: N = 33 then varied run to run in the last bits and in its iteration counts.)"""
    from mpcqp import scenarios

    batch = scenarios.config3(256, horizon=N, seed=1300 + N)
    params = _params(N)
    a, _ = _solve_with_model(params, batch.x0, batch.ref, batch.u_prev)
    b, _ = _solve_with_model(params, batch.x0, batch.ref, batch.u_prev)
    for k in ("U", "X", "u0", "status", "iters", "active"):
        assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), f"N={N}: {k} differs between runs"


@pytest.mark.parametrize("N,config,settings", [(1, "config3", {}), (5, "config3", {}), (10, "config3", {}),
                                               (15, "config3", {"polish_near": 0.0}), (20, "config3", {}),
                                               (20, "config2", {}), (20, "config3", {"polish_from": 0, "polish_near": 0.0}),
                                               (31, "config3", {})])
def test_reproducible_mode_bit_exact_with_c_restatement(cuda, N, config, settings):
    """mpcqp_params.reproducible = 1 at the short horizons too (the bench's N = 20 included): every
    QP's solution, status and ADMM / polish / factorization / line-search counts identical to the C
    restatement given the same model -- 100 % of QPs -- and the exact optimum as the fast kernel."""
    import cpu_solver
    from mpcqp import scenarios

    batch = scenarios.config2(64, horizon=N) if config == "config2" else scenarios.config3(64, horizon=N, seed=800 + N)
    params = _params(N)
    out, model = _solve_with_model(params, batch.x0, batch.ref, batch.u_prev, reproducible=1, **settings)
    ref = cpu_solver.cpu_solve_models(params, model, **settings)
    assert np.array_equal(out["status"], ref["status"])
    assert np.array_equal(out["iters"], ref["iters"]), np.argwhere((out["iters"] != ref["iters"]).any(axis=1))
    assert np.array_equal(out["U"], ref["U"])
    assert np.array_equal(out["X"], ref["X"])
    assert np.array_equal(out["active"], ref["active"])
    fast, _ = _solve_with_model(params, batch.x0, batch.ref, batch.u_prev, **settings)
    assert np.array_equal(fast["active"], out["active"]) and _rel(fast["U"], out["U"]) <= REL_TOL


@pytest.mark.parametrize("N", [63, 64, 100, 127])
def test_long_window_k1_matches_restatement(cuda, N):
    """K1 on windows longer than a wave (N + 1 > 64 rows: chunks of 64 with carries) against the
    C restatement's build bit for bit, and numpy's unwrap, with 2 pi jumps inside and across chunks."""
    import cpu_solver
    from mpcqp import scenarios

    batch = scenarios.config3(12, horizon=N, seed=40 + N)
    ref = batch.ref.copy()
    ref[::3, 30:, 2] += 2 * np.pi
    ref[1::3, 64:, 2] -= 4 * np.pi
    ref[2::3, 65:, 2] += 2 * np.pi
    params = _params(N)
    out, model = _solve_with_model(params, batch.x0, ref, batch.u_prev, reproducible=1)
    cpu = cpu_solver.cpu_solve(params, batch.x0, ref, batch.u_prev, want_model=True)["model"]
    # window rows (x, y, unwrapped yaw, v), x0 and u_prev bit for bit; the linearisation's
    # coefficients to 1e-12 (device sincos vs the host libm)
    assert np.array_equal(model[:, 7 * N: 11 * N + 10], cpu[:, 7 * N: 11 * N + 10])
    assert np.array_equal(model[:, 7 * N + 2: 11 * N + 4: 4], np.unwrap(ref[:, :, 2], axis=1))
    assert _rel(model[:, : 7 * N], cpu[:, : 7 * N]) <= 1e-12


def test_horizon_past_the_thread_count(cuda):
    """N = 200 (2N = 400 variables > 256 threads per QP: the in-memory sweep, chunked K1 and every
    strided loop past one pass) against the exact oracle, through MPCController.solve."""
    import mpc_oracle as mo
    from mpcqp import scenarios
    from mpcqp.control.mpc_controller import MPCController

    N = 200
    batch = scenarios.config3(2, horizon=N, seed=5)
    params = _params(N)
    for b in range(batch.size):
        u0, X, U = MPCController(params).solve(batch.x0[b], batch.ref[b], u_prev=batch.u_prev[b])
        ex = mo.solve_exact(params, batch.x0[b], batch.ref[b], batch.u_prev[b])
        assert ex.converged and U is not None
        assert max(_rel(U, ex.Umat), _rel(X, ex.X)) <= REL_TOL


def test_long_horizon_newton_and_max_iter(cuda):
    """Method newton and an ADMM capped below convergence: statuses and counts as the C code."""
    import cpu_solver
    from mpcqp import scenarios

    N = 36
    batch = scenarios.config3(32, horizon=N, seed=9)
    params = _params(N)
    for method, settings in (("newton", {}), ("admm", dict(max_iter=40, polish_from=0, polish_near=0.0))):
        out, model = _solve_with_model(params, batch.x0, batch.ref, batch.u_prev, method=method, reproducible=1,
                                       **settings)
        ref = cpu_solver.cpu_solve_models(params, model, method=1 if method == "newton" else 0, **settings)
        assert np.array_equal(out["status"], ref["status"]), method
        assert np.array_equal(out["iters"], ref["iters"]), method
        assert np.array_equal(out["U"], ref["U"]), method
        fast, _ = _solve_with_model(params, batch.x0, batch.ref, batch.u_prev, method=method, **settings)
        assert np.array_equal(fast["status"], ref["status"]), method
        assert _rel(fast["U"], ref["U"]) <= REL_TOL, method


def test_mpc_controller_drop_in_at_horizon_40(cuda):
    """MPCController(params).solve at a horizon the one-wave kernel cannot hold, with a window
    longer than N+1 rows (the reference reads rows 0..N)."""
    import mpc_oracle as mo
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import MPCController
    from mpcqp import scenarios
    from mpcqp.control.ref_builder import build_reference

    plan = scenarios.load_default_plan()
    ref_g = build_reference(plan["path"], 15.0, 40, 0.1)
    params = MPCConfig(horizon=40).to_parameters(0.8)
    x0 = np.array([plan["start"][0], plan["start"][1], float(plan["yaw0"]), 5.0])
    u0, X, U = MPCController(params).solve(x0, ref_g[:45], u_prev=np.zeros(2))
    ex = mo.solve_exact(params, x0, ref_g[:41], np.zeros(2))
    assert _rel(U, ex.Umat) <= REL_TOL and _rel(X, ex.X) <= REL_TOL
    assert X.shape == (4, 41) and U.shape == (2, 40)


@pytest.mark.parametrize("N", [40, 56, 80])
def test_fleet_at_long_horizons(cuda, N):
    """The device closed loop at N = 40, 56 (the mid kernel's 4-part bucket) and 80 (k_fleet_build -- in chunks of 64 window rows at
    80 -- + the long-horizon solve) against the oracle's restatement of control_stage.py:84-150 on
    the same plans."""
    import mpc_oracle as mo
    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.pipeline.fleet import FleetTracker, initial_state

    V, steps = 4, 30 if N <= 40 else 12
    paths, starts, goals = scenarios.fleet5(V, seed=21)
    mpc = MPCConfig(horizon=N, sim_steps=steps)
    ft = FleetTracker(mpc, map_resolution=0.8, max_vehicles=V, max_ref_len=200, device="cuda:0")
    refs = ft.reset_from_plans(paths, starts, goals)
    res = ft.run()
    params = mpc.to_parameters(0.8)
    for v in range(V):
        s0 = initial_state(paths[v], starts[v])
        states = mo.track_loop(params, refs[v], s0[:2], s0[2], goals[v], steps)
        assert len(states) == len(res.states[v])
        np.testing.assert_allclose(res.states[v], np.asarray(states), rtol=0, atol=1e-6)
    ft.close()
