"""GPU tests of the reference-facing surface: MPCController.solve (B=1 shim),
TrajectoryTracker.step / track, against the reference's own known answer and closed loop."""
from __future__ import annotations

import logging
from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_mpc_controller_reference_test_case(cuda):
    """Reference tests/test_mpc_controller.py:7-17, plus the exact optimum."""
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import MPCController

    cfg = MPCConfig(horizon=5)
    controller = MPCController(cfg.to_parameters(map_resolution=0.2))
    x0 = np.array([0.0, 0.0, 0.0, 5.0])
    ref = np.tile(np.array([1.0, 0.0, 0.0, 5.0]), (cfg.horizon + 1, 1))
    u0, Xp, Up = controller.solve(x0, ref)
    assert u0 is not None and Xp is not None and Up is not None
    assert Xp[0, 1] > x0[0]
    assert u0.shape == (2,) and Xp.shape == (4, 6) and Up.shape == (2, 5)
    np.testing.assert_allclose(u0, [-9.1046224514, 0.0], atol=1e-8)
    np.testing.assert_allclose(Xp[:, 0], x0)


def _default_plan(golden):
    g = golden("default_plan.npz")
    planning = SimpleNamespace(plan=SimpleNamespace(success=True, path=[tuple(map(float, p)) for p in g["path"]]))
    maps = SimpleNamespace(start=tuple(g["start"]), goal=tuple(g["goal"]))
    return g, planning, maps


@pytest.mark.parametrize("N,sim_steps,settings", [(10, 100, {}), (15, 300, {}),
                                                  (10, 100, {"polish_from": 150}), (15, 300, {"polish_from": 50})])
def test_tracker_reproduces_reference_closed_loop(cuda, golden, N, sim_steps, settings):
    """BASELINE config 1 (N=10, 100 steps) and the code default (N=15): the reference's
    TrajectoryTracker loop (closed_loop.npz, exact solve substituted for OSQP) is reproduced
    step for step with every QP solved on the GPU: under the B=1 drop-in's latency schedule
    ({}: mpc_controller.latency_settings, polish_from 25) and under polish_from 150 and 50, all of
    which reach the same exact optimum."""
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    g, planning, maps = _default_plan(golden)
    loop = golden("closed_loop.npz")
    tracker = TrajectoryTracker(MPCConfig(horizon=N, sim_steps=sim_steps), VizConfig(),
                                solver_settings=dict(settings), relaxed_solver_settings=dict(settings))
    result = tracker.track(planning, maps, map_resolution=float(g["map_resolution"]), visualize=False)
    states = np.asarray(result.states)
    ref_states = loop[f"N{N}_states"]
    assert states.shape == ref_states.shape == (65, 4)
    np.testing.assert_allclose(states, ref_states, rtol=0, atol=1e-7)
    assert np.hypot(*(states[-1, :2] - np.asarray(maps.goal))) < 8.0


def test_step_is_one_loop_iteration(cuda, golden):
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    loop = golden("closed_loop.npz")
    tracker = TrajectoryTracker(MPCConfig(horizon=15), VizConfig())
    params = tracker.mpc.to_parameters(0.8)
    for k in (0, 10, 40):
        nxt, u0, Xp = tracker.step(loop["N15_x0"][k], loop["N15_window"][k], loop["N15_u_prev"][k], params)
        np.testing.assert_allclose(u0, loop["N15_u0"][k], rtol=0, atol=1e-8)
        np.testing.assert_allclose(nxt, loop["N15_states"][k], rtol=0, atol=1e-8)
        assert Xp.shape == (4, 16)


def test_three_argument_step_reproduces_reference_loop(cuda, golden):
    """SURVEY §8b's contract ``step(state, ref_window, u_prev) -> (next_state, u0, X)``: no params
    argument, so the tracker uses ``MPCConfig.to_parameters(0.8)`` (the reference's
    ``MapConfig.map_resolution`` default) -- the resolution closed_loop.npz was generated at.
    Every one of the 65 recorded N = 15 windows of the reference's own loop is replayed."""
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    loop = golden("closed_loop.npz")
    assert float(golden("default_plan.npz")["map_resolution"]) == 0.8
    tracker = TrajectoryTracker(MPCConfig(horizon=15), VizConfig())
    for k in range(len(loop["N15_x0"])):
        nxt, u0, Xp = tracker.step(loop["N15_x0"][k], loop["N15_window"][k], loop["N15_u_prev"][k])
        np.testing.assert_allclose(u0, loop["N15_u0"][k], rtol=0, atol=1e-8)
        np.testing.assert_allclose(nxt, loop["N15_states"][k], rtol=0, atol=1e-8)
        assert Xp.shape == (4, 16)
        np.testing.assert_array_equal(Xp[:, 0], loop["N15_x0"][k])


def test_unsolvable_input_takes_the_relaxation_path_and_aborts(cuda, caplog):
    """Non-finite data -> status numerical_error -> relaxation retry (control_stage.py:45-56)
    -> still None -> (None, None, None), as the reference's loop expects (:108-110)."""
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    tracker = TrajectoryTracker(MPCConfig(horizon=5), VizConfig())
    params = tracker.mpc.to_parameters(0.8)
    state = np.array([np.nan, 0.0, 0.0, 5.0])
    ref = np.tile(np.array([1.0, 0.0, 0.0, 5.0]), (6, 1))
    with caplog.at_level(logging.WARNING):
        out = tracker.step(state, ref, np.zeros(2), params)
    assert all(v is None for v in out)
    assert any("relaxation" in r.getMessage() for r in caplog.records)


def test_batched_controller_reuses_device_inputs(cuda):
    """Device-resident inputs are consumed in place (no host round trip) and results stay on
    the device."""
    import torch
    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = scenarios.config3(128)
    ctrl = BatchedMPCController(MPCConfig(horizon=20).to_parameters(0.8), 128, device="cuda:0")
    x0 = torch.from_numpy(b.x0).to(cuda)
    ref = torch.from_numpy(b.ref).to(cuda)
    up = torch.from_numpy(b.u_prev).to(cuda)
    sol = ctrl.solve_batch(x0, ref, up)
    assert sol.u0.device.type == "cuda" and sol.X.shape == (128, 4, 21)
    torch.cuda.synchronize()
    assert (sol.status == 1).all().item()
    np.testing.assert_array_equal(sol.u0.cpu().numpy(), sol.U[:, :, 0].cpu().numpy())
    ctrl.close()


def test_solve_one_equals_solve_batch(cuda):
    """The B=1 drop-in (BatchedMPCController.solve_one, behind MPCController.solve) returns
    exactly what solve_batch returns for the same QP, at a fused (N = 20) and a long (N = 40)
    horizon, including the unsolvable case's status: the staged path (mpcqp_stage /
    mpcqp_solve_staged: the kernels read and write the workspace's mapped host blocks in place,
    on its private stream), with windows longer than N + 1 rows and u_prev omitted."""
    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    for N in (20, 40):
        b = scenarios.config3(5, horizon=N, seed=11)
        ref = b.ref.copy()
        ref[3, 2:, 0] = np.nan  # status numerical_error
        up = b.u_prev.copy()
        up[4] = 0.0
        ctrl = BatchedMPCController(MPCConfig(horizon=N).to_parameters(0.8), 5, device="cuda:0")
        sol = ctrl.solve_batch(b.x0, ref, up)
        st, U, X = sol.status.cpu().numpy(), sol.U.cpu().numpy(), sol.X.cpu().numpy()
        for q in range(5):
            longer = np.vstack([ref[q], ref[q][-1:] + 1.0])  # an extra row the solve must not read
            status, u0, Xq, Uq = ctrl.solve_one(b.x0[q], longer, None if q == 4 else up[q])
            assert ctrl._one is not None
            assert status == st[q]
            if status == _lib.SOLVED:
                assert np.array_equal(Uq, U[q]) and np.array_equal(Xq, X[q]) and np.array_equal(u0, U[q][:, 0])
        assert st[3] == _lib.NUMERICAL_ERROR
        ctrl.close()


def test_drop_in_unpolished_result_is_osqp_scaled(cuda):
    """A QP the drop-in does not finish with the polished exact optimum (here ADMM capped at
    max_iter = 50) is solved again under OSQP's 10 Ruiz passes: MPCController then returns exactly
    what a scaling = 10 solve of the same QP returns, so an unpolished result does not depend on this
    build's one-pass default.  A polished QP returns the exact optimum, which no scaling
    changes.  With the polish off, every drop-in solve runs OSQP's 10 passes."""
    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController, MPCController

    N = 15
    b = scenarios.config3(24, horizon=N, seed=3)
    params = MPCConfig(horizon=N).to_parameters(0.8)
    for capped in (dict(max_iter=50, polish_from=0, polish_near=0.0),
                   dict(max_iter=50, polish=0, polish_from=0, polish_near=0.0)):
        res = {}
        for sc in (1, 10):
            c = BatchedMPCController(params, 24, device="cuda:0", scaling=sc, **capped)
            sol = c.solve_batch(b.x0, b.ref, b.u_prev)
            res[sc] = (sol.status.cpu().numpy().copy(), sol.U.cpu().numpy().copy())
            c.close()
        st1, U1 = res[1]
        st10, U10 = res[10]
        polished = (st1 == _lib.SOLVED) & bool(capped.get("polish", 1))
        assert (~polished).any()  # the fallback case occurs
        if capped.get("polish", 1):
            assert polished.any()
        for q in range(24):
            u0, X, Uq = MPCController(params, **capped).solve(b.x0[q], b.ref[q], u_prev=b.u_prev[q])
            exp_st, exp_U = (st1[q], U1[q]) if polished[q] else (st10[q], U10[q])
            if exp_st in (_lib.SOLVED, _lib.SOLVED_INACCURATE):
                # the drop-in runs the resident server kernel (k_serve), the batch k_solve: the same
                # operations, contracted only within a source expression (-ffp-contract=on), so the
                # same bits, unpolished ADMM iterates included
                assert Uq is not None and np.array_equal(Uq, exp_U), q
            else:
                assert Uq is None, q


def test_b1_server_matches_launch_per_call(cuda, monkeypatch):
    """The resident B=1 server (mpcqp_solve_served) returns exactly what a launch per call
    (mpcqp_solve_staged) returns, across its idle exit (no request for > 2 ms: the next call starts
    the wave again), a parameter change (set_params stops it) and back-to-back requests."""
    import time

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = scenarios.config3(12, horizon=15, seed=41)
    params = MPCConfig(horizon=15).to_parameters(0.8)
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MPCQP_B1_SERVER", mode)
        ctrl = BatchedMPCController(params, 1, device="cuda:0")
        out = []
        for q in range(12):
            if q in (4, 9):
                time.sleep(0.01)  # past the server's 2 ms idle limit
            if q == 7:
                ctrl.set_params(params)  # stops a live server
            out.append(ctrl.solve_one(b.x0[q], b.ref[q], b.u_prev[q]))
        ctrl.close()
        res[mode] = out
    for q in range(12):
        a, c = res["0"][q], res["1"][q]
        assert a[0] == c[0] == 1
        for x, y in zip(a[1:], c[1:]):
            assert np.array_equal(x, y), q
