"""GPU tests of the device-resident closed loop (csrc/mpcqp_fleet.hip).

Every vehicle of a fleet must follow the reference's single-vehicle loop
(src/pipeline/control_stage.py:100-150):
  * the reference's own loop on the default plan (closed_loop.npz, exact solver in place of
    OSQP) is reproduced by every vehicle, step count included (65 steps to the goal);
  * vehicles with different plans / starts / goals match the exact oracle's loop
    (oracle/mpc_oracle.track_loop) and this build's host loop (TrajectoryTracker.track);
  * masked vehicles (goal reached, aborted, out of steps) stop; a vehicle whose QP has no
    solution aborts without disturbing the others.
Tolerance: states to 1e-7 absolute (px) over the whole loop -- the QPs themselves match to
<= 1e-8 relative (test_gpu_parity.py); the plant's sin/cos/tan may differ from glibc by an ulp.
"""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ATOL = 1e-7


def _default_plan(golden):
    g = golden("default_plan.npz")
    path = [tuple(map(float, p)) for p in g["path"]]
    return g, path


def _branches(golden):
    """The RRT* branch splines of the BASELINE config-3 generator (branches.npz)."""
    br = golden("branches.npz")
    off = br["spline_off"]
    return [br["spline"][off[i]:off[i + 1]] for i in range(len(off) - 1)]


def _tracker(N, V, M, sim_steps, map_resolution=0.8, use_graph=True, fused=False, **settings):
    from mpcqp.config import MPCConfig
    from mpcqp.pipeline.fleet import FleetTracker

    mpc = MPCConfig(horizon=N, sim_steps=sim_steps)
    return FleetTracker(mpc, map_resolution=map_resolution, max_vehicles=V, max_ref_len=M, device="cuda:0",
                        use_graph=use_graph, fused=fused, **settings)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("N,sim_steps", [(10, 100), (15, 300)])
def test_fleet_reproduces_reference_closed_loop(cuda, golden, N, sim_steps, fused):
    from mpcqp import _lib

    g, path = _default_plan(golden)
    loop = golden("closed_loop.npz")
    V = 16
    ft = _tracker(N, V, 64, sim_steps, float(g["map_resolution"]), fused=fused)
    ft.reset_from_plans([path] * V, np.tile(g["start"], (V, 1)), np.tile(g["goal"], (V, 1)))
    res = ft.run()
    ref_states = loop[f"N{N}_states"]
    assert (res.phase == _lib.FLEET_GOAL).all()
    assert (res.steps == len(ref_states)).all()
    for v in range(V):
        np.testing.assert_allclose(res.states[v], ref_states, rtol=0, atol=ATOL)
        np.testing.assert_allclose(res.inputs[v], loop[f"N{N}_u0"], rtol=0, atol=1e-6)
    # vehicles are independent and identical here: bit-identical traces
    for v in range(1, V):
        np.testing.assert_array_equal(res.states[v], res.states[0])
    ft.close()


def _varied_fleet(golden, V, seed=5):
    g, path = _default_plan(golden)
    paths = _branches(golden) + [np.asarray(path)]
    rng = np.random.default_rng(seed)
    chosen = [paths[i % len(paths)] for i in range(V)]
    starts = np.array([p[0] for p in chosen]) + rng.uniform(-3, 3, size=(V, 2))
    goals = np.array([p[-1] for p in chosen])
    return g, chosen, starts, goals


def test_fleet_matches_exact_oracle_loop(cuda, golden):
    import mpc_oracle as mo
    from mpcqp.control.ref_builder import build_reference

    N, steps = 15, 40
    g, paths, starts, goals = _varied_fleet(golden, 4)
    ft = _tracker(N, 4, 128, steps, float(g["map_resolution"]))
    refs = ft.reset_from_plans(paths, starts, goals)
    res = ft.run()
    op = mo.default_params(N, float(g["map_resolution"]))
    for v in range(4):
        ref = build_reference(paths[v], 15.0, N, 0.1)
        p = paths[v]
        yaw0 = float(np.arctan2(p[1][1] - p[0][1], p[1][0] - p[0][0]))
        ex = np.asarray(mo.track_loop(op, ref, starts[v], yaw0, goals[v], steps))
        np.testing.assert_array_equal(refs[v], ref)
        assert res.steps[v] == len(ex)
        np.testing.assert_allclose(res.states[v], ex, rtol=0, atol=ATOL)
    ft.close()


def test_fleet_matches_host_tracker(cuda, golden):
    """Vehicle v of the fleet == TrajectoryTracker.track on vehicle v's plan (13 plans, 60 steps)."""
    from mpcqp import _lib
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    N, steps, V = 20, 60, 13
    g, paths, starts, goals = _varied_fleet(golden, V, seed=11)
    ft = _tracker(N, 32, 128, steps, 0.8)
    ft.reset_from_plans(paths, starts, goals)
    res = ft.run(check_every=7)
    tracker = TrajectoryTracker(MPCConfig(horizon=N, sim_steps=steps), VizConfig())
    for v in range(V):
        planning = SimpleNamespace(plan=SimpleNamespace(success=True, path=[tuple(map(float, q)) for q in paths[v]]))
        maps = SimpleNamespace(start=tuple(starts[v]), goal=tuple(goals[v]))
        host = np.asarray(tracker.track(planning, maps, map_resolution=0.8, visualize=False).states)
        assert res.steps[v] == len(host)
        np.testing.assert_allclose(res.states[v], host, rtol=0, atol=ATOL)
        expect = _lib.FLEET_GOAL if np.hypot(*(host[-1, :2] - goals[v])) < 8.0 else _lib.FLEET_OUT_OF_STEPS
        assert res.phase[v] == expect
    ft.close()


def test_graph_and_stream_paths_agree_bitwise(cuda, golden):
    N, steps, V = 20, 30, 40
    g, paths, starts, goals = _varied_fleet(golden, V, seed=3)
    out = []
    for use_graph in (True, False):
        ft = _tracker(N, V, 128, steps, use_graph=use_graph)
        ft.reset_from_plans(paths, starts, goals)
        out.append(ft.run(check_every=9))
        ft.close()
    a, b = out
    np.testing.assert_array_equal(a.steps, b.steps)
    np.testing.assert_array_equal(a.phase, b.phase)
    for v in range(V):
        np.testing.assert_array_equal(a.states[v], b.states[v])


def test_unsolvable_vehicle_aborts_alone(cuda, golden):
    """A vehicle whose QP is non-finite fails the nominal AND the relaxed solve
    (control_stage.py:45-56) and aborts at step 0 (:108-110); the rest of the fleet runs on."""
    from mpcqp import _lib

    N, steps, V = 10, 20, 6
    g, path = _default_plan(golden)
    ft = _tracker(N, V, 64, steps, float(g["map_resolution"]))
    ft.reset_from_plans([path] * V, np.tile(g["start"], (V, 1)), np.tile(g["goal"], (V, 1)))
    ft.buffers()["state"][2, 0] = float("nan")
    ft.step(1)
    b = ft.buffers()
    assert b["mask"][:, 2].cpu().tolist() == [1, 1]  # nominal solve, then the relaxed retry
    assert (b["status"][:, 2].cpu().numpy() == _lib.NUMERICAL_ERROR).all()
    assert b["mask"][1, [v for v in range(V) if v != 2]].sum().item() == 0  # nobody else retried
    res = ft.run(steps - 1)
    assert res.phase[2] == _lib.FLEET_ABORTED and res.steps[2] == 0
    others = [v for v in range(V) if v != 2]
    assert (res.phase[others] == _lib.FLEET_OUT_OF_STEPS).all() and (res.steps[others] == steps).all()
    loop = golden("closed_loop.npz")
    for v in others:
        np.testing.assert_allclose(res.states[v], loop["N10_states"][:steps], rtol=0, atol=ATOL)
    ft.close()


def test_fleet_large_batch_properties(cuda, golden):
    """4096 vehicles (config-3 scale) on the 13 plans: every QP solved, identical vehicles give
    identical traces, and the trace is consistent with the plant applied to the recorded inputs."""
    import mpc_oracle as mo

    N, steps, V = 20, 12, 4096
    g, paths, starts, goals = _varied_fleet(golden, 13, seed=21)
    idx = np.arange(V) % 13
    ft = _tracker(N, V, 128, steps)
    ft.reset_from_plans([paths[i] for i in idx], starts[idx], goals[idx])
    res = ft.run()
    b = ft.buffers()
    assert ((res.steps == steps) | (res.phase == 1)).all()
    st = b["status"][0, :V].cpu().numpy()
    assert (st == 1).all()
    for v in range(13, V, 997):
        np.testing.assert_array_equal(res.states[v], res.states[v % 13])
    params = ft.params
    for v in range(0, V, 512):
        x = np.asarray(res.states[v])
        u = np.asarray(res.inputs[v])
        for k in range(1, len(x)):
            nxt = mo.f_discrete(x[k - 1], u[k], params.dt, params.wheelbase_px)
            np.testing.assert_allclose(x[k], nxt, rtol=0, atol=1e-9)
    ft.close()


# every buffer the loop owns (the masks are scratch: the stepped path clears them for vehicles that
# no longer run, the fused loop leaves each vehicle's last-step masks)
_LOOP_BUFFERS = ("state", "u_prev", "path_idx", "phase", "steps", "trace", "u_trace", "X", "status", "u0")


@pytest.mark.parametrize("N,V,steps,seed", [(10, 40, 60, 3), (20, 300, 45, 7), (24, 64, 30, 9), (30, 64, 30, 13)])
def test_fused_loop_equals_stepped_loop_bitwise(cuda, golden, N, V, steps, seed):
    """mpcqp_fleet_loop (one launch, k_fleet_loop) == mpcqp_fleet_run (graph-replayed steps), every
    output buffer bit for bit: N = 10 / 20 keep the model block in LDS, N = 24 / 30 re-derive it
    from the window for the outputs (packed Pbar), N = 30 at the register limit."""
    g, paths, starts, goals = _varied_fleet(golden, V, seed=seed)
    bufs = []
    for fused in (False, True):
        ft = _tracker(N, V, 128, steps, fused=fused)
        ft.reset_from_plans(paths, starts, goals)
        res = ft.run()
        bufs.append({k: ft.buffers()[k].cpu().numpy().copy() for k in _LOOP_BUFFERS})
        ft.close()
    a, b = bufs
    for k in _LOOP_BUFFERS:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert (res.phase != 0).all() or (res.steps == steps).all()


def test_fused_loop_partial_runs_and_resume(cuda, golden):
    """steps < needed: the fused loop stops every vehicle after that many steps and a second call
    resumes from the device state -- the same as stepping."""
    N, V = 15, 24
    g, paths, starts, goals = _varied_fleet(golden, V, seed=17)
    out = []
    for fused in (False, True):
        ft = _tracker(N, V, 128, 80, fused=fused)
        ft.reset_from_plans(paths, starts, goals)
        ft.step(7)
        ft.step(11)
        res = ft.run()
        out.append((res, {k: ft.buffers()[k].cpu().numpy().copy() for k in _LOOP_BUFFERS}))
        ft.close()
    for k in _LOOP_BUFFERS:
        np.testing.assert_array_equal(out[0][1][k], out[1][1][k], err_msg=k)


def test_fused_loop_unsolvable_vehicle_aborts_alone(cuda, golden):
    from mpcqp import _lib

    N, steps, V = 10, 20, 6
    g, path = _default_plan(golden)
    ft = _tracker(N, V, 64, steps, float(g["map_resolution"]), fused=True)
    ft.reset_from_plans([path] * V, np.tile(g["start"], (V, 1)), np.tile(g["goal"], (V, 1)))
    ft.buffers()["state"][2, 0] = float("nan")
    res = ft.run()
    b = ft.buffers()
    assert b["mask"][:, 2].cpu().tolist() == [1, 1]  # nominal solve, then the relaxed retry
    assert (b["status"][:, 2].cpu().numpy() == _lib.NUMERICAL_ERROR).all()
    assert res.phase[2] == _lib.FLEET_ABORTED and res.steps[2] == 0
    others = [v for v in range(V) if v != 2]
    assert (res.phase[others] == _lib.FLEET_OUT_OF_STEPS).all() and (res.steps[others] == steps).all()
    loop = golden("closed_loop.npz")
    for v in others:
        np.testing.assert_allclose(res.states[v], loop["N10_states"][:steps], rtol=0, atol=ATOL)
    ft.close()


def test_fused_loop_falls_back_past_one_wave(cuda, golden):
    """Horizons past the one-wave kernel (N = 40, mid kernel) run mpcqp_fleet_loop through the
    stepped graph path: the same results as mpcqp_fleet_run."""
    N, V, steps = 40, 8, 12
    g, paths, starts, goals = _varied_fleet(golden, V, seed=23)
    bufs = []
    for fused in (False, True):
        ft = _tracker(N, V, 160, steps, fused=fused)
        ft.reset_from_plans(paths, starts, goals)
        ft.run()
        bufs.append({k: ft.buffers()[k].cpu().numpy().copy() for k in _LOOP_BUFFERS})
        ft.close()
    for k in _LOOP_BUFFERS:
        np.testing.assert_array_equal(bufs[0][k], bufs[1][k], err_msg=k)


def test_fused_loop_dispatch_order_past_the_wave_slots(cuda, golden):
    """More vehicles than wave slots (2 per SIMD): the fused loop dispatches them longest reference
    first (k_fleet_order); every vehicle still equals the stepped path bit for bit."""
    import torch

    props = torch.cuda.get_device_properties(0)
    N, steps = 10, 25
    V = 8 * props.multi_processor_count + 300
    g, paths, starts, goals = _varied_fleet(golden, 13, seed=29)
    idx = np.arange(V) % 13
    bufs = []
    for fused in (False, True):
        ft = _tracker(N, V, 128, steps, fused=fused)
        ft.reset_from_plans([paths[i] for i in idx], starts[idx], goals[idx])
        ft.run()
        bufs.append({k: ft.buffers()[k].cpu().numpy().copy() for k in _LOOP_BUFFERS})
        ft.close()
    for k in _LOOP_BUFFERS:
        np.testing.assert_array_equal(bufs[0][k], bufs[1][k], err_msg=k)
