"""GPU tests of the config-5 swarm (mpcqp/pipeline/swarm.py, csrc/mpcqp_swarm.hip): batched RRT*
plans, device references, the fleet closed loop and the PER-STEP device replan trigger with the
replanning itself on the device, end to end on the default inflated grid.

Between replans every vehicle follows the reference's single-vehicle loop: a vehicle that was
never replanned reproduces the oracle's restatement of TrajectoryTracker.track on its own plan
(1e-7 px); a replanned vehicle reproduces it up to the replan step, its new plan is the reference
planner's from where it stood with its replan seed, and after the replan it reproduces the
reference loop body on the new reference.  The checkers run on the host only: the loop is
mpc_oracle.track_loop / track_from with the C restatement's solves, the plans are
oracle/rrt_oracle.grow_tree on the seed's own sample stream with oracle extraction and pruning --
nothing in them touches the GPU."""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_HORIZON = 15


def _pairs(occ, V, seed):
    rng = np.random.default_rng(seed)
    free = np.argwhere(occ == 1)
    starts, goals = [], []
    while len(starts) < V:
        a, b = free[rng.integers(0, len(free), 2)]
        if np.hypot(*(a - b)) > 30:  # keep the trips non-trivial
            starts.append(a[::-1].astype(float))
            goals.append(b[::-1].astype(float))
    return np.array(starts), np.array(goals)


def _planner_params(seed=13):
    from mpcqp.planning.rrt_star import default_planner_parameters

    return default_planner_parameters(max_iterations=1500, random_seed=int(seed))


def _swarm(occ, V, sim_steps, **kw):
    from mpcqp.config import MPCConfig
    from mpcqp.pipeline.swarm import Swarm

    return Swarm(occ, MPCConfig(horizon=N_HORIZON, sim_steps=sim_steps), _planner_params(),
                 map_resolution=0.8, max_vehicles=V, device="cuda:0", **kw)


def _c_solve(params, state, window, u_prev):
    """One QP by the C restatement (oracle/mpcqp_cpu.c): no GPU in the checker."""
    import cpu_solver

    out = cpu_solver.cpu_solve(params, np.asarray(state, float)[None], np.asarray(window, float)[None],
                               np.asarray(u_prev, float)[None], nthreads=1)
    if out["status"][0] not in (1, 2):
        return None, None, None
    return out["u0"][0].copy(), out["X"][0].copy(), out["U"][0].copy()


def _oracle_params():
    import mpc_oracle as mo

    return mo.default_params(N_HORIZON, 0.8)


def _host_track(path, start, goal, steps):
    """The reference's track loop (control_stage.py:79-150) restated by the oracle
    (mpc_oracle.track_loop), every QP solved by the C restatement on the host."""
    import mpc_oracle as mo
    from mpcqp.control.ref_builder import build_reference

    ref = build_reference(path, 15.0, N_HORIZON, 0.1)
    yaw0 = float(np.arctan2(path[1][1] - path[0][1], path[1][0] - path[0][0])) if len(path) > 1 else 0.0
    return np.asarray(mo.track_loop(_oracle_params(), ref, start, yaw0, goal, steps, solve_fn=_c_solve))


def _host_continue(state, u_prev, path, goal, steps):
    """The loop body of control_stage.py:100-150 from a given state / u_prev on a new plan (the
    swarm's replan: pose, speed and u_prev carry over, path_idx restarts at 0) -- mpc_oracle.track_from
    with the C restatement's solves."""
    import mpc_oracle as mo
    from mpcqp.control.ref_builder import build_reference

    ref = build_reference(path, 15.0, N_HORIZON, 0.1)
    return np.asarray(mo.track_from(_oracle_params(), ref, state, u_prev, goal, steps, solve_fn=_c_solve))


def _oracle_plan(occ, start, goal, seed, cr=False):
    """RRTStarPlanner.plan (rrt_star.py:201-283) on the host: oracle/rrt_oracle.grow_tree fed the
    seed's own sample stream (draw_samples), oracle extraction and shortcut pruning, then the
    Catmull-Rom smoothing of the host restatement (pinned by branches.npz).  cr: the steer's
    trig correctly rounded (the device's) instead of glibc's."""
    import rrt_oracle as ro
    from mpcqp.common.geometry import catmull_rom_spline
    from mpcqp.planning.rrt_star import draw_samples

    prm = _planner_params(seed)
    smp = draw_samples(int(seed), goal, occ.shape, prm.goal_sample_rate, prm.max_iterations)
    nodes, _, gi = ro.grow_tree(occ, start, goal, smp, step=prm.step, goal_radius=prm.goal_radius,
                                rewire_radius=prm.rewire_radius, collision_step=prm.collision_step,
                                trig=ro.CR_TRIG if cr else ro.LIBM_TRIG)
    if gi < 0:
        return None
    path = ro.extract_path(nodes, gi)
    if prm.prune_path and len(path) >= 2:
        pruned = ro.shortcut_prune(occ, path, prm.collision_step)
        if len(pruned) >= 2:
            path = pruned
    if len(path) >= 2 and prm.spline_samples > 1:
        spline = catmull_rom_spline(path, samples_per_segment=prm.spline_samples, alpha=prm.spline_alpha,
                                    dedupe_tol=prm.dedupe_tolerance)
        if len(spline) >= 2:
            path = [tuple(map(float, q)) for q in spline]
    return path


def _check_plan(occ, start, goal, seed, path, tol=1e-4):
    """The device plan against the host restatement of the reference planner (_oracle_plan): same
    number of points, coordinates within the ~1e-5 px the duplicated end knots amplify an ulp to
    (the trees themselves are bit-exact, test_gpu_planning.py).  Where the plan differs from the
    libm restatement's, it must be the plan with correctly rounded steer trig (glibc's rounding,
    rare).  Returns "libm" or "cr"."""
    got = np.asarray(path)

    def same(plan):
        return plan is not None and np.asarray(plan).shape == got.shape and \
            np.abs(np.asarray(plan) - got).max() <= tol

    if same(_oracle_plan(occ, start, goal, seed)):
        return "libm"
    plan = _oracle_plan(occ, start, goal, seed, cr=True)
    assert plan is not None
    ref = np.asarray(plan)
    assert ref.shape == got.shape, (ref.shape, got.shape)
    np.testing.assert_allclose(got, ref, rtol=0, atol=tol)
    return "cr"


def test_device_smoothing_matches_reference_planner(cuda, golden):
    """mpcqp_catmull_rom (via paths_batch(smoothing="device")) against the host restatement of
    rrt_star.py:104-159 on 48 plans, and on the reference's own default plan."""
    from mpcqp.common.geometry import catmull_rom_spline
    from mpcqp.planning.rrt_star import BatchedRRTStarPlanner

    occ = golden("default_plan.npz")["occupancy"]
    starts, goals = _pairs(occ, 48, 3)
    pl = BatchedRRTStarPlanner(occ, _planner_params(), device="cuda:0")
    dev = pl.paths_batch(starts, goals, np.arange(48), smoothing="device")
    host = pl.paths_batch(starts, goals, np.arange(48), smoothing="host")
    assert sum(p is not None for p in dev) > 40
    for d, h in zip(dev, host):
        assert (d is None) == (h is None)
        if d is not None:
            assert len(d) == len(h)
            np.testing.assert_allclose(np.asarray(d), np.asarray(h), rtol=0, atol=1e-4)
    # edge cases: two points, duplicates (dedupe), collinear, a single point
    import torch

    cases = [[(0.0, 0.0), (10.0, 5.0)], [(0.0, 0.0), (0.0, 0.0), (3.0, 4.0), (3.0, 4.0), (9.0, 1.0)],
             [(0.0, 0.0), (1.0, 1.0), (2.0, 2.0), (5.0, 5.0)], [(7.0, 7.0)]]
    W = max(len(c) for c in cases)
    arr = np.zeros((len(cases), W, 2))
    for i, c in enumerate(cases):
        arr[i, : len(c)] = c
    out, n = pl.smooth(torch.from_numpy(arr).to(cuda), torch.tensor([len(c) for c in cases], device=cuda))
    out, n = out.cpu().numpy(), n.cpu().numpy()
    for i, c in enumerate(cases):
        ref = catmull_rom_spline(c, samples_per_segment=20, alpha=0.5)
        assert n[i] == len(ref), (i, n[i], len(ref))
        np.testing.assert_allclose(out[i, : n[i]], ref, rtol=0, atol=1e-9)


def test_swarm_vehicles_follow_the_reference_loop(cuda, golden):
    from mpcqp import _lib

    occ = golden("default_plan.npz")["occupancy"]
    V, steps = 24, 120
    starts, goals = _pairs(occ, V, 1)
    sw = _swarm(occ, V, steps, replan_distance=1e9)  # no off-track replans: the plain per-vehicle loop
    res = sw.run(starts, goals, seeds=np.arange(V), check_every=20)
    assert (res.replans == 0).all()
    assert res.planned.mean() > 0.8
    for v in np.flatnonzero(res.planned)[:8]:
        host = _host_track(res.paths[v], starts[v], goals[v], steps)
        assert res.steps[v] == len(host)
        np.testing.assert_allclose(res.states[v], host, rtol=0, atol=1e-7)
        _check_plan(occ, starts[v], goals[v], v, res.paths[v])
    done = res.phase[res.planned]
    assert np.isin(done, [_lib.FLEET_GOAL, _lib.FLEET_OUT_OF_STEPS]).all()


def test_per_step_replan_100_vehicles(cuda, golden):
    """BASELINE config 5 at its size: 100 vehicles on the default inflated grid, the trigger
    evaluated on the device after EVERY step.  Every initial plan is the reference planner's; every
    never-replanned vehicle equals the reference loop (oracle restatement, C solves) on its own
    plan; every replanned vehicle equals it up to its replan step, its new plan is the reference
    planner's from where it stood with its replan seed, and from there it follows the reference
    loop body on the new reference."""
    from mpcqp import _lib
    from mpcqp.pipeline.swarm import replan_seed

    occ = golden("default_plan.npz")["occupancy"]
    V, steps = 100, 150
    starts, goals = _pairs(occ, V, 7)
    sw = _swarm(occ, V, steps, replan_distance=5.5, max_replans=1)
    res = sw.run(starts, goals, seeds=np.arange(V), check_every=25)
    replanned = np.flatnonzero(res.replans > 0)
    assert len(replanned) > 0, "the trigger never fired"
    assert res.planned.sum() >= 90
    ok_replans = [v for v in replanned if res.replan_steps[v, 0] > 0]
    assert ok_replans, "no replan produced a new plan"
    for v in np.flatnonzero(res.planned & (res.replans == 0)):
        host = _host_track(res.paths[v], starts[v], goals[v], steps)
        assert res.steps[v] == len(host), v
        np.testing.assert_allclose(res.states[v], host, rtol=0, atol=1e-7)
    kinds = [_check_plan(occ, starts[v], goals[v], v, res.paths[v])  # every initial plan: seed v
             for v in np.flatnonzero(res.planned)]
    assert kinds.count("cr") <= 2, kinds
    for v in ok_replans:
        s = int(res.replan_steps[v, 0])  # steps taken when the replan committed
        host = _host_track(res.paths[v], starts[v], goals[v], s)
        np.testing.assert_allclose(res.states[v][:s], host[:s], rtol=0, atol=1e-7)
        start = res.last_replan_start[v]
        np.testing.assert_array_equal(start, res.states[v][s - 1][:2])  # planned from where it stood
        _check_plan(occ, start, goals[v], replan_seed(v, 0), res.last_replan_path[v])
        cont = _host_continue(res.states[v][s - 1], res.inputs[v][s - 1], res.last_replan_path[v], goals[v],
                              int(res.steps[v]) - s)
        assert len(cont) == int(res.steps[v]) - s, v
        np.testing.assert_allclose(res.states[v][s:], cont, rtol=0, atol=1e-6)
    reached = res.phase == _lib.FLEET_GOAL
    for v in np.flatnonzero(reached):  # goal test of control_stage.py:147-150 on the last state
        assert np.hypot(*(res.states[v][-1, :2] - goals[v])) < 8.0


def test_sharded_swarm_equals_one_swarm(cuda, golden):
    """Config 5 sharded by vehicle (run_swarm_sharded, the multi-GPU path): three ranks emulated in
    one process on one GPU, each running its contiguous block on its own Swarm; the gathered result
    equals the one-Swarm run of all vehicles exactly (steps, phases, replans, every state), with the
    replan trigger live (2.5 px)."""
    from mpcqp.pipeline.swarm import run_swarm_sharded, shard_vehicles

    occ = golden("default_plan.npz")["occupancy"]
    V, world = 40, 3
    starts, goals = _pairs(occ, V, 21)
    one = _swarm(occ, V, 200, replan_distance=2.5).run(starts, goals, seeds=np.arange(V), check_every=25)
    shards = []
    for r in range(world):  # each "rank": its own Swarm sized to its block
        lo, hi = shard_vehicles(V, world, r)
        sw = _swarm(occ, hi - lo, 200, replan_distance=2.5)
        shards.append(run_swarm_sharded(sw.run, starts, goals, np.arange(V), rank=r, world=world,
                                        all_gather_object=lambda out, obj, r=r: out.__setitem__(r, obj),
                                        check_every=25))
    # every rank gathered only its own part here; merging the three reproduces the all-gather
    from mpcqp.pipeline.swarm import merge_swarm_results

    parts = []
    for r in range(world):
        lo, hi = shard_vehicles(V, world, r)
        p = shards[r]
        assert len(p.steps) == hi - lo
        parts.append(p)
    got = merge_swarm_results(parts)
    assert one.replans.sum() > 0, "the trigger should fire at 2.5 px"
    np.testing.assert_array_equal(got.steps, one.steps)
    np.testing.assert_array_equal(got.phase, one.phase)
    np.testing.assert_array_equal(got.replans, one.replans)
    np.testing.assert_array_equal(got.planned, one.planned)
    assert all(np.array_equal(a, b) for a, b in zip(got.states, one.states))


@pytest.mark.parametrize("V,steps,dist,max_replans,seed", [(100, 150, 5.5, 1, 7), (40, 200, 2.5, 2, 21),
                                                           (64, 120, 1.5, 3, 33)])
def test_fused_swarm_equals_stepped_swarm(cuda, golden, V, steps, dist, max_replans, seed):
    """mpcqp_swarm_loop (max_replans + 1 fused-loop launches, the trigger inside the loop) == the
    graph-stepped swarm (mpcqp_swarm_run): every vehicle's states, inputs, phase, steps, replans,
    replan steps, replan start and new plan identical bit for bit, with the trigger firing."""
    starts, goals = _pairs(golden("default_plan.npz")["occupancy"], V, seed)
    occ = golden("default_plan.npz")["occupancy"]
    res = [_swarm(occ, V, steps, replan_distance=dist, max_replans=max_replans, fused=fused)
           .run(starts, goals, seeds=np.arange(V), check_every=25) for fused in (False, True)]
    a, b = res
    assert a.replans.sum() > 0, "the trigger should fire"
    for k in ("steps", "phase", "replans", "planned", "replan_steps", "last_replan_start"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    for v in range(V):
        np.testing.assert_array_equal(a.states[v], b.states[v])
        np.testing.assert_array_equal(a.inputs[v], b.inputs[v])
        pa, pb = a.last_replan_path[v], b.last_replan_path[v]
        assert (pa is None) == (pb is None)
        if pa is not None:
            np.testing.assert_array_equal(pa, pb)
