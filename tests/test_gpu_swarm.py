"""GPU tests of the config-5 swarm (mpcqp/pipeline/swarm.py): batched RRT* plans, device
references, fleet closed loop and the replan trigger, end to end on the default inflated grid.

Between replans every vehicle follows the reference's single-vehicle loop: a vehicle that was
never replanned reproduces TrajectoryTracker.track on its own plan (1e-7 px), and its plan is
the reference planner's (RRTStarPlanner with that vehicle's seed)."""
from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


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


def _swarm(occ, V, sim_steps, **kw):
    from mpcqp.config import MPCConfig
    from mpcqp.pipeline.swarm import Swarm
    from mpcqp.planning.rrt_star import default_planner_parameters

    return Swarm(occ, MPCConfig(horizon=15, sim_steps=sim_steps), default_planner_parameters(max_iterations=1500),
                 map_resolution=0.8, max_vehicles=V, device="cuda:0", **kw)


def test_swarm_vehicles_follow_the_reference_loop(cuda, golden):
    from mpcqp import _lib
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker
    from mpcqp.planning.rrt_star import RRTStarPlanner, default_planner_parameters

    occ = golden("default_plan.npz")["occupancy"]
    V, steps = 24, 120
    starts, goals = _pairs(occ, V, 1)
    sw = _swarm(occ, V, steps, replan_distance=1e9)  # no replans: the plain per-vehicle loop
    res = sw.run(starts, goals, seeds=np.arange(V), check_every=20)
    assert (res.replans == 0).all()
    assert res.planned.mean() > 0.8
    tracker = TrajectoryTracker(MPCConfig(horizon=15, sim_steps=steps), VizConfig())
    for v in np.flatnonzero(res.planned)[:6]:
        plan = RRTStarPlanner(occ, default_planner_parameters(max_iterations=1500, random_seed=int(v))).plan(
            tuple(starts[v]), tuple(goals[v]))
        assert plan.success
        host = np.asarray(tracker.track(SimpleNamespace(plan=plan), SimpleNamespace(start=tuple(starts[v]),
                                        goal=tuple(goals[v])), map_resolution=0.8, visualize=False).states)
        assert res.steps[v] == len(host)
        np.testing.assert_allclose(res.states[v], host, rtol=0, atol=1e-7)
    done = res.phase[res.planned]
    assert np.isin(done, [_lib.FLEET_GOAL, _lib.FLEET_OUT_OF_STEPS]).all()


def test_replan_trigger(cuda, golden):
    """A tight off-track threshold forces replans: replanned vehicles get a fresh reference
    from where they stand and keep tracking; every vehicle ends in a terminal phase or runs on."""
    from mpcqp import _lib

    occ = golden("default_plan.npz")["occupancy"]
    V = 32
    starts, goals = _pairs(occ, V, 2)
    sw = _swarm(occ, V, 150, replan_distance=4.0, max_replans=2)
    res = sw.run(starts, goals, seeds=np.arange(V), check_every=10)
    assert res.replans.sum() > 0
    assert (res.replans <= 2).all()
    reached = res.phase == _lib.FLEET_GOAL
    assert reached.sum() >= 0.5 * res.planned.sum()
    for v in np.flatnonzero(reached):  # goal test of control_stage.py:147-150 on the last state
        assert np.hypot(*(res.states[v][-1, :2] - goals[v])) < 8.0
