"""GPU tests of two QPs per wave (k_solve_pair, k_fleet_loop<N, true>; mpcqp_set_pairing).

For horizons N <= 15 a QP has 2N <= 30 variables, so lanes 0-31 and 32-63 of a wave can solve two
QPs.  Every operation of a paired QP is the one-QP-per-wave kernel's on the same values (the
half-wave sums and scans add the same terms in the same order), so the outputs must be equal BIT
FOR BIT to the unpaired kernel's -- status, iteration counters, active sets, u0, X, U -- under
every solver setting (unpolished ADMM iterates at max_iter included), in the batch solve and in the fused closed loop / swarm loop, including odd
batch sizes (a lone QP in the last wave) and a QP with non-finite inputs next to a good one.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_OUTS = ("u0", "X", "U", "status", "iters", "active")


def _solve(params, batch, pairing, **settings):
    import torch

    from mpcqp.control.mpc_controller import BatchedMPCController

    ctrl = BatchedMPCController(params, batch.size, device="cuda:0", pairing=pairing, **settings)
    sol = ctrl.solve_batch(batch.x0, batch.ref, batch.u_prev)
    torch.cuda.synchronize()
    out = {k: getattr(sol, k).cpu().numpy().copy() for k in _OUTS}
    ctrl.close()
    return out


@pytest.mark.parametrize("N", [1, 4, 10, 15])
@pytest.mark.parametrize("variant", ["default", "osqp_settings", "max_iter_50", "newton"])
def test_pair_batch_equals_one_qp_per_wave_bitwise(cuda, N, variant):
    from mpcqp import scenarios
    from mpcqp.config import MPCConfig

    settings = {"default": {}, "osqp_settings": {"scaling": 10, "polish_from": 0, "polish_near": 0.0},
                "max_iter_50": {"max_iter": 50, "polish_from": 0, "polish_near": 0.0},
                "newton": {"method": "newton"}}[variant]
    batch = scenarios.config3(257, horizon=N)  # odd: the last wave holds one QP
    if variant == "default":  # non-finite inputs in one half of a wave, a good QP in the other
        batch.x0[6, 0] = np.nan
    params = MPCConfig(horizon=N).to_parameters(0.8)
    one = _solve(params, batch, "off", **settings)
    two = _solve(params, batch, "on", **settings)
    for k in _OUTS:
        # unpolished ADMM iterates (max_iter_50) included: the kernels contract multiply-adds only
        # within a source expression (-ffp-contract=on), so both variants round the same way
        np.testing.assert_array_equal(one[k], two[k], err_msg=k)
    if variant == "default":
        assert one["status"][6] == -10 and one["status"][7] == 1
    if variant in ("default", "osqp_settings"):
        assert (one["status"][np.arange(257) != 6] == 1).all()


def test_pair_auto_pairs_past_the_wave_slots(cuda):
    """"auto": a batch with more QPs than wave slots (8 per CU) runs paired, a smaller one unpaired;
    both equal the forced modes bit for bit."""
    import torch

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    N = 12
    params = MPCConfig(horizon=N).to_parameters(0.8)
    for B in (8 * cus - 1, 8 * cus + 3):
        batch = scenarios.config3(B, horizon=N)
        auto = _solve(params, batch, "auto")
        forced = _solve(params, batch, "on" if B > 8 * cus else "off")
        for k in _OUTS:
            np.testing.assert_array_equal(auto[k], forced[k], err_msg=(B, k))


_LOOP_BUFFERS = ("state", "u_prev", "path_idx", "phase", "steps", "trace", "u_trace", "X", "status", "u0")


@pytest.mark.parametrize("N,V,steps,seed,settings", [(15, 41, 80, 3, {}), (10, 64, 60, 11, {}),
                                                      (15, 41, 80, 7, {"max_iter": 30, "polish": 0,
                                                                        "polish_from": 0, "polish_near": 0.0})])
def test_pair_fused_loop_equals_stepped_loop_bitwise(cuda, golden, N, V, steps, seed, settings):
    """The fused closed loop with two vehicles per wave (k_fleet_loop<N, true>: each half its own
    loop state and control flow; an odd fleet leaves the last wave one vehicle) == the graph-stepped
    loop, every buffer bit for bit -- also with the polish off and ADMM capped at 30 iterations, where
    unpolished ADMM iterates drive the plant."""
    from test_gpu_fleet import _tracker, _varied_fleet

    g, paths, starts, goals = _varied_fleet(golden, V, seed=seed)
    bufs = []
    for fused, pairing in ((False, "off"), (True, "on")):
        ft = _tracker(N, V, 128, steps, fused=fused, **settings)
        for c in (ft._nominal, ft._relaxed):
            c.set_pairing(pairing)
        ft.reset_from_plans(paths, starts, goals)
        res = ft.run()
        bufs.append({k: ft.buffers()[k].cpu().numpy().copy() for k in _LOOP_BUFFERS})
        ft.close()
    for k in _LOOP_BUFFERS:
        np.testing.assert_array_equal(bufs[0][k], bufs[1][k], err_msg=k)
    assert (res.phase != 0).any()
    if settings:  # unpolished solves drove the plant for many steps
        assert (bufs[0]["steps"] > 20).any()


def test_pair_fused_swarm_equals_stepped_swarm(cuda, golden):
    """The fused swarm loop (trigger inside the loop) with two vehicles per wave == the stepped swarm,
    with replans firing."""
    from test_gpu_swarm import _pairs, _swarm

    V, steps = 40, 200
    occ = golden("default_plan.npz")["occupancy"]
    starts, goals = _pairs(occ, V, 21)
    res = [_swarm(occ, V, steps, replan_distance=2.5, max_replans=2, fused=fused, pairing=pairing)
           .run(starts, goals, seeds=np.arange(V), check_every=25)
           for fused, pairing in ((False, "off"), (True, "on"))]
    a, b = res
    assert a.replans.sum() > 0, "the trigger should fire"
    for k in ("steps", "phase", "replans", "planned", "replan_steps", "last_replan_start"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    for v in range(V):
        np.testing.assert_array_equal(a.states[v], b.states[v])
        np.testing.assert_array_equal(a.inputs[v], b.inputs[v])
