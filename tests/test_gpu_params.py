"""GPU parity over the MPCParameters block, not just its defaults.

Every field of ``MPCParameters`` (``src/control/mpc_controller.py:17-30``) changes the QP the
reference hands to OSQP (``:53-117``): a symmetric non-diagonal Q / Q_N (cvxpy's quad_form takes
only symmetric matrices), R with an off-diagonal term, dt, the wheelbase, tightened bounds,
slack weights x10 and /10, and the relaxed du_bounds of ``control_stage.py:50-56``.  Each variant
runs through the C-ABI at N = 10, 20, 30 against the exact oracle (``mpc_oracle.solve_exact``,
which condenses the reference's acceleration form independently of the kernel's speed form):
U, X, u0 to 1e-8 relative, identical active sets.

The retry branch of ``_solve_with_relaxation`` (``control_stage.py:43-56``) is exercised where
the nominal solve fails and the relaxed one succeeds: a nominal workspace limited to one ADMM
iteration without polish (status max_iter) and a relaxed one with the defaults -- host tracker
and device fleet both return the oracle's optimum of the relaxed problem on the 0.6-scaled window.
"""
from __future__ import annotations

import numpy as np
import pytest
from param_variants import VARIANTS

pytestmark = pytest.mark.gpu

REL_TOL = 1e-8
FAIL_NOMINAL = dict(max_iter=1, polish=0, polish_from=0, polish_near=0.0)


def _base(N, res=0.8):
    from mpcqp.config import MPCConfig

    return MPCConfig(horizon=N).to_parameters(res)


def _variant(name, N):
    from param_variants import resolution, variant

    return variant(_base(N, resolution(name)), name)


def _solve(params, x0, ref, u_prev, **settings):
    import torch
    from mpcqp.control.mpc_controller import BatchedMPCController

    ctrl = BatchedMPCController(params, len(x0), device="cuda:0", **settings)
    sol = ctrl.solve_batch(x0, ref, u_prev)
    torch.cuda.synchronize()
    out = {k: getattr(sol, k).cpu().numpy().copy() for k in sol._fields}
    ctrl.close()
    return out


def _rel(a, b):
    return float(np.abs(a - b).max() / max(1.0, np.abs(b).max()))


@pytest.mark.parametrize("N", [10, 20, 30])
@pytest.mark.parametrize("name", VARIANTS)
def test_parameter_block_matches_exact_oracle(cuda, name, N):
    import mpc_oracle as mo
    from mpcqp import scenarios

    params = _variant(name, N)
    batch = scenarios.config3(48, horizon=N, seed=1000 + N)
    out = _solve(params, batch.x0, batch.ref, batch.u_prev)
    assert (out["status"] == 1).all(), np.unique(out["status"], return_counts=True)
    n_active = 0
    for b in range(batch.size):
        ex = mo.solve_exact(params, batch.x0[b], batch.ref[b], batch.u_prev[b])
        assert ex.converged
        e = max(_rel(out["U"][b], ex.Umat), _rel(out["X"][b], ex.X), _rel(out["u0"][b], ex.Umat[:, 0]))
        assert e <= REL_TOL, f"{name} N={N} QP {b}: rel err {e:.3e}"
        assert np.array_equal(out["active"][b], ex.active), f"{name} N={N} QP {b}: active set differs"
        n_active += int((ex.active != 0).any())
    assert n_active > 0  # the variant's soft rows are exercised


def test_parameter_block_matches_c_restatement(cuda):
    """The same variants at N=20 against the C restatement: same statuses, same active sets."""
    import cpu_solver
    from mpcqp import scenarios

    batch = scenarios.config3(128, horizon=20, seed=77)
    for name in VARIANTS:
        params = _variant(name, 20)
        out = _solve(params, batch.x0, batch.ref, batch.u_prev)
        ref = cpu_solver.cpu_solve(params, batch.x0, batch.ref, batch.u_prev)
        assert np.array_equal(out["status"], ref["status"]), name
        assert np.array_equal(out["active"], ref["active"]), name
        assert _rel(out["U"], ref["U"]) <= REL_TOL, name


def test_max_iter_status_follows_osqp(cuda):
    """At max_iter the solve reports solved_inaccurate when the iterate passes OSQP's
    approximate test (eps x10, no polish) and max_iter_reached otherwise -- as the C restatement."""
    import cpu_solver
    from mpcqp import scenarios

    batch = scenarios.config3(256, horizon=20, seed=5)
    params = _base(20)
    seen = set()
    for max_iter in (1, 30, 60, 100):
        st = dict(max_iter=max_iter, polish_from=0, polish_near=0.0)
        out = _solve(params, batch.x0, batch.ref, batch.u_prev, **st)
        ref = cpu_solver.cpu_solve(params, batch.x0, batch.ref, batch.u_prev, **st)
        agree = (out["status"] == ref["status"]).mean()
        assert agree >= 0.99, (max_iter, agree)
        seen |= set(np.unique(out["status"]).tolist())
    assert {-2, 1, 2} <= seen, seen


def _window_case(N=15, k=12):
    """A window of the reference's own closed loop (closed_loop.npz, N=15)."""
    from pathlib import Path

    d = np.load(Path(__file__).resolve().parent / "golden" / "closed_loop.npz")
    return d[f"N{N}_x0"][k], d[f"N{N}_window"][k], d[f"N{N}_u_prev"][k]


def test_relaxed_retry_succeeds_host(cuda):
    """control_stage.py:43-56 on the drop-in tracker: the nominal solve fails (one ADMM iteration,
    no polish), the relaxed one returns the exact optimum of the relaxed QP on the 0.6-scaled window."""
    import mpc_oracle as mo
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.control.mpc_controller import MPCController
    from mpcqp.pipeline.control_stage import TrajectoryTracker
    from mpcqp.pipeline.fleet import relaxed_parameters

    x0, window, up = _window_case()
    params = MPCConfig(horizon=15).to_parameters(0.8)
    assert MPCController(params, **FAIL_NOMINAL).solve(x0, window, u_prev=up) == (None, None, None)
    tr = TrajectoryTracker(MPCConfig(horizon=15), VizConfig(), solver_settings=FAIL_NOMINAL)
    u0, X, U = tr._solve_with_relaxation(x0, window, up, params)
    assert u0 is not None
    w6 = np.array(window, copy=True)
    w6[:, 3] *= 0.6
    ex = mo.solve_exact(relaxed_parameters(params), x0, w6, up)
    assert _rel(U, ex.Umat) <= REL_TOL and _rel(X, ex.X) <= REL_TOL
    # and the relaxed optimum differs from the nominal one (the retry changed the answer)
    nom = mo.solve_exact(params, x0, window, up)
    assert _rel(U, nom.Umat) > 1e-3


@pytest.mark.parametrize("fused", [False, True])
def test_relaxed_retry_succeeds_fleet(cuda, fused):
    """The same branch in the device fleet (k_fleet_build relax=1 + the relaxed workspace): one
    step of 8 vehicles whose nominal workspace cannot solve; applied input and next state equal
    the oracle's relaxed optimum and f_discrete."""
    import mpc_oracle as mo
    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.ref_builder import build_reference
    from mpcqp.pipeline.fleet import FleetTracker, initial_state, relaxed_parameters

    N = 15
    paths, starts, goals = scenarios.fleet5(8, seed=11)
    mpc = MPCConfig(horizon=N, sim_steps=3)
    ft = FleetTracker(mpc, map_resolution=0.8, max_vehicles=8, max_ref_len=160, device="cuda:0",
                      use_graph=False, fused=fused, relaxed_settings={}, **FAIL_NOMINAL)
    refs = ft.reset_from_plans(paths, starts, goals)
    ft.step(1)
    res = ft.result()
    st = ft.buffers()["status"].cpu().numpy()
    assert (st[0] == -2).all() and (st[1] == 1).all(), st
    params = mpc.to_parameters(0.8)
    rp = relaxed_parameters(params)
    for v in range(8):
        w = scenarios.window(refs[v], 0, N).copy()
        w[:, 3] *= 0.6
        s0 = initial_state(paths[v], starts[v])
        ex = mo.solve_exact(rp, s0, w, np.zeros(2))
        assert _rel(res.inputs[v][0], ex.Umat[:, 0]) <= REL_TOL
        nxt = mo.f_discrete(s0, res.inputs[v][0], params.dt, params.wheelbase_px)
        np.testing.assert_allclose(res.states[v][0], nxt, rtol=0, atol=1e-9)
    ft.close()
