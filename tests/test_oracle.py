"""CPU tests of the oracle itself, pinned to the reference's golden vectors (tests/golden/).

The oracle is the parity reference for the GPU path, so it is checked first:
  * its vehicle model against the reference's f_discrete / linearize outputs,
  * its QP against the reference's own known-answer test (tests/test_mpc_controller.py)
    and against an independent solver (scipy trust-constr) on the un-condensed formulation,
  * its closed loop against the reference TrajectoryTracker's own loop,
  * the C restatement (CPU baseline) against the numpy exact solve.
"""
from __future__ import annotations

import numpy as np
import pytest

import mpc_oracle as mo


def test_vehicle_model_matches_reference_golden(golden):
    g = golden("vehicle.npz")
    for i in range(len(g["x"])):
        fd = mo.f_discrete(g["x"][i], g["u"][i], g["dt"][i], g["L"][i])
        A, B, fx = mo.linearize(g["x"][i], g["u"][i], g["dt"][i], g["L"][i])
        np.testing.assert_array_equal(fd, g["f_discrete"][i])
        np.testing.assert_array_equal(A, g["A"][i])
        np.testing.assert_array_equal(B, g["B"][i])
        np.testing.assert_array_equal(fx, g["fx"][i])


def test_reference_known_answer_case():
    """tests/test_mpc_controller.py:7-17 of the reference (MPCConfig(horizon=5), res 0.2)."""
    p = mo.default_params(horizon=5, map_resolution=0.2)
    x0 = np.array([0.0, 0.0, 0.0, 5.0])
    ref = np.tile(np.array([1.0, 0.0, 0.0, 5.0]), (6, 1))
    sol = mo.solve_exact(p, x0, ref)
    assert sol.converged
    assert sol.X[0, 1] > x0[0]  # the reference's assertion
    np.testing.assert_allclose(sol.Umat[:, 0], [-9.1046224514, 0.0], atol=1e-9)
    np.testing.assert_allclose(sol.X[0, 1], 0.5, atol=1e-12)


def _random_case(rng, N):
    plan_ref = np.column_stack([np.linspace(0, 30, N + 1), np.linspace(0, 5, N + 1),
                                np.linspace(0.0, 0.8, N + 1), np.full(N + 1, 12.0)])
    x0 = plan_ref[0] + rng.normal(0, 1, 4) * [2, 2, 0.3, 3]
    return x0, plan_ref, rng.normal(0, 1, 2) * [3, 0.05]


def _trust_constr(P, q, A, lo, hi, n):
    """scipy trust-constr from zero with sparse P and A (its sparse factorisations keep N = 30
    to seconds; dense, the same run takes minutes)."""
    import scipy.sparse as sp
    from scipy.optimize import LinearConstraint, minimize

    Ps, As = sp.csr_matrix(P), sp.csr_matrix(A)
    return minimize(lambda v: 0.5 * v @ (Ps @ v) + q @ v, np.zeros(n), jac=lambda v: Ps @ v + q,
                    hess=lambda v: Ps, method="trust-constr", constraints=[LinearConstraint(As, lo, hi)],
                    options=dict(gtol=1e-12, xtol=1e-14, maxiter=6000))


@pytest.mark.parametrize("seed", [0, 1])
def test_condensed_solution_solves_full_formulation(seed):
    """The condensed solution, lifted to the cvxpy variable vector (11N+5), is feasible for
    the un-condensed QP of mpc_controller.py:53-117, attains the same objective, and agrees
    with scipy's trust-constr on that formulation."""
    rng = np.random.default_rng(seed)
    N = 5
    p = mo.default_params(N)
    x0, ref, up = _random_case(rng, N)
    sol = mo.solve_exact(p, x0, ref, up)
    P, q, r0, A, lo, hi, lay = mo.full_qp(p, x0, ref, up)
    assert lay["n"] == 11 * N + 5 and A.shape[0] == 19 * N + 7
    xs = mo.lift(p, sol, up)
    z = A @ xs
    assert np.all(z >= lo - 1e-9) and np.all(z <= hi + 1e-9)
    np.testing.assert_allclose(0.5 * xs @ P @ xs + q @ xs + r0, sol.objective, rtol=1e-12)
    res = _trust_constr(P, q, A, lo, hi, xs.size)
    assert np.abs(res.x[lay["oU"]: lay["oSv"]] - xs[lay["oU"]: lay["oSv"]]).max() < 1e-4
    assert 0.5 * res.x @ P @ res.x + q @ res.x + r0 >= sol.objective - 1e-9


def _pinned_cases():
    """(N, x0, window, u_prev): windows of the reference's own closed loop (closed_loop.npz) at
    N = 10 and 15, a config-3 sample at N = 20 and a config-4 sample at N = 30."""
    from pathlib import Path

    from mpcqp import scenarios

    d = np.load(Path(__file__).resolve().parent / "golden" / "closed_loop.npz")
    c3 = scenarios.config3(64, horizon=20)
    c4 = scenarios.config4(64, horizon=30)
    return [
        (10, d["N10_x0"][0], d["N10_window"][0], d["N10_u_prev"][0]),
        (10, d["N10_x0"][30], d["N10_window"][30], d["N10_u_prev"][30]),
        (15, d["N15_x0"][12], d["N15_window"][12], d["N15_u_prev"][12]),
        (15, d["N15_x0"][50], d["N15_window"][50], d["N15_u_prev"][50]),
        (20, c3.x0[5], c3.ref[5], c3.u_prev[5]),
        (20, c3.x0[41], c3.ref[41], c3.u_prev[41]),
        (30, c4.x0[3], c4.ref[3], c4.u_prev[3]),
        (30, c4.x0[17], c4.ref[17], c4.u_prev[17]),
    ]


@pytest.mark.parametrize("case", range(8))
def test_exact_solution_has_kkt_certificate_on_full_formulation(case):
    """Independent optimality certificate on the reference's un-condensed QP (11N+5 variables,
    19N+7 rows of mpc_controller.py:53-117): the lifted exact solution is feasible and there are
    multipliers with the right signs on its active rows (bounded least squares, scipy) that make
    the Lagrangian stationary.  A strictly convex QP has exactly one such point."""
    from scipy.optimize import lsq_linear

    N, x0, ref, up = _pinned_cases()[case]
    p = mo.default_params(N)
    sol = mo.solve_exact(p, x0, ref, up)
    assert sol.converged
    P, q, r0, A, lo, hi, lay = mo.full_qp(p, x0, ref, up)
    xs = mo.lift(p, sol, up)
    z = A @ xs
    tol = 1e-9 * np.maximum(1.0, np.abs(z))
    assert np.all(z >= lo - tol) and np.all(z <= hi + tol)
    eq = lo == hi
    at_hi = ~eq & np.isfinite(hi) & (np.abs(z - hi) <= tol)
    at_lo = ~eq & np.isfinite(lo) & (np.abs(z - lo) <= tol)
    act = eq | at_hi | at_lo
    # L = f + y'(Ax): y >= 0 on rows at their upper bound, y <= 0 at the lower bound
    lb = np.where(at_hi[act], 0.0, -np.inf)
    ub = np.where(at_lo[act], 0.0, np.inf)
    g = P @ xs + q
    fit = lsq_linear(A[act].T, -g, bounds=(lb, ub), lsmr_tol="auto", method="bvls")
    stat = np.abs(A[act].T @ fit.x + g).max()
    assert stat <= 1e-8 * max(1.0, np.abs(g).max()), f"N={N}: stationarity residual {stat:.3e}"


@pytest.mark.parametrize("case", range(8))
def test_exact_solution_matches_trust_constr(case):
    """scipy trust-constr (an interior-point solver, nothing shared with the oracle) on the
    un-condensed formulation at N = 10, 15, 20, 30 agrees with the exact solve's inputs to 2e-6
    and cannot beat its objective (SURVEY.md §8c3 ii)."""
    N, x0, ref, up = _pinned_cases()[case]
    p = mo.default_params(N)
    sol = mo.solve_exact(p, x0, ref, up)
    P, q, r0, A, lo, hi, lay = mo.full_qp(p, x0, ref, up)
    xs = mo.lift(p, sol, up)
    res = _trust_constr(P, q, A, lo, hi, xs.size)
    dU = np.abs(res.x[lay["oU"]: lay["oSv"]] - xs[lay["oU"]: lay["oSv"]]).max()
    # an interior-point method stops ~1e-6 relative short of the optimum (the tight pin is the KKT
    # certificate above); 2e-6 covers all eight windows
    assert dU <= 2e-6 * max(1.0, np.abs(xs[lay["oU"]: lay["oSv"]]).max()), f"N={N}: |dU| {dU:.3e}"
    assert 0.5 * res.x @ P @ res.x + q @ res.x + r0 >= sol.objective - 1e-9 * max(1.0, abs(sol.objective))


def test_exact_solution_is_stationary():
    rng = np.random.default_rng(5)
    for N in (5, 10, 20):
        p = mo.default_params(N)
        x0, ref, up = _random_case(rng, N)
        qp = mo.condense(p, x0, ref, up)
        U, codes, its, ok = mo.solve_condensed(qp)
        assert ok
        assert np.abs(mo.gradient(qp, U)).max() <= 1e-9 * max(1.0, np.abs(qp.g).max())


def test_closed_loop_matches_reference_loop(golden):
    """The oracle's restatement of control_stage.py:84-150, driven by the exact solve,
    reproduces the reference TrajectoryTracker's own loop (captured in closed_loop.npz)."""
    plan = golden("default_plan.npz")
    loop = golden("closed_loop.npz")
    for N in (10, 15):
        p = mo.default_params(N, float(plan["map_resolution"]))
        rec: list = []
        states = mo.track_loop(p, plan[f"ref_global_N{N}"], plan["start"], float(plan["yaw0"]), plan["goal"],
                               100 if N == 10 else 300, record=rec)
        ref_states = loop[f"N{N}_states"]
        assert len(states) == len(ref_states) == 65
        np.testing.assert_allclose(np.asarray(states), ref_states, rtol=0, atol=1e-9)
        np.testing.assert_allclose(np.asarray([r[1] for r in rec]), loop[f"N{N}_window"], rtol=0, atol=1e-12)
        np.testing.assert_allclose(np.asarray([r[2] for r in rec]), loop[f"N{N}_u_prev"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("cfg,B", [("config2", 4), ("config3", 96), ("config4", 48)])
def test_c_restatement_matches_exact_oracle(cfg, B):
    import cpu_solver
    from mpcqp import scenarios

    batch = getattr(scenarios, cfg)(B)
    p = mo.default_params(batch.horizon)
    for method in (0, 1):
        out = cpu_solver.cpu_solve(p, batch.x0, batch.ref, batch.u_prev, method=method, nthreads=4)
        assert (out["status"] == 1).all()
        for b in range(B):
            ex = mo.solve_exact(p, batch.x0[b], batch.ref[b], batch.u_prev[b])
            err = np.abs(out["U"][b] - ex.Umat).max() / max(1.0, np.abs(ex.Umat).max())
            assert err <= 1e-9, (b, err)
            np.testing.assert_array_equal(out["active"][b], ex.active)


def test_c_restatement_unwrap_is_numpy_bit_exact(golden):
    """The C build step's np.unwrap against numpy on the golden edge cases (exact +-pi jumps)."""
    import cpu_solver

    g = golden("unwrap.npz")
    p = mo.default_params(30)
    for i, L in enumerate(g["lens"]):
        N = int(L) - 1
        pN = mo.default_params(N)
        ref = np.zeros((1, N + 1, 4))
        ref[0, :, 2] = g["p"][i, :L]
        ref[0, :, 3] = 10.0
        out = cpu_solver.cpu_solve(pN, np.zeros((1, 4)), ref, None, want_model=True)
        yaw = out["model"][0, 7 * N + 2: 7 * N + 2 + 4 * (N + 1): 4]
        np.testing.assert_array_equal(yaw, g["unwrapped"][i, :L])
    assert p.horizon == 30


def test_rrt_oracle_reproduces_reference_trees(golden):
    """oracle/rrt_oracle.grow_tree with the planner's own sample stream == the reference's
    RRTStarPlanner trees (planning.npz, generated from the reference), bit for bit."""
    import rrt_oracle as ro
    from mpcqp.planning.rrt_star import default_planner_parameters, draw_samples

    g = golden("planning.npz")
    occ = g["rrt_occupancy"]
    prm = default_planner_parameters()
    for k in range(5):
        sx, sy, gx, gy, seed, iters = g[f"rrt{k}_case"]
        smp = draw_samples(int(seed), (gx, gy), occ.shape, prm.goal_sample_rate, int(iters))
        nodes, it, gi = ro.grow_tree(occ, (sx, sy), (gx, gy), smp, step=prm.step, goal_radius=prm.goal_radius,
                                     rewire_radius=prm.rewire_radius, collision_step=prm.collision_step)
        np.testing.assert_array_equal(nodes, g[f"rrt{k}_nodes"])
        assert [int(g[f"rrt{k}_meta"][0]), it, gi] == [int(gi >= 0), *map(int, g[f"rrt{k}_meta"][1:])]


def test_correctly_rounded_trig_oracle(golden):
    """rrt_oracle.cr_*: the exact (decimal) correctly rounded steer trig.  Within an ulp of glibc's
    and equal to it on >= 99 % of arguments; a rounding-error-free identity holds exactly; and the
    reference's own trees (planning.npz) come out bit for bit the same with it -- the device's
    trig (correctly rounded) can match the reference wherever glibc rounds correctly."""
    import math

    import rrt_oracle as ro
    from mpcqp.planning.rrt_star import default_planner_parameters, draw_samples

    rng = np.random.default_rng(4)
    t = rng.uniform(-math.pi, math.pi, 3000)
    for f, g in ((ro.cr_cos, math.cos), (ro.cr_sin, math.sin)):
        a = np.array([f(v) for v in t])
        b = np.array([g(v) for v in t])
        assert (a == b).mean() >= 0.99
        assert np.all(np.abs(a - b) <= np.spacing(np.abs(b)))
    y, x = rng.uniform(-80, 80, (2, 3000))
    a = np.array([ro.cr_atan2(p, q) for p, q in zip(y, x)])
    b = np.array([math.atan2(p, q) for p, q in zip(y, x)])
    assert (a == b).mean() >= 0.99 and np.all(np.abs(a - b) <= np.spacing(np.abs(b)))
    assert ro.cr_atan2(1.0, 1.0) == math.pi / 4 and ro.cr_cos(0.0) == 1.0 and ro.cr_atan2(0.0, -1.0) == math.pi
    g = golden("planning.npz")
    occ = g["rrt_occupancy"]
    prm = default_planner_parameters()
    for k in range(5):
        sx, sy, gx, gy, seed, iters = g[f"rrt{k}_case"]
        smp = draw_samples(int(seed), (gx, gy), occ.shape, prm.goal_sample_rate, int(iters))
        nodes, it, gi = ro.grow_tree(occ, (sx, sy), (gx, gy), smp, step=prm.step, goal_radius=prm.goal_radius,
                                     rewire_radius=prm.rewire_radius, collision_step=prm.collision_step,
                                     trig=ro.CR_TRIG)
        np.testing.assert_array_equal(nodes, g[f"rrt{k}_nodes"])


def test_inflation_oracle_reproduces_reference(golden):
    import rrt_oracle as ro

    g = golden("planning.npz")
    np.testing.assert_array_equal(ro.dilate(g["inflate_default_in"], int(g["inflate_default_radius"])),
                                  g["inflate_default_out"])
    for k, r in enumerate(g["inflate_random_radius"]):
        np.testing.assert_array_equal(ro.dilate(g["inflate_random_in"][k], int(r)), g["inflate_random_out"][k])
