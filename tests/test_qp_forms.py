"""The oracle's QP against the QP the reference's OWN code assembles (``qp_forms.npz``).

``tests/golden/gen_qp_forms.py`` ran the reference's unmodified ``MPCController.solve``
(``/root/reference/src/control/mpc_controller.py:53-132``) on a recording cvxpy module and stored
the standard form ``0.5 x'Px + q'x + r0, l <= Ax <= u`` it states: 189 QPs -- the 130 windows of
the reference's closed loop at N = 10/15, config-3/4 samples at N = 20/30 and the nine parameter
variants at N = 10/20/30.  ``mpc_oracle.full_qp`` (the restatement every parity test relies on)
must reproduce it element for element, and the exact optimum the GPU is checked against must carry
a KKT certificate on the reference's own matrices.
"""
from __future__ import annotations

import json

import numpy as np
import pytest

import mpc_oracle as mo
from param_variants import resolution, variant


@pytest.fixture(scope="module")
def forms(golden):
    return golden("qp_forms.npz")


def _case(g, i):
    N = int(g["horizon"][i])
    n, m = int(g["col_off"][i + 1] - g["col_off"][i]), int(g["row_off"][i + 1] - g["row_off"][i])
    P = np.zeros((n, n))
    s = slice(g["P_off"][i], g["P_off"][i + 1])
    P[g["P_i"][s], g["P_j"][s]] = g["P_v"][s]
    A = np.zeros((m, n))
    s = slice(g["A_off"][i], g["A_off"][i + 1])
    A[g["A_i"][s], g["A_j"][s]] = g["A_v"][s]
    cols = slice(g["col_off"][i], g["col_off"][i + 1])
    rows = slice(g["row_off"][i], g["row_off"][i + 1])
    name = str(g["variants"][i])
    p = mo.default_params(N, resolution(name) if name != "default" else 0.8)
    if name != "default":
        p = variant(p, name)
    window = g["window"][g["window_off"][i]: g["window_off"][i + 1]].reshape(N + 1, 4)
    return dict(N=N, P=P, q=g["q"][cols], r0=float(g["r0"][i]), A=A, l=g["l"][rows], u=g["u"][rows], params=p,
                x0=g["x0"][i], window=window, u_prev=g["u_prev"][i], tag=str(g["tags"][i]))


def test_fixture_covers_the_promised_cases(forms):
    tags = [str(t) for t in forms["tags"]]
    assert len(tags) == 189
    assert sum(t.startswith("loop_N10_") for t in tags) == 65 and sum(t.startswith("loop_N15_") for t in tags) == 65
    assert {str(v) for v in forms["variants"]} >= {"q_nondiag", "tight_bounds", "relaxed_du", "default"}
    assert set(forms["horizon"].tolist()) == {10, 15, 20, 30}


def test_oracle_full_qp_equals_reference_assembly(forms):
    """Every matrix and bound of ``full_qp`` equals the reference's, row for row (rounding aside:
    the constant r0 is summed in a different order)."""
    for i in range(len(forms["tags"])):
        c = _case(forms, i)
        P, q, r0, A, lo, hi, lay = mo.full_qp(c["params"], c["x0"], c["window"], c["u_prev"])
        assert P.shape == c["P"].shape and A.shape == c["A"].shape, c["tag"]
        np.testing.assert_allclose(P, c["P"], rtol=1e-15, atol=0, err_msg=c["tag"])
        np.testing.assert_allclose(A, c["A"], rtol=1e-15, atol=0, err_msg=c["tag"])
        np.testing.assert_allclose(q, c["q"], rtol=1e-14, atol=1e-14, err_msg=c["tag"])
        np.testing.assert_array_equal(np.isinf(lo), np.isinf(c["l"]), err_msg=c["tag"])
        np.testing.assert_array_equal(np.isinf(hi), np.isinf(c["u"]), err_msg=c["tag"])
        np.testing.assert_allclose(lo, c["l"], rtol=1e-15, atol=1e-15, err_msg=c["tag"])
        np.testing.assert_allclose(hi, c["u"], rtol=1e-15, atol=1e-15, err_msg=c["tag"])
        assert abs(r0 - c["r0"]) <= 1e-12 * max(1.0, abs(c["r0"])), c["tag"]


def test_reference_solver_settings_are_the_products(forms):
    """The OSQP keyword arguments the reference passes (mpc_controller.py:121-131) are the
    product's defaults."""
    from mpcqp import _lib

    kw = json.loads(str(forms["solve_kwargs"]))
    d = _lib.DEFAULT_SOLVER_SETTINGS
    assert kw["solver"] == "OSQP" and kw["warm_start"] is True and kw["verbose"] is False
    for k in ("eps_abs", "eps_rel", "max_iter", "rho", "alpha"):
        assert kw[k] == d[k], k
    assert bool(kw["polish"]) == bool(d["polish"]) and bool(kw["adaptive_rho"]) == bool(d["adaptive_rho"])


@pytest.mark.parametrize("stride", [0, 1, 2])
def test_exact_optimum_is_kkt_on_reference_matrices(forms, stride):
    """The exact optimum (the GPU's parity target), lifted to the reference's variables, is feasible
    and stationary with correctly signed multipliers on the reference's own (P, q, A, l, u): the
    unique optimum of the problem the reference states.  Every parameter variant, and every 8th
    closed-loop / config case."""
    from scipy.optimize import lsq_linear

    idx = [i for i, v in enumerate(forms["variants"]) if str(v) != "default"]
    idx += [i for i, v in enumerate(forms["variants"]) if str(v) == "default"][::8]
    for i in idx[stride::3]:
        c = _case(forms, i)
        sol = mo.solve_exact(c["params"], c["x0"], c["window"], c["u_prev"])
        assert sol.converged, c["tag"]
        xs = mo.lift(c["params"], sol, c["u_prev"])
        z = c["A"] @ xs
        tol = 1e-9 * np.maximum(1.0, np.abs(z))
        assert np.all(z >= c["l"] - tol) and np.all(z <= c["u"] + tol), c["tag"]
        eq = c["l"] == c["u"]
        at_hi = ~eq & np.isfinite(c["u"]) & (np.abs(z - c["u"]) <= tol)
        at_lo = ~eq & np.isfinite(c["l"]) & (np.abs(z - c["l"]) <= tol)
        act = eq | at_hi | at_lo
        g = c["P"] @ xs + c["q"]
        fit = lsq_linear(c["A"][act].T, -g, bounds=(np.where(at_hi[act], 0.0, -np.inf),
                                                     np.where(at_lo[act], 0.0, np.inf)),
                         lsmr_tol="auto", method="bvls")
        stat = np.abs(c["A"][act].T @ fit.x + g).max()
        assert stat <= 1e-8 * max(1.0, np.abs(g).max()), f"{c['tag']}: stationarity residual {stat:.3e}"


def test_ruiz_passes_do_not_change_the_polished_optimum(forms):
    """This build runs one Ruiz pass by default where OSQP runs 10.  On every one of
    the reference's 189 QPs both settings end polished (status 1) at the same exact optimum: identical
    active sets, U within 1e-9 of each other and of the exact solver.  (The algorithm restated in C,
    oracle/mpcqp_cpu.c, whose counters the GPU kernels match QP for QP.)  An unpolished result would
    depend on the scaling: the B=1 drop-in then re-solves under 10 passes
    (tests/test_gpu_pipeline.py::test_drop_in_unpolished_result_is_osqp_scaled)."""
    import cpu_solver

    for i in range(len(forms["tags"])):
        c = _case(forms, i)
        ex = mo.solve_exact(c["params"], c["x0"], c["window"], c["u_prev"])
        outs = [cpu_solver.cpu_solve(c["params"], c["x0"][None], c["window"][None], c["u_prev"][None], nthreads=1,
                                     scaling=sc) for sc in (1, 10)]
        for o in outs:
            assert int(o["status"][0]) == 1, c["tag"]
            assert np.array_equal(o["active"][0], ex.active), c["tag"]
            err = np.abs(o["U"][0] - ex.Umat).max() / max(1.0, np.abs(ex.Umat).max())
            assert err <= 1e-9, (c["tag"], err)
        assert np.array_equal(outs[0]["active"], outs[1]["active"]), c["tag"]
