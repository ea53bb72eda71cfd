"""GPU tests of the B = 1 server (mpcqp_solve_served) beyond equality with a launch per call
(tests/test_gpu_pipeline.py): one resident wave per device while the drop-in alternates its nominal,
relaxed and OSQP-scaled workspaces; no blocking of default-priority streams; the failure paths (a wave
that leaves unannounced, a refused launch, non-finite inputs) and unpolished results."""
from __future__ import annotations

import ctypes
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _live(ctrl) -> bool:
    from mpcqp import _lib

    return _lib.lib().mpcqp_debug_serve_fault(ctrl._ws, 3) == 1


def _solve_all(ctrls, b, order):
    return [ctrls[k].solve_one(b.x0[q], b.ref[q], b.u_prev[q]) for q, k in order]


def test_one_resident_server_while_alternating_workspaces(cuda, monkeypatch):
    """The drop-in's retry pattern (nominal, relaxed, OSQP-scaled fallback) on the served path: every
    answer equals a launch per call bit for bit, only the workspace that served last keeps a resident
    wave (a switch stops the other one), and no call waits on another workspace's wave."""
    import dataclasses

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    N = 15
    b = scenarios.config3(30, horizon=N, seed=17)
    nominal = MPCConfig(horizon=N).to_parameters(0.8)
    du = nominal.du_bounds  # the relaxed retry's parameter block (control_stage.py:45-49)
    relaxed = dataclasses.replace(nominal, du_bounds=((du[0][0] - 5.0, du[0][1] + 5.0),
                                                      (du[1][0] - 0.05, du[1][1] + 0.05)))
    specs = [(nominal, {}), (relaxed, {}), (nominal, {"scaling": 10})]
    order = [(q, q % 3 if q % 4 else (q // 4) % 3) for q in range(30)]
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MPCQP_B1_SERVER", mode)
        ctrls = [BatchedMPCController(p, 1, device="cuda:0", **s) for p, s in specs]
        _solve_all(ctrls, b, order[:3])  # warm
        t0 = time.perf_counter()
        worst = 0.0
        out = []
        for q, k in order:
            t = time.perf_counter()
            out.append(ctrls[k].solve_one(b.x0[q], b.ref[q], b.u_prev[q]))
            worst = max(worst, time.perf_counter() - t)
            if mode == "1":
                live = [_live(c) for c in ctrls]
                assert live[k] and sum(live) == 1, (q, live)
        res[mode] = out
        # a switch costs a stop and a launch, never another wave's 2 ms idle exit
        assert worst < 1.5e-3 * 4, worst
        assert time.perf_counter() - t0 < 0.5
        for c in ctrls:
            c.close()
    for q in range(30):
        a, c = res["0"][q], res["1"][q]
        assert a[0] == c[0]
        for x, y in zip(a[1:], c[1:]):
            assert np.array_equal(x, y), q


def test_server_does_not_hold_default_priority_streams(cuda):
    """While the closed loop keeps its server resident (a request every few tens of microseconds), work
    enqueued on eight fresh default-priority torch streams finishes within a millisecond or two: the
    server's high-priority stream has a hardware queue of its own, so no packet waits behind it."""
    import torch

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    b = scenarios.config3(8, horizon=10, seed=3)
    streams = [torch.cuda.Stream() for _ in range(8)]
    x = torch.zeros(8, device="cuda:0")
    for i, s in enumerate(streams):  # the add kernel's first launch loads its code object: not measured here
        with torch.cuda.stream(s):
            x[i].add_(-1.0)
    torch.cuda.synchronize()
    ctrl = BatchedMPCController(MPCConfig(horizon=10).to_parameters(0.8), 1, device="cuda:0")
    ctrl.solve_one(b.x0[0], b.ref[0], b.u_prev[0])
    assert _live(ctrl)
    evs = []
    t0 = time.perf_counter()
    for i, s in enumerate(streams):
        with torch.cuda.stream(s):
            x[i].add_(1.0)
            e = torch.cuda.Event()
            e.record(s)
            evs.append(e)
    done = {}
    q = 0
    while time.perf_counter() - t0 < 0.05:
        st, *_ = ctrl.solve_one(b.x0[q % 8], b.ref[q % 8], b.u_prev[q % 8])
        assert st == 1
        q += 1
        for i, e in enumerate(evs):
            if i not in done and e.query():
                done[i] = time.perf_counter() - t0
    assert _live(ctrl)
    assert len(done) == 8, f"streams still blocked after 50 ms of served requests: {sorted(set(range(8)) - set(done))}"
    assert max(done.values()) < 0.01, done
    torch.cuda.synchronize()
    assert torch.equal(x.cpu(), torch.zeros(8))
    ctrl.close()


def test_server_failure_paths(cuda, monkeypatch):
    """A wave that leaves without telling the host is found gone and relaunched (the answer still
    comes); a refused launch fails the call (LibraryError; MPCController.solve maps it to
    (None, None, None)) and the next call launches again; a non-finite input returns status -10 next
    to a live server and the following QP is solved normally."""
    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control import mpc_controller as mc
    from mpcqp.control.mpc_controller import BatchedMPCController

    monkeypatch.setenv("MPCQP_B1_SERVER", "1")
    N = 10
    b = scenarios.config3(6, horizon=N, seed=5)
    params = MPCConfig(horizon=N).to_parameters(0.8)
    ref_c = BatchedMPCController(params, 6, device="cuda:0")
    sol = ref_c.solve_batch(b.x0, b.ref, b.u_prev)
    exp_st, exp_U = sol.status.cpu().numpy().copy(), sol.U.cpu().numpy().copy()
    ref_c.close()
    assert (exp_st == 1).all()
    L = _lib.lib()
    ctrl = BatchedMPCController(params, 1, device="cuda:0")

    def check(q):
        st, u0, X, U = ctrl.solve_one(b.x0[q], b.ref[q], b.u_prev[q])
        assert st == 1 and np.array_equal(U, exp_U[q]), q

    check(0)
    assert _live(ctrl)
    # 1. the wave leaves unannounced: the host still believes it resident
    assert L.mpcqp_debug_serve_fault(ctrl._ws, 2) == 0
    assert _live(ctrl)
    check(1)
    assert _live(ctrl)
    # 2. a refused launch (after the wave is gone): the call fails, the next one launches again
    assert L.mpcqp_debug_serve_fault(ctrl._ws, 2) == 0
    assert L.mpcqp_debug_serve_fault(ctrl._ws, 1) == 0
    with pytest.raises(_lib.LibraryError, match="refused"):
        ctrl.solve_one(b.x0[2], b.ref[2], b.u_prev[2])
    check(2)
    # 3. non-finite input beside a live server: status -10, then business as usual
    x0 = b.x0[3].copy()
    x0[1] = np.nan
    st, *_ = ctrl.solve_one(x0, b.ref[3], b.u_prev[3])
    assert st == _lib.NUMERICAL_ERROR
    assert _live(ctrl)
    check(3)
    check(4)
    # the drop-in maps a refused launch to (None, None, None)
    drop = mc._single_controller(params)
    drop.solve_one(b.x0[5], b.ref[5], b.u_prev[5])
    assert L.mpcqp_debug_serve_fault(drop._ws, 2) == 0
    assert L.mpcqp_debug_serve_fault(drop._ws, 1) == 0
    assert mc.MPCController(params).solve(b.x0[5], b.ref[5], u_prev=b.u_prev[5]) == (None, None, None)
    u0, X, U = mc.MPCController(params).solve(b.x0[5], b.ref[5], u_prev=b.u_prev[5])
    assert u0 is not None
    ctrl.close()


@pytest.mark.parametrize("capped", [dict(max_iter=50, polish_from=0, polish_near=0.0),
                                    dict(max_iter=30, polish=0, polish_from=0, polish_near=0.0)])
def test_served_unpolished_and_nan_against_launch(cuda, monkeypatch, capped):
    """Unpolished results (ADMM capped at max_iter, with and without the polish) and NaN inputs on
    the served path against a launch per call: statuses, the four counters and U equal bit for bit
    (the kernels contract multiply-adds only within a source expression)."""
    from mpcqp import _lib, scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    N = 20
    b = scenarios.config3(16, horizon=N, seed=9)
    x0 = b.x0.copy()
    x0[5, 0] = np.nan
    x0[11, 3] = np.inf
    params = MPCConfig(horizon=N).to_parameters(0.8)
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MPCQP_B1_SERVER", mode)
        ctrl = BatchedMPCController(params, 1, device="cuda:0", **capped)
        out = []
        for q in range(16):
            st, u0, X, U = ctrl.solve_one(x0[q], b.ref[q], b.u_prev[q])
            out.append((st, ctrl._one["iters"].copy(), U))
        ctrl.close()
        res[mode] = out
    sts = [r[0] for r in res["1"]]
    assert sts[5] == sts[11] == _lib.NUMERICAL_ERROR
    assert any(s in (_lib.SOLVED_INACCURATE, _lib.MAX_ITER_REACHED) for s in sts)
    for q in range(16):
        (sa, ia, Ua), (sb, ib, Ub) = res["0"][q], res["1"][q]
        assert sa == sb and np.array_equal(ia, ib), q
        if sa in (_lib.SOLVED, _lib.SOLVED_INACCURATE, _lib.MAX_ITER_REACHED):
            assert np.array_equal(Ua, Ub), q


def test_two_threads_on_two_workspaces(cuda, monkeypatch):
    """Two threads, each running its own closed-loop-like sequence of B = 1 requests on its own
    workspace of the same device at the same time: every answer equals the batch launch's bit for bit.
    A request stops the other workspace's wave only while that workspace is between calls (its lock
    is free), so no pending request is overwritten and no call runs into the 30 s timeout."""
    import threading

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    monkeypatch.setenv("MPCQP_B1_SERVER", "1")
    N, Q = 10, 60
    b = scenarios.config3(Q, horizon=N, seed=23)
    params = MPCConfig(horizon=N).to_parameters(0.8)
    ref_c = BatchedMPCController(params, Q, device="cuda:0")
    sol = ref_c.solve_batch(b.x0, b.ref, b.u_prev)
    exp_st, exp_U = sol.status.cpu().numpy().copy(), sol.U.cpu().numpy().copy()
    ref_c.close()
    ctrls = [BatchedMPCController(params, 1, device="cuda:0") for _ in range(2)]
    results = [[], []]
    errors = []

    def run(t):
        try:
            for rep in range(3):
                for q in range(t, Q, 2) if rep % 2 == 0 else range(Q - 1 - t, -1, -2):
                    st, u0, X, U = ctrls[t].solve_one(b.x0[q], b.ref[q], b.u_prev[q])
                    results[t].append((q, st, U.copy()))
        except Exception as exc:  # pragma: no cover - reported below
            errors.append(repr(exc))

    th = [threading.Thread(target=run, args=(t,)) for t in range(2)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th), "a served call hung"
    assert not errors, errors
    assert time.perf_counter() - t0 < 20.0
    for t in range(2):
        assert len(results[t]) == 3 * (Q // 2)
        for q, st, U in results[t]:
            assert st == exp_st[q] == 1 and np.array_equal(U, exp_U[q]), (t, q)
    for c in ctrls:
        c.close()
