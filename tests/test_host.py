"""CPU tests of the host layer: C-ABI exports and struct layout, the Python mirror of the
reference interface, the scenario generators against the reference's golden vectors, and
the "no CPU fallback" rule.  No GPU calls are made here."""
from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "mpcqp.h"


def _binding():
    import __graft_entry__ as g

    if not g.LIB.exists():
        g.build_library()
    from mpcqp import _lib

    return _lib


def test_library_build_id_matches_the_sources():
    """The shipped libmpcqp.so is the one HEAD's sources build: its compiled-in build id equals the
    hash of the sources and the compile recipe (a stale library fails here, whatever its mtime)."""
    import __graft_entry__ as g

    _lib_mod = _binding()
    want = g.source_hash()
    assert g.library_build_id() == want, "libmpcqp.so is stale: rebuild with __graft_entry__.build()"
    assert _lib_mod.lib().mpcqp_build_id().decode() == want


def test_library_exports_every_header_symbol():
    _lib_mod = _binding()
    text = HEADER.read_text()
    decls = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(mpcqp_[a-z_0-9]+)\s*\(", text, re.M)
    assert len(decls) >= 12
    handle = ctypes.CDLL(str(_lib_mod.LIB_PATH))
    for name in decls:
        assert hasattr(handle, name), f"{name} declared in include/mpcqp.h but not exported"
    assert set(decls) == set(_lib_mod.exported_symbols())
    L = _lib_mod.lib()
    assert L.mpcqp_version() == _lib_mod.ABI_VERSION == 9
    assert L.mpcqp_num_rows(20) == 101
    assert L.mpcqp_model_stride(20) % 8 == 0


@pytest.mark.parametrize("cls_name,c_name", [("MpcqpParams", "mpcqp_params"), ("MpcqpFleet", "mpcqp_fleet"),
                                             ("MpcqpRrtParams", "mpcqp_rrt_params"), ("MpcqpSwarm", "mpcqp_swarm")])
def test_struct_layout_matches_c(tmp_path, cls_name, c_name):
    """ctypes mirrors of mpcqp_params / mpcqp_fleet == the C compiler's layout (sizeof, offsets)."""
    from mpcqp import _lib

    cls = getattr(_lib, cls_name)
    fields = [f for f, _ in cls._fields_]
    src = tmp_path / "layout.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "mpcqp.h"\nint main(void){\n'
        f'  printf("%zu\\n", sizeof({c_name}));\n'
        + "".join(f'  printf("%zu\\n", offsetof({c_name}, {f}));\n' for f in fields)
        + "  return 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), "-o", str(exe), str(src)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(cls)
    for f, off in zip(fields, vals[1:]):
        assert getattr(cls, f).offset == off, f


def test_fleet_host_helpers_mirror_control_stage():
    """relaxed_parameters == the retry parameters of control_stage.py:50-56; initial_state ==
    :74-79; the fleet phase codes mirror include/mpcqp.h."""
    from mpcqp import _lib
    from mpcqp.config import MPCConfig
    from mpcqp.pipeline.fleet import initial_state, relaxed_parameters

    base = MPCConfig(horizon=10).to_parameters(0.8)
    rel = relaxed_parameters(base)
    assert rel.du_bounds == ((-17.0, 17.0), (-0.2, 0.2))
    assert rel.u_bounds == base.u_bounds and rel.horizon == base.horizon
    np.testing.assert_array_equal(initial_state([(0.0, 0.0), (1.0, 1.0)], (3.0, 4.0)),
                                  [3.0, 4.0, np.arctan2(1.0, 1.0), 5.0])
    np.testing.assert_array_equal(initial_state([(2.0, 2.0)], (3.0, 4.0)), [3.0, 4.0, 0.0, 5.0])
    text = HEADER.read_text()
    for name in ("RUNNING", "GOAL", "ABORTED", "OUT_OF_STEPS"):
        m = re.search(rf"#define MPCQP_FLEET_{name}\s+(\d+)", text)
        assert m and int(m.group(1)) == getattr(_lib, f"FLEET_{name}")


def test_to_c_params_carries_reference_settings():
    from mpcqp._lib import to_c_params
    from mpcqp.config import MPCConfig

    c = to_c_params(MPCConfig(horizon=20).to_parameters(0.8))
    assert c.horizon == 20 and abs(c.wheelbase_px - 3.5) < 1e-15
    # OSQP settings of mpc_controller.py:121-131
    assert (c.eps_abs, c.eps_rel, c.max_iter, c.polish, c.adaptive_rho, c.rho, c.alpha) == \
        (1e-3, 1e-3, 60000, 1, 1, 0.1, 1.6)
    assert list(c.u_bounds) == [-35.0, 35.0, -0.6, 0.6]
    assert list(c.du_bounds) == [-12.0, 12.0, -0.15, 0.15]
    assert (c.slack_velocity, c.slack_input, c.slack_rate) == (1e3, 5e2, 5e2)


def test_checker_defaults_equal_product_defaults():
    """The C restatement (oracle/cpu_solver.py) solves with the product's default settings, so a
    default-settings comparison checks the same algorithm; and the per-workload schedules."""
    import cpu_solver
    from mpcqp._lib import DEFAULT_SOLVER_SETTINGS, to_c_params
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import latency_settings
    from mpcqp.pipeline.fleet import closed_loop_settings

    p = MPCConfig(horizon=20).to_parameters(0.8)
    prod, chk = to_c_params(p), cpu_solver.make_cparams(p)
    for name, _ in cpu_solver.CParams._fields_:
        if name != "reproducible":  # the product's kernel choice; the C restatement has one algorithm
            a, b = getattr(prod, name), getattr(chk, name)
            a, b = (list(a), list(b)) if hasattr(a, "__len__") else (a, b)
            assert a == b, name
    # one Ruiz pass and the batch polish schedule; OSQP's 10 passes stay a setting
    assert (DEFAULT_SOLVER_SETTINGS["scaling"], DEFAULT_SOLVER_SETTINGS["polish_from"]) == (1, 75)
    assert to_c_params(p, scaling=10).scaling == 10
    for N in (1, 10, 15, 20, 31):
        assert latency_settings(N) == closed_loop_settings(N) == {"polish_from": 25}
    assert latency_settings(40) == closed_loop_settings(40) == {}


def test_config_defaults_mirror_reference():
    from mpcqp.config import MPCConfig

    cfg = MPCConfig()
    assert (cfg.horizon, cfg.sim_steps, cfg.dt, cfg.v_px_s, cfg.wheelbase_m) == (15, 300, 0.1, 15.0, 2.8)
    p = MPCConfig(horizon=5).to_parameters(map_resolution=0.2)  # reference tests/test_mpc_controller.py
    assert p.wheelbase_px == pytest.approx(14.0)
    np.testing.assert_array_equal(p.q, np.diag([4.0, 4.0, 0.6, 0.1]))


def test_vehicle_model_matches_reference_golden(golden):
    from mpcqp.control.vehicle_model import f_discrete, linearize

    g = golden("vehicle.npz")
    for i in range(0, len(g["x"]), 3):
        np.testing.assert_array_equal(f_discrete(g["x"][i], g["u"][i], g["dt"][i], g["L"][i]), g["f_discrete"][i])
        A, B, fx = linearize(g["x"][i], g["u"][i], g["dt"][i], g["L"][i])
        np.testing.assert_array_equal(A, g["A"][i])
        np.testing.assert_array_equal(B, g["B"][i])


def test_build_reference_matches_reference_golden(golden):
    from mpcqp.control.ref_builder import build_reference

    g = golden("default_plan.npz")
    for N in (5, 10, 15, 20, 30):
        np.testing.assert_array_equal(build_reference(g["path"], 15.0, N, 0.1), g[f"ref_global_N{N}"])


def test_scenario_branches_match_reference_golden(golden):
    """config-3 generator pieces (Catmull-Rom + build_reference on RRT* branches), bit-exact."""
    from mpcqp.common.geometry import catmull_rom_spline
    from mpcqp.control.ref_builder import build_reference

    g = golden("branches.npz")
    for i in range(len(g["node_index"])):
        br = g["branch"][g["branch_off"][i]: g["branch_off"][i + 1]]
        sp = catmull_rom_spline(br, samples_per_segment=20, alpha=0.5)
        np.testing.assert_array_equal(sp, g["spline"][g["spline_off"][i]: g["spline_off"][i + 1]])
        np.testing.assert_array_equal(build_reference(sp, 15.0, 20, 0.1), g["ref"][g["ref_off"][i]: g["ref_off"][i + 1]])


def test_catmull_rom_vectorised_equals_per_sample_loop():
    """The per-segment vectorised smoothing == the reference's per-sample loop
    (rrt_star.py:93-159, restated scalar here), bit for bit, on duplicates, collinear and
    integer points and alpha in {0, 0.5, 1}."""
    from mpcqp.common.geometry import catmull_rom_spline

    def scalar(points, S, alpha, eps=1e-9, tol=1e-9):
        keep = [np.asarray(points[0], float)]
        for p in np.asarray(points, float)[1:]:
            if np.linalg.norm(p - keep[-1]) > tol:
                keep.append(p)
        pts = np.asarray(keep)
        if len(pts) <= 2:  # straight-line branches, not the loop under test
            return None
        ext = np.vstack([pts[0], pts, pts[-1]])
        out = []
        for i in range(len(pts) - 1):
            p0, p1, p2, p3 = ext[i:i + 4]
            ts = [0.0]
            for a, b in ((p0, p1), (p1, p2), (p2, p3)):
                d = np.linalg.norm(b - a)
                ts.append(ts[-1] + ((d ** alpha) if d > eps else eps))
            t0, t1, t2, t3 = ts
            d01, d12, d23 = max(t1 - t0, eps), max(t2 - t1, eps), max(t3 - t2, eps)
            d02, d13 = max(t2 - t0, eps), max(t3 - t1, eps)
            for t in np.linspace(t1, t2, max(2, S + 1), endpoint=False):
                a1 = (t1 - t) / d01 * p0 + (t - t0) / d01 * p1
                a2 = (t2 - t) / d12 * p1 + (t - t1) / d12 * p2
                a3 = (t3 - t) / d23 * p2 + (t - t2) / d23 * p3
                b1 = (t2 - t) / d02 * a1 + (t - t0) / d02 * a2
                b2 = (t3 - t) / d13 * a2 + (t - t1) / d13 * a3
                out.append((t2 - t) / d12 * b1 + (t - t1) / d12 * b2)
        out.append(pts[-1])
        return np.asarray(out)

    rng = np.random.default_rng(5)
    for k in range(60):
        pts = rng.uniform(0, 80, (int(rng.integers(3, 25)), 2))
        if k % 3 == 0:
            pts[1] = pts[0]
            pts[-1] = pts[-2] + 1e-12
        if k % 4 == 0:
            pts = np.round(pts)
        if k % 5 == 0:
            pts[:, 1] = 7.0
        for alpha in (0.0, 0.5, 1.0):
            S = int(rng.integers(1, 25))
            want = scalar(pts, S, alpha)
            got = catmull_rom_spline(pts, samples_per_segment=S, alpha=alpha)
            if want is not None:
                np.testing.assert_array_equal(got, want)


def test_scenarios_shapes_and_determinism():
    from mpcqp import scenarios

    a, b = scenarios.config3(64), scenarios.config3(64)
    np.testing.assert_array_equal(a.x0, b.x0)
    assert a.ref.shape == (64, 21, 4) and a.u_prev.shape == (64, 2)
    c4 = scenarios.config4(32)
    assert c4.ref.shape == (32, 31, 4) and (c4.x0[:, 3] >= 0).all() and (c4.x0[:, 3] <= 15).all()
    c2 = scenarios.config2(8)
    assert (c2.x0 == c2.x0[0]).all() and c2.x0[0, 3] == 5.0


def test_no_cpu_fallback_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mpcqp._lib import LibraryError
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController, MPCController

    params = MPCConfig(horizon=5).to_parameters(0.2)
    with pytest.raises(LibraryError):
        BatchedMPCController(params, 4)
    with pytest.raises(LibraryError):
        MPCController(params).solve(np.zeros(4), np.zeros((6, 4)))


def test_product_never_imports_the_oracle():
    pkg = ROOT / "rrt-mpc_amd"
    pattern = re.compile(r"import\s+(mpc_oracle|cpu_solver)|from\s+(oracle|mpc_oracle|cpu_solver)\b|"
                         r"libmpcqp_cpu|#include\s+\"[^\"]*oracle")
    for f in list(pkg.rglob("*.py")) + list(pkg.rglob("*.hip")):
        m = pattern.search(f.read_text())
        assert m is None, f"{f} loads the oracle: {m.group(0) if m else ''}"


def test_tracker_rejects_failed_plans():
    """control_stage.py:69-72 error behaviour."""
    from types import SimpleNamespace

    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    t = TrajectoryTracker(MPCConfig(), VizConfig())
    maps = SimpleNamespace(start=(0, 0), goal=(1, 1))
    with pytest.raises(RuntimeError, match="did not succeed"):
        t.track(SimpleNamespace(plan=SimpleNamespace(success=False, path=[(0, 0)])), maps, map_resolution=0.8)
    with pytest.raises(RuntimeError, match="empty path"):
        t.track(SimpleNamespace(plan=SimpleNamespace(success=True, path=[])), maps, map_resolution=0.8)


def test_window_gather_matches_reference_loop(golden):
    from mpcqp.pipeline.control_stage import window_at

    plan = golden("default_plan.npz")
    loop = golden("closed_loop.npz")
    ref_g = plan["ref_global_N15"]
    wins = loop["N15_window"]
    # the reference advanced path_idx by at most one per step; recover it from the windows
    for k, w in enumerate(wins):
        idx = int(np.argmin(np.abs(ref_g[:, 0] - w[0, 0]) + np.abs(ref_g[:, 1] - w[0, 1])))
        np.testing.assert_array_equal(window_at(ref_g, idx, 15), w)


def test_solver_kernel_resources():
    """Every k_solve<N> keeps 2 waves per SIMD and its working set in registers: the build
    records hipcc's resource remarks (build/kernel_resources.json).  A demoted KKT-inverse
    row (scratch memory) once made config 4 (N = 30) 25x slower."""
    import json

    path = ROOT / "build" / "kernel_resources.json"
    if not path.exists():
        pytest.skip("library not built in this tree (build() writes the resource record)")
    rec = json.loads(path.read_text())
    res = {int(k): v for k, v in rec.items() if ":" not in k}
    loops = {int(k.split(":")[1]): v for k, v in rec.items() if k.startswith("loop:")}
    pairs = {k: v for k, v in rec.items() if k.startswith(("pair:", "loop_pair:"))}
    assert sorted(res) == list(range(1, 33))
    assert sorted(loops) == list(range(1, 33))
    # two QPs (vehicles) per wave, N <= 15: still 2 waves per SIMD, two LDS blocks per workgroup
    assert sorted(pairs) == sorted([f"pair:{N}" for N in range(1, 16)] + [f"loop_pair:{N}" for N in range(1, 16)])
    for k, r in pairs.items():
        assert r["Occupancy"] >= 2 and r["AGPRs"] == 0, (k, r)
        assert r["ScratchSize"] <= (0 if k.startswith("pair:") else 512), (k, r)
        assert r["LDS"] <= 160 * 1024 // 8, (k, r)
    for N, r in loops.items():
        # the fused closed loop (k_fleet_loop<N>) runs the same solver at 2 waves per SIMD; values
        # live across the steps (loop state, output pointers) spill at the step boundary only
        assert r["Occupancy"] >= 2 and r["AGPRs"] == 0, (N, r)
        assert r["ScratchSize"] <= (640 if N == 32 else 512), (N, r)
        assert r["LDS"] <= 160 * 1024 // 8, (N, r)
    for N, r in res.items():
        # every horizon at 2 waves per SIMD and 8 workgroups per CU (N >= 24: Pbar packed, <= 18 KB
        # of LDS); N >= 29 fills the 256 registers and spills a handful of values outside the
        # inverse (<= 64 bytes); N = 32 (2N = 64: every lane a column, g in a second condensing
        # pass) spills part of the setup column around that pass (setup only, <= 320 bytes)
        assert r["Occupancy"] >= 2, (N, r)
        assert r["AGPRs"] == 0, (N, r)
        assert r["ScratchSize"] <= (320 if N == 32 else 64 if N >= 29 else 0), (N, r)
        assert r["LDS"] <= 160 * 1024 // 8, (N, r)  # 8 workgroups = 2 waves on each of 4 SIMDs


def test_three_argument_step_resolves_parameters(golden, monkeypatch):
    """``TrajectoryTracker.step(state, ref_window, u_prev)`` on the host logic: the
    B=1 device call swapped for the C restatement (no GPU here), every N = 15 window of the
    reference's own loop replayed without a params argument (-> ``to_parameters(0.8)``); after a
    ``track()`` at another resolution the tracker keeps that call's parameters."""
    import mpcqp.control.mpc_controller as mc
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    from _dropin_driver import _CpuSingle

    seen = []

    def single(params, method="admm", **settings):
        seen.append(float(params.wheelbase_px))
        return _CpuSingle(params, **settings)

    monkeypatch.setattr(mc, "_single_controller", single)
    loop = golden("closed_loop.npz")
    tracker = TrajectoryTracker(MPCConfig(horizon=15), VizConfig())
    for k in range(len(loop["N15_x0"])):
        nxt, u0, Xp = tracker.step(loop["N15_x0"][k], loop["N15_window"][k], loop["N15_u_prev"][k])
        np.testing.assert_allclose(u0, loop["N15_u0"][k], rtol=0, atol=1e-8)
        np.testing.assert_allclose(nxt, loop["N15_states"][k], rtol=0, atol=1e-8)
        assert Xp.shape == (4, 16)
    assert set(seen) == {2.8 / 0.8}
    tracker.step(loop["N15_x0"][0], loop["N15_window"][0], loop["N15_u_prev"][0], map_resolution=0.2)
    assert seen[-1] == 2.8 / 0.2
    plan = golden("default_plan.npz")
    from types import SimpleNamespace

    planning = SimpleNamespace(plan=SimpleNamespace(success=True, path=[tuple(map(float, p)) for p in plan["path"]]))
    maps = SimpleNamespace(start=tuple(plan["start"]), goal=tuple(plan["goal"]))
    tracker.mpc = MPCConfig(horizon=15, sim_steps=1)
    tracker.track(planning, maps, map_resolution=0.4, visualize=False)
    tracker.step(loop["N15_x0"][0], loop["N15_window"][0], loop["N15_u_prev"][0])
    assert seen[-1] == seen[-2] == 2.8 / 0.4


def test_initial_states_equal_per_vehicle_initial_state():
    """The fleet's vectorised start states (one elementwise arctan2 over all vehicles) equal
    ``initial_state`` (control_stage.py:74-79) per vehicle bit for bit, one-point paths included."""
    from mpcqp import scenarios
    from mpcqp.pipeline.fleet import initial_state, initial_states

    paths, starts, goals = scenarios.fleet5(512)
    paths = list(paths) + [np.array([[3.0, 4.0]]), [(1.0, 2.0), (1.0, 2.0)], [(0.0, 0.0), (-1.0, -1e-300)]]
    starts = np.vstack([starts, [[1.0, 1.0], [2.0, 2.0], [3.0, 3.0]]])
    got = initial_states(paths, starts)
    want = np.array([initial_state(p, s) for p, s in zip(paths, starts)])
    np.testing.assert_array_equal(got, want)


def test_packed_paths_equal_per_path_packing():
    """PackedPaths (one concatenation; the per-path fallback for ragged / empty / odd inputs) packs
    exactly what a per-path np.asarray(...).reshape(-1, 2) packing gives."""
    from mpcqp import scenarios
    from mpcqp.control.ref_builder import PackedPaths

    paths, _, _ = scenarios.fleet5(64)
    cases = [list(paths), [], [np.zeros((0, 2))], [np.array([[1.0, 2.0], [3.0, 4.0]]), []],
             [[(1, 2), (3, 4)], np.array([[5.0, 6.0]])], [np.array([[1, 2], [3, 5]])],
             [np.array([1.0, 2.0, 3.0, 4.0]), np.array([[5.0, 6.0]])]]
    for c in cases:
        pk = PackedPaths(c)
        arrs = [np.asarray(q, dtype=float).reshape(-1, 2) for q in c]
        assert pk.V == len(c)
        assert pk.counts.tolist() == [len(a) for a in arrs]
        assert pk.off.tolist() == [0] + np.cumsum([len(a) for a in arrs]).astype(int).tolist()
        if arrs and sum(len(a) for a in arrs):
            assert pk.pts.dtype == np.float64
            np.testing.assert_array_equal(pk.pts, np.concatenate(arrs))
        for a, b in zip(pk.arrs, arrs):
            np.testing.assert_array_equal(a, b)


def test_argument_checks_without_a_device():
    """Entry points that validate their arguments before touching the device return MPCQP_E_ARG for
    a null workspace or a bad mode, and report why (no GPU in this container)."""
    import ctypes

    _lib_mod = _binding()
    L = _lib_mod.lib()
    E_ARG = -1
    assert L.mpcqp_set_pairing(None, _lib_mod.PAIR_ON) == E_ARG
    assert b"null ws" in L.mpcqp_last_error()
    assert L.mpcqp_solve_served(None) == E_ARG
    assert L.mpcqp_solve_staged(None) == E_ARG
    hin, hout = ctypes.c_void_p(), ctypes.c_void_p()
    offs = (ctypes.c_int32 * 6)()
    assert L.mpcqp_stage(None, ctypes.byref(hin), ctypes.byref(hout), offs) == E_ARG


def test_params_key_normalises_bounds_containers():
    """The B=1 controller cache keys bounds by value: tuples, lists, arrays and tuples of arrays of the
    same numbers give one key (one workspace), and none of them is unhashable."""
    import dataclasses

    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import _params_key

    p = MPCConfig(horizon=10).to_parameters(0.8)
    forms = [p.du_bounds, [list(r) for r in p.du_bounds], np.asarray(p.du_bounds),
             tuple(np.asarray(r) for r in p.du_bounds), tuple(tuple(np.float64(v) for v in r) for r in p.du_bounds)]
    keys = {_params_key(dataclasses.replace(p, du_bounds=f), 0, {}) for f in forms}
    assert len(keys) == 1
    other = dataclasses.replace(p, du_bounds=((-1.0, 1.0), (-0.1, 0.1)))
    assert _params_key(other, 0, {}) not in keys
