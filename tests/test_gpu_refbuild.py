"""GPU tests of the batched build_reference (csrc/mpcqp_refbuild.hip)
against the reference's own outputs (default_plan.npz / branches.npz, bit-level goldens of
src/control/ref_builder.py) and this build's host restatement on randomised polylines.

Tolerance: 1e-12 absolute on the reference's own paths; 1e-11 relative + 1e-11 absolute on the
random polylines (up to 400 points: the arc lengths sum one device-hypot rounding per segment,
and atan2 is the device's -- both libms are within an ulp of each other).  Row counts must be
identical."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-12


def _check(dev_ref, dev_len, host_refs, rtol=0.0, atol=TOL):
    ref = dev_ref.cpu().numpy()
    lens = dev_len.cpu().numpy()
    for v, h in enumerate(host_refs):
        assert lens[v] == len(h), (v, lens[v], len(h))
        np.testing.assert_allclose(ref[v, : len(h)], h, rtol=rtol, atol=atol)


def test_default_plan_matches_reference_golden(cuda, golden):
    from mpcqp.control.ref_builder import build_reference_batch

    g = golden("default_plan.npz")
    for N in (5, 10, 15, 20, 30):
        ref, ln = build_reference_batch([g["path"]], 15.0, N, 0.1, device=cuda)
        _check(ref, ln, [g[f"ref_global_N{N}"]])


def test_branch_splines_match_reference_golden(cuda, golden):
    from mpcqp.control.ref_builder import build_reference_batch

    br = golden("branches.npz")
    so, ro = br["spline_off"], br["ref_off"]
    paths = [br["spline"][so[i]:so[i + 1]] for i in range(len(so) - 1)]
    refs = [br["ref"][ro[i]:ro[i + 1]] for i in range(len(ro) - 1)]
    ref, ln = build_reference_batch(paths, 15.0, 20, 0.1, device=cuda)
    _check(ref, ln, refs)


def _random_paths(rng, count):
    paths = []
    for k in range(count):
        kind = k % 8
        if kind == 0:
            paths.append(rng.uniform(0, 80, size=(int(rng.integers(2, 400)), 2)))  # long, chunked
        elif kind == 1:
            p = np.cumsum(rng.normal(0, 3, size=(int(rng.integers(3, 60)), 2)), axis=0) + 40
            p[3 % len(p)] = p[2 % len(p)]  # a zero-length segment
            paths.append(p)
        elif kind == 2:
            paths.append(rng.uniform(0, 80, size=(1, 2)))  # single point
        elif kind == 3:
            q = rng.uniform(0, 80, size=(1, 2))
            paths.append(np.vstack([q, q, q]))  # total < 1e-9: returned unchanged
        elif kind == 4:  # zig-zag: headings jump across +-pi
            t = np.arange(int(rng.integers(5, 90)))
            paths.append(np.column_stack([40 + 10 * (t % 2) - 5 * (t // 2 % 2), 40 + 0.3 * t]))
        elif kind == 5:  # circles: unwrap accumulates several turns
            t = np.linspace(0, 6 * np.pi, int(rng.integers(50, 300)))
            paths.append(np.column_stack([40 + 20 * np.cos(t), 40 + 20 * np.sin(t)]))
        elif kind == 6:  # exact multiple of the step: the total is not appended
            paths.append(np.array([[0.0, 0.0], [0.0, 20.0], [12.0, 36.0]]))
        else:
            paths.append(np.array([[10.0, 10.0], [10.0 + 1e-3, 10.0]]))  # shorter than one step
    return paths


@pytest.mark.parametrize("speed,N", [(15.0, 20), (40.0, 10), (90.0, 30), (3.0, 1)])
def test_random_polylines_match_host(cuda, speed, N):
    from mpcqp.control.ref_builder import build_reference, build_reference_batch

    rng = np.random.default_rng(int(speed * 100) + N)
    paths = _random_paths(rng, 48)
    ref, ln = build_reference_batch(paths, speed, N, 0.1, device=cuda)
    _check(ref, ln, [build_reference(p, speed, N, 0.1) for p in paths], rtol=1e-11, atol=1e-11)


def test_empty_overflow_and_bad_paths(cuda):
    import torch
    from mpcqp import _lib
    from mpcqp.control.ref_builder import build_reference_batch

    ref, ln = build_reference_batch([np.zeros((0, 2)), np.array([[1.0, 2.0], [30.0, 2.0]])], 15.0, 5, 0.1,
                                    device=cuda)
    assert ln.cpu().tolist() == [0, 16]  # empty path -> 0 rows; 29 px / 2 px steps + total
    # ref_stride too small: negative row count, nothing written
    ref, ln = build_reference_batch([np.array([[0.0, 0.0], [100.0, 0.0]])], 15.0, 5, 0.1, device=cuda, ref_stride=8)
    assert ln.cpu().tolist() == [-51]
    # a polyline longer than max_points
    L = _lib.lib()
    pts = torch.zeros((10, 2), dtype=torch.float64, device=cuda)
    off = torch.tensor([0, 10], dtype=torch.int32, device=cuda)
    out = torch.zeros((1, 32, 4), dtype=torch.float64, device=cuda)
    lens = torch.zeros((1,), dtype=torch.int32, device=cuda)
    _lib.check(L.mpcqp_build_reference(1, pts.data_ptr(), off.data_ptr(), 4, 15.0, 5, 0.1, 32, out.data_ptr(),
                                       lens.data_ptr(), None), "build_reference")
    assert lens.cpu().tolist() == [_lib.REF_BAD_PATH]
    assert L.mpcqp_build_reference(1, pts.data_ptr(), off.data_ptr(), _lib.REF_MAX_POINTS + 1, 15.0, 5, 0.1, 32,
                                   out.data_ptr(), lens.data_ptr(), None) == -1
    assert L.mpcqp_build_reference(1, pts.data_ptr(), off.data_ptr(), 4, 15.0, 0, 0.1, 32,
                                   out.data_ptr(), lens.data_ptr(), None) == -2


def test_fleet_on_device_references_matches_host_references(cuda, golden):
    """The closed loop on references built on the device == on references built on the host."""
    from mpcqp.config import MPCConfig
    from mpcqp.pipeline.fleet import FleetTracker

    br = golden("branches.npz")
    so = br["spline_off"]
    paths = [br["spline"][so[i]:so[i + 1]] for i in range(len(so) - 1)]
    starts = np.array([p[0] for p in paths]) + 1.5
    goals = np.array([p[-1] for p in paths])
    out = []
    for dev_ref in (False, True):
        ft = FleetTracker(MPCConfig(horizon=20, sim_steps=40), map_resolution=0.8, max_vehicles=len(paths),
                          max_ref_len=128, device=cuda)
        ft.reset_from_plans(paths, starts, goals, device_reference=dev_ref)
        out.append(ft.run())
        ft.close()
    a, b = out
    np.testing.assert_array_equal(a.steps, b.steps)
    for v in range(len(paths)):
        np.testing.assert_allclose(a.states[v], b.states[v], rtol=0, atol=1e-9)
