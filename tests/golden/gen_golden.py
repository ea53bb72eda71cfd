"""Generate the golden fixtures in this directory by importing the reference's Python.

Run in the build container only (``/root/reference`` does not exist on the GPU box):

    python tests/golden/gen_golden.py

The reference imports ``cvxpy`` at module load (``src/__init__.py:4`` ->
``src/config.py:13`` -> ``src/control/mpc_controller.py:7``); cvxpy/OSQP are not
installed, so an *import-only* stub module is registered first.  Nothing in the
stub solves anything: the one place the reference would call OSQP
(``MPCController.solve``) is replaced by the oracle's exact solver
(``oracle/mpc_oracle.py``), so the closed-loop fixtures pin the reference's own
loop semantics (``control_stage.py:79-150``, ``ref_builder.py``,
``geometry.py``, ``vehicle_model.py``) around the unique QP optimum.

Outputs (numpy ``.npz``, no pickled objects):
  vehicle.npz       f_discrete / linearize on a seeded grid        (vehicle_model.py:11-45)
  default_plan.npz  default map + RRT* plan + build_reference(N)   (config 1 inputs)
  branches.npz      root->node branches of the default RRT* tree, their
                    catmull_rom_spline and build_reference(v=15,N=20)  (config 3 generator)
  closed_loop.npz   the reference's TrajectoryTracker.track / PipelineOrchestrator
                    loop at N=10 (config 1) and N=15 (code default) with the exact solve
  unwrap.npz        np.unwrap edge cases (mpc_controller.py:60)
"""
from __future__ import annotations

import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REFERENCE = Path(os.environ.get("RRT_MPC_REFERENCE", "/root/reference"))


def _install_cvxpy_stub() -> None:
    stub = types.ModuleType("cvxpy")

    class SolverError(Exception):
        pass

    stub.SolverError = SolverError
    stub.OPTIMAL = "optimal"
    stub.OPTIMAL_INACCURATE = "optimal_inaccurate"
    stub.OSQP = "OSQP"
    sys.modules["cvxpy"] = stub


def main() -> None:
    _install_cvxpy_stub()
    sys.path.insert(0, str(REFERENCE))
    sys.path.insert(0, str(REPO / "oracle"))
    import matplotlib

    matplotlib.use("Agg")
    import mpc_oracle as mo
    from src.config import default_config
    from src.control import vehicle_model as vm
    from src.control.ref_builder import build_reference
    from src.pipeline import control_stage
    from src.pipeline.map_stage import MapStage
    from src.pipeline.orchestrator import PipelineOrchestrator
    from src.pipeline.planning_stage import PlanningStage
    from src.planning.rrt_star import catmull_rom_spline

    # ---------------- vehicle model ----------------
    rng = np.random.default_rng(1234)
    M = 256
    xs = np.column_stack(
        [rng.uniform(-100, 100, M), rng.uniform(-100, 100, M), rng.uniform(-7, 7, M), rng.uniform(-5, 60, M)]
    )
    us = np.column_stack([rng.uniform(-40, 40, M), rng.uniform(-1.2, 1.2, M)])
    dts = rng.choice([0.05, 0.1, 0.2], M)
    Ls = rng.choice([3.5, 5.0, 14.0], M)
    fd = np.zeros((M, 4))
    A = np.zeros((M, 4, 4))
    B = np.zeros((M, 4, 2))
    fx = np.zeros((M, 4))
    for i in range(M):
        fd[i] = vm.f_discrete(xs[i], us[i], dts[i], Ls[i])
        A[i], B[i], fx[i] = vm.linearize(xs[i], us[i], dts[i], Ls[i])
    np.savez(HERE / "vehicle.npz", x=xs, u=us, dt=dts, L=Ls, f_discrete=fd, A=A, B=B, fx=fx)

    # ---------------- unwrap edge cases ----------------
    rng = np.random.default_rng(99)
    cases = [
        np.array([0.0, np.pi, 0.0, -np.pi, 0.0]),
        np.array([0.0, np.pi + 1e-12, 2 * np.pi, 3 * np.pi, 0.0]),
        np.array([3.0, -3.0, 3.0, -3.0, 3.1]),
        np.array([0.0, -np.pi, -2 * np.pi, np.pi, 0.0]),
        rng.uniform(-10, 10, 31),
        np.cumsum(rng.uniform(-4, 4, 31)),
    ]
    L_ = max(len(c) for c in cases)
    P = np.full((len(cases), L_), np.nan)
    U = np.full((len(cases), L_), np.nan)
    lens = np.array([len(c) for c in cases])
    for i, c in enumerate(cases):
        P[i, : len(c)] = c
        U[i, : len(c)] = np.unwrap(c)
    np.savez(HERE / "unwrap.npz", p=P, unwrapped=U, lens=lens)

    # ---------------- default map + plan ----------------
    tmp = Path(tempfile.mkdtemp(prefix="rrtmpc_golden_"))
    cfg = default_config()
    cfg.map.map_file = str(tmp / "base.png")
    cfg.map.inflated_map_file = str(tmp / "inflated.png")
    cfg.map.generate = True
    cfg.viz.backend = "Agg"
    cfg.viz.animate_tree = False
    cfg.viz.record_frames = False
    maps = MapStage(cfg.map).build()
    planning = PlanningStage(cfg.planner).plan(maps)
    plan = planning.plan
    assert plan.success
    path = np.asarray(plan.path, dtype=float)
    nodes = np.array([[n.x, n.y, n.cost, -1 if n.parent is None else n.parent] for n in plan.nodes], dtype=float)
    out = dict(
        path=path,
        start=np.asarray(maps.start, dtype=float),
        goal=np.asarray(maps.goal, dtype=float),
        nodes=nodes,
        raw_path=np.asarray(plan.raw_path, dtype=float),
        occupancy=maps.occupancy.astype(np.uint8),
        map_resolution=np.float64(cfg.map.map_resolution),
        yaw0=np.float64(np.arctan2(path[1][1] - path[0][1], path[1][0] - path[0][0])),
    )
    for N in (5, 10, 15, 20, 30):
        out[f"ref_global_N{N}"] = build_reference(plan.path, cfg.mpc.v_px_s, N, cfg.mpc.dt)
    np.savez(HERE / "default_plan.npz", **out)

    # ---------------- RRT* branches (config-3 generator) ----------------
    parent = nodes[:, 3].astype(int)

    def branch(idx):
        pts = []
        while idx >= 0:
            pts.append(nodes[idx, :2])
            idx = parent[idx]
        return np.asarray(pts[::-1])

    depth = np.zeros(len(nodes), dtype=int)
    for i in range(len(nodes)):
        d, j = 0, i
        while parent[j] >= 0:
            d += 1
            j = parent[j]
        depth[i] = d
    eligible = np.flatnonzero(depth >= 3)
    pick = eligible[:: max(1, len(eligible) // 12)][:12]
    br_pts, br_off, sp_pts, sp_off, rf_pts, rf_off = [], [0], [], [0], [], [0]
    for idx in pick:
        b = branch(int(idx))
        s = catmull_rom_spline([tuple(p) for p in b], samples_per_segment=20, alpha=0.5)
        r = build_reference([tuple(p) for p in s], 15.0, 20, 0.1)
        br_pts.append(b)
        br_off.append(br_off[-1] + len(b))
        sp_pts.append(s)
        sp_off.append(sp_off[-1] + len(s))
        rf_pts.append(r)
        rf_off.append(rf_off[-1] + len(r))
    np.savez(
        HERE / "branches.npz",
        node_index=pick,
        depth=depth,
        branch=np.vstack(br_pts),
        branch_off=np.asarray(br_off),
        spline=np.vstack(sp_pts),
        spline_off=np.asarray(sp_off),
        ref=np.vstack(rf_pts),
        ref_off=np.asarray(rf_off),
    )

    # ---------------- closed loop through the reference's own tracker ----------------
    records: list = []

    class RecordingController:
        def __init__(self, params):
            self._inner = mo.OracleController(params)
            self.params = params

        def solve(self, x0, ref_traj, *, u_init=None, u_prev=None):
            res = self._inner.solve(x0, ref_traj, u_prev=u_prev)
            records.append((np.array(x0, float), np.array(ref_traj, float),
                            np.zeros(2) if u_prev is None else np.array(u_prev, float), res[0]))
            return res

    control_stage.MPCController = RecordingController
    loops = {}
    for N, sim_steps in ((10, 100), (15, 300)):
        records.clear()
        cfgN = default_config()
        cfgN.map = cfg.map
        cfgN.viz = cfg.viz
        cfgN.mpc.horizon = N
        cfgN.mpc.sim_steps = sim_steps
        result = PipelineOrchestrator(cfgN).run(visualize=False)
        states = np.asarray(result.states, dtype=float)
        loops[f"N{N}_states"] = states
        loops[f"N{N}_x0"] = np.asarray([r[0] for r in records])
        loops[f"N{N}_window"] = np.asarray([r[1] for r in records])
        loops[f"N{N}_u_prev"] = np.asarray([r[2] for r in records])
        loops[f"N{N}_u0"] = np.asarray([r[3] for r in records])
        print(f"closed loop N={N}: {len(states)} steps, {len(records)} solves")
    np.savez(HERE / "closed_loop.npz", **loops)
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    main()
