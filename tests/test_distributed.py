"""Multi-process (gloo) tests of bench.py's data-parallel path on CPU.

The ranks drive bench.py's own distributed functions -- ``shard_bounds``, ``DistContext``,
``timed_steps``, ``reduce_stats``, ``gather_rows``, ``spot_check`` -- with the C restatement
standing in for the GPU shard solve (there is no GPU in this container).  Weak scaling (per-rank
batch) and strong scaling (a fixed global batch, including one that does not divide evenly) must
both reproduce the single-process solve exactly.
"""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, out_dir):
    for p in (ROOT / "rrt-mpc_amd", ROOT / "oracle", ROOT):
        sys.path.insert(0, str(p))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist

    import bench
    import cpu_solver
    import mpc_oracle as mo

    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = bench.DistContext(world, rank, rank, "gloo", torch.device("cpu"))
    batch = bench.make_global_batch("config3", total)
    lo, hi = bench.shard_bounds(total, world, rank)
    counts = bench.shard_counts(total, world)
    params = mo.default_params(batch.horizon)
    res = {}

    def step(k):
        res.update(cpu_solver.cpu_solve(params, batch.x0[lo:hi], batch.ref[lo:hi], batch.u_prev[lo:hi], nthreads=1))

    elapsed = bench.timed_steps(step, 2, 1, ctx)
    T, (solved,) = bench.reduce_stats(ctx, elapsed + rank, [float((res["status"] == 1).sum())])
    per_rank = bench.gather_scalar(ctx, 10.0 * rank + 0.5)
    g = {k: bench.gather_rows(ctx, torch.from_numpy(res[k]), counts).numpy() for k in ("u0", "status", "U", "active")}
    if rank == 0:
        chk = bench.spot_check(params, batch.x0, batch.ref, batch.u_prev, g["U"], g["active"], g["status"],
                               np.arange(0, total, 5))
        np.savez(Path(out_dir) / "dist.npz", T=T, elapsed=elapsed, per_rank=np.array(per_rank), solved=solved, u0=g["u0"], status=g["status"],
                 U=g["U"], err=chk["max_rel_err_U"], mism=chk["active_set_mismatches"] + chk["status_mismatches"])
    ctx.barrier()
    ctx.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,total", [(2, 96), (3, 71)])
def test_sharded_solve_matches_single_process(tmp_path, world, total):
    """world ranks over gloo: contiguous shards (71 over 3 ranks: 24/24/23), MAX of time, SUM of
    solved, all_gather of u0/status/U in rank order == the single-process solve bit for bit."""
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    import bench
    import cpu_solver
    import mpc_oracle as mo

    mp.start_processes(_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    d = np.load(tmp_path / "dist.npz")
    # MAX over ranks: rank r reported its elapsed time + r seconds
    assert float(d["T"]) >= max(float(d["elapsed"]), world - 1.0)
    # per-rank scalars gathered in rank order (bench's rank_ms_per_step)
    assert d["per_rank"].tolist() == [10.0 * r + 0.5 for r in range(world)]
    assert float(d["solved"]) == total
    b = bench.make_global_batch("config3", total)
    full = cpu_solver.cpu_solve(mo.default_params(b.horizon), b.x0, b.ref, b.u_prev, nthreads=2)
    np.testing.assert_array_equal(d["u0"], full["u0"])
    np.testing.assert_array_equal(d["U"], full["U"])
    np.testing.assert_array_equal(d["status"], full["status"])
    assert float(d["err"]) == 0.0 and int(d["mism"]) == 0


def test_shard_bounds_cover_any_total():
    sys.path.insert(0, str(ROOT))
    import bench

    for total in (0, 1, 7, 16384, 16385):
        for world in (1, 2, 3, 8):
            b = [bench.shard_bounds(total, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == total
            assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))
            sizes = [hi - lo for lo, hi in b]
            assert max(sizes) - min(sizes) <= 1
            assert sizes == bench.shard_counts(total, world)


def test_weak_shards_are_contiguous_and_cover_the_batch():
    sys.path.insert(0, str(ROOT))
    import bench

    whole = bench.make_batch("config3", 32, 1, 0)
    parts = [bench.make_batch("config3", 8, 4, r) for r in range(4)]
    np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), whole[0])
    np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]), whole[1])


def _stub_swarm_run(starts, goals, seeds, sim_steps=None):
    """A deterministic stand-in for Swarm.run (no GPU here): every per-vehicle field a function of
    that vehicle's own inputs, so a sharded run must reassemble the single-process result exactly."""
    sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))
    from mpcqp.pipeline.swarm import SwarmResult

    V = len(starts)
    seeds = np.asarray(seeds)
    states = [np.array([[s[0], s[1], float(k)] for k in range(int(sd) % 5 + 1)]) for s, sd in zip(starts, seeds)]
    return SwarmResult(states=states, phase=(seeds % 3).astype(np.int32), steps=(seeds * 7 % 11).astype(np.int32),
                       replans=(seeds % 2).astype(np.int64), planned=seeds % 4 != 0,
                       paths=[[tuple(s), tuple(g)] for s, g in zip(starts, goals)],
                       replan_steps=np.stack([seeds, -seeds], axis=1).astype(np.int32),
                       last_replan_start=np.asarray(starts, float), last_replan_path=[None] * V,
                       inputs=[np.full((2, 2), float(sd)) for sd in seeds],
                       timings={"plan_s": 0.1 * len(starts), "track_replan_s": float(seeds.sum())})


def _swarm_worker(rank, world, port, V, out_dir):
    for p in (ROOT / "rrt-mpc_amd", ROOT):
        sys.path.insert(0, str(p))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import pickle

    import torch.distributed as dist

    from mpcqp.pipeline.swarm import run_swarm_sharded

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(3)
    starts, goals = rng.uniform(0, 80, (V, 2)), rng.uniform(0, 80, (V, 2))
    res = run_swarm_sharded(_stub_swarm_run, starts, goals, np.arange(V) + 100, rank=rank, world=world,
                            all_gather_object=dist.all_gather_object, sim_steps=5)
    with open(Path(out_dir) / f"swarm_{rank}.pkl", "wb") as f:
        pickle.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,V", [(2, 100), (3, 7), (4, 3)])
def test_sharded_swarm_matches_single_process(tmp_path, world, V):
    """Config 5 over `world` ranks (gloo): contiguous vehicle blocks (3 vehicles over 4 ranks leaves one
    rank empty), one all_gather_object of the shard results; every rank gets the single-process result
    in vehicle order, timings the max over ranks."""
    import pickle

    sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))
    from mpcqp.pipeline.swarm import shard_vehicles

    mp.start_processes(_swarm_worker, args=(world, _free_port(), V, str(tmp_path)), nprocs=world,
                       start_method="spawn", join=True)
    rng = np.random.default_rng(3)
    starts, goals = rng.uniform(0, 80, (V, 2)), rng.uniform(0, 80, (V, 2))
    full = _stub_swarm_run(starts, goals, np.arange(V) + 100)
    for r in range(world):
        with open(tmp_path / f"swarm_{r}.pkl", "rb") as f:
            got = pickle.load(f)
        for k in ("phase", "steps", "replans", "planned", "replan_steps", "last_replan_start"):
            np.testing.assert_array_equal(getattr(got, k), getattr(full, k), err_msg=k)
        assert len(got.states) == V and all(np.array_equal(a, b) for a, b in zip(got.states, full.states))
        assert all(np.array_equal(a, b) for a, b in zip(got.inputs, full.inputs))
        assert got.paths == full.paths
        blocks = [shard_vehicles(V, world, q) for q in range(world)]
        assert got.timings["plan_s"] == pytest.approx(max(0.1 * (hi - lo) for lo, hi in blocks))
