#!/usr/bin/env python3
"""Benchmark: batched bicycle-MPC QP solves/s on MI355X (BASELINE.json metric).

One "step" = one pass of the hot path over one batch resident in HBM: ``mpcqp_build`` +
``mpcqp_solve`` (window -> LTV model -> condense -> ADMM/OSQP -> polish) for every QP of the
shard.  Default workload = BASELINE config 3 (B=4096 randomised RRT*-branch references,
horizon 20) per GPU.

Multi-GPU (one process per GPU, ``torch.distributed``; backend ``nccl`` = RCCL):
  * weak scaling (default): every rank solves its own contiguous shard of a ``batch x world``
    global batch;
  * strong scaling (``--global-batch G``, e.g. config 4: 16384 over 2/4/8 GPUs): the ranks
    split a fixed global batch contiguously.
There is no data-path collective (the QPs are independent).  Around the timed region: a barrier
on both sides, a MAX of the elapsed time and a SUM of the counters; after it one ``all_gather``
of u0/status whose global result rank 0 spot-checks against the C restatement.

    python bench.py --gpus 1 --steps 20 --warmup 3
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N --config config4 --global-batch 16384

Prints ONE JSON line on rank 0 (driver contract; roofline + cpu_baseline objects).

The distributed helpers (``shard_bounds``, ``DistContext``, ``timed_steps``, ``reduce_stats``,
``gather_rows``, ``spot_check``) are plain functions: tests/test_distributed.py drives the same
ones with the gloo backend on CPU.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time
from pathlib import Path
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))
sys.path.insert(0, str(ROOT))

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 dense (vector == matrix), AMD spec
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md
BASELINE_METRIC = "MPC QP solves/s (horizon=20, batch=4096) @1/2/4/8 GPU; rel-err vs OSQP"
DEFAULT_BATCH = {"config2": 1024, "config3": 4096, "config4": 16384}


def qp_bytes(N: int) -> int:
    """Compulsory f64 I/O per QP: x0, window, u_prev in; u0, X, U out."""
    return 8 * (10 * N + 16)


def qp_flops(N: int, iters: np.ndarray, scaling: int = 10, check: int = 25) -> np.ndarray:
    """Algorithmic FP64 flops per QP as implemented, from the kernel's counters
    (ADMM iterations, polish passes, factorizations + passes, line-search trials):
      setup      condensing 50 N (n+1) + Ruiz `scaling` x 3 n^2
      ADMM       (factorizations - passes) x (n^3 + 4 n^2): explicit SPD inverse by the sweep;
                 iterations x (2 n^2 + 30 n): dense inverse product + banded row operators + prox;
                 one termination check per `check` iterations x (2 n^2 + 30 n)
      polish     one full factorization per polish run, then per pass 2 n^2 (inverse product)
                 + 2 n^2 (one rank-1 update of the inverse, a floor: a pass updates every changed
                 row) + 40 n; 4 n^2 for the final refinement; line-search trials x 10 m."""
    n, m = 2 * N, 5 * N
    admm, pol, fact, ls = (iters[:, i].astype(np.float64) for i in range(4))
    f = 50.0 * N * (n + 1) + scaling * 3.0 * n * n
    f = f + np.maximum(fact - pol, 0.0) * (n ** 3 + 4.0 * n * n)
    f = f + admm * (2.0 * n * n + 30.0 * n) + np.floor(admm / check) * (2.0 * n * n + 30.0 * n)
    f = f + (pol > 0) * (n ** 3 + 4.0 * n * n + 4.0 * n * n) + pol * (4.0 * n * n + 40.0 * n)
    f = f + ls * (10.0 * m)
    return f


# ------------------------------------------------------------------ workload + sharding
def make_global_batch(config: str, total: int, horizon: int = 0):
    from mpcqp import scenarios

    if config not in scenarios.CONFIGS:
        raise SystemExit(f"unknown config {config}")
    if horizon:  # development / long-horizon lines: the config's generator at another N
        return scenarios.CONFIGS[config](total, horizon=horizon)
    return scenarios.CONFIGS[config](total)


def shard_bounds(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous shard [lo, hi) of rank `rank`; the first total % world ranks
    take one QP more, so any total splits."""
    base, extra = divmod(int(total), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard_counts(total: int, world: int) -> List[int]:
    return [b - a for a, b in (shard_bounds(total, world, r) for r in range(world))]


def make_batch(config: str, batch_per_gpu: int, world: int, rank: int):
    """Weak-scaling shard: rank `rank`'s contiguous part of a batch_per_gpu x world global batch."""
    b = make_global_batch(config, batch_per_gpu * world)
    lo, hi = shard_bounds(batch_per_gpu * world, world, rank)
    return b.x0[lo:hi], b.ref[lo:hi], b.u_prev[lo:hi], b.horizon, b.name


class DistContext:
    """Rank / world of this process and the collectives the bench uses (no-ops at world 1).
    Tensors live on `device` (CUDA for nccl, CPU for gloo)."""

    def __init__(self, world: int = 1, rank: int = 0, local_rank: int = 0, backend: Optional[str] = None,
                 device=None) -> None:
        self.world, self.rank, self.local_rank, self.backend, self.device = world, rank, local_rank, backend, device
        self._dist = None
        if world > 1:
            import torch.distributed as dist

            self._dist = dist

    @classmethod
    def from_env(cls, backend: str = "nccl") -> "DistContext":
        """One process per GPU as torch.distributed.run starts it (RANK / LOCAL_RANK / WORLD_SIZE)."""
        import torch
        import torch.distributed as dist

        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        # one process per GPU; ranks beyond the visible devices wrap (rehearsal on one GPU)
        dev_index = local_rank % max(1, torch.cuda.device_count())
        device = torch.device("cuda", dev_index)
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            torch.cuda.set_device(dev_index)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=device)
            else:
                dist.init_process_group("gloo")
        torch.cuda.set_device(device)
        ctx = cls(world, rank, local_rank, backend if world > 1 else None, device)
        # gloo collectives take host tensors
        ctx.coll_device = device if backend == "nccl" else torch.device("cpu")
        return ctx

    coll_device = None

    def _cdev(self):
        return self.coll_device if self.coll_device is not None else self.device

    def barrier(self) -> None:
        if self._dist is not None:
            self._dist.barrier()

    def all_reduce(self, t, op: str):
        if self._dist is not None:
            self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX if op == "max" else self._dist.ReduceOp.SUM)
        return t

    def all_gather(self, t) -> list:
        if self._dist is None:
            return [t]
        parts = [t.new_empty(t.shape) for _ in range(self.world)]
        self._dist.all_gather(parts, t)
        return parts

    def close(self) -> None:
        if self._dist is not None:
            self._dist.destroy_process_group()


def timed_steps(step: Callable[[int], None], steps: int, warmup: int, ctx: DistContext,
                sync: Callable[[], None] = lambda: None) -> float:
    """W untimed warmup steps, then EXACTLY `steps` steps bracketed by a barrier + device sync on
    both sides; returns this rank's elapsed seconds (bench.py contract)."""
    for _ in range(warmup):
        step(-1)
    sync()
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    sync()
    ctx.barrier()
    return time.perf_counter() - t0


def reduce_stats(ctx: DistContext, elapsed: float, sums: List[float]) -> Tuple[float, List[float]]:
    """MAX over ranks of the elapsed time, SUM of the counters."""
    import torch

    t = torch.tensor([elapsed], dtype=torch.float64, device=ctx._cdev())
    s = torch.tensor([float(v) for v in sums], dtype=torch.float64, device=ctx._cdev())
    ctx.all_reduce(t, "max")
    ctx.all_reduce(s, "sum")
    return float(t.item()), [float(v) for v in s.cpu().tolist()]


def gather_scalar(ctx: DistContext, v: float) -> List[float]:
    """Every rank's value of a per-rank scalar, in rank order (one all_gather; [v] at world 1): the
    per-rank elapsed times beside the MAX over ranks, so shard imbalance is visible."""
    import torch

    t = torch.tensor([float(v)], dtype=torch.float64, device=ctx._cdev())
    return [float(p.item()) for p in ctx.all_gather(t)]


def gather_rows(ctx: DistContext, t, counts: List[int]):
    """All ranks' shards of a row-distributed tensor, concatenated in rank order (shards of
    unequal length are padded to the largest for the collective)."""
    import torch

    if ctx.world == 1:
        return t
    m = max(counts)
    pad = t.new_zeros((m,) + tuple(t.shape[1:]))
    pad[: t.shape[0]] = t
    parts = ctx.all_gather(pad.to(ctx._cdev()))
    return torch.cat([p[:c] for p, c in zip(parts, counts)])


# ------------------------------------------------------------------ launcher (--gpus N without torchrun)
def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_cmd(gpus: int, argv: List[str], script: Optional[str] = None, port: Optional[int] = None) -> List[str]:
    """The command the parent runs for `bench.py --gpus N` started without torch.distributed.run: the
    driver's own launch line (one rank per GPU, rendezvous on 127.0.0.1) around this script."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(gpus)}",
            "--master-addr=127.0.0.1", f"--master-port={port or free_port()}", script or str(Path(__file__).resolve()),
            *argv]


def launch_ranks(gpus: int, argv: List[str], script: Optional[str] = None) -> int:
    """Parent process of a multi-GPU run: starts `gpus` ranks (torch.distributed.run as a child; this
    process never touches the GPU, so no rank is exec'd from a GPU-initialised process), lets rank 0's
    JSON line through on the shared stdout, and returns non-zero when any rank failed (the launcher
    tears the other ranks down and exits non-zero then)."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK"):
        env.pop(k, None)
    import subprocess

    return subprocess.run(rank_launch_cmd(gpus, argv, script), env=env).returncode


def world_mismatch(gpus: int, env: Optional[Dict[str, str]] = None) -> Optional[str]:
    """An error message when the ranks that were started disagree with --gpus, else None."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is not None and int(ws) != int(gpus):
        return f"--gpus {gpus} but WORLD_SIZE={ws}: launch one rank per GPU (--nproc-per-node {gpus}) or fix --gpus"
    return None


# ------------------------------------------------------------------ checker / CPU baseline leg
def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def host_threads() -> Tuple[int, int]:
    """(threads to use, cores visible to this process).  All visible cores, unless the host
    assigns this job a share through OMP_NUM_THREADS (the GPU box sets 16 per GPU)."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        visible = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    threads = min(visible, int(env)) if env and env.isdigit() and int(env) > 0 else visible
    return threads, visible


def cgroup_cpu_quota() -> Optional[float]:
    """Cores this process's cgroup may use (cpu.max quota / period), None when unlimited or unknown: on
    the GPU box the affinity mask shows the whole node while the job's CPU share is far smaller."""
    for f in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(f).read().split()[:2]
            return None if q == "max" else int(q) / int(per)
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def spot_check(params, x0, ref, u_prev, U, active, status, idx, iters=None, settings=None) -> dict:
    """Checker: the GPU solutions of QPs `idx` against the C restatement, whose polish ends at the
    exact optimum of the QP (strictly convex: the same optimum OSQP+polish returns in the
    reference).  Parity against OSQP itself is unpinned here (OSQP is not installed)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import cpu_solver

    idx = np.asarray(idx)
    threads, _ = host_threads()
    out = cpu_solver.cpu_solve(params, x0[idx], ref[idx], u_prev[idx], nthreads=threads, **(settings or {}))
    Uc = out["U"].reshape(len(idx), -1)
    Ug = np.asarray(U)[idx].reshape(len(idx), -1)
    err = np.abs(Ug - Uc).max(axis=1) / np.maximum(1.0, np.abs(Uc).max(axis=1))
    res = {
        "vs": "exact optimum (C restatement's polish, oracle/mpcqp_cpu.c); OSQP itself is absent, "
              "so parity with OSQP's own iterates is unpinned",
        "qps": int(len(idx)),
        "max_rel_err_U": float(err.max()) if len(idx) else 0.0,
        "active_set_mismatches": int((np.asarray(active)[idx] != out["active"]).any(axis=1).sum()),
        "status_mismatches": int((np.asarray(status)[idx] != out["status"]).sum()),
    }
    if iters is not None and len(idx):
        # iteration indexing: the fraction of QPs whose four counters (ADMM iterations, polish passes,
        # factorizations, line-search trials) equal the C restatement's; the fast kernel's wave-tree
        # reductions round differently from the sequential sums (reproducible = 1 agrees on all)
        it = np.asarray(iters)[idx]
        same = it == out["iters"]
        res["iters_agreement"] = float(same.all(axis=1).mean())
        res["iters_agreement_per_counter"] = {k: float(same[:, i].mean()) for i, k in
                                              enumerate(("admm", "polish", "factorizations", "ls_trials"))}
    return res


def cpu_baseline(params, x0, ref, u_prev, seconds: float, settings=None) -> dict:
    """The C restatement (oracle/, kind "port") on the host cores, bounded sample."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import cpu_solver

    threads, visible = host_threads()
    cpu_solver.cpu_solve(params, x0[:64], ref[:64], u_prev[:64], nthreads=threads, **(settings or {}))  # warm (build + page-in)
    done, solved, t0 = 0, 0, time.perf_counter()
    while True:
        out = cpu_solver.cpu_solve(params, x0, ref, u_prev, nthreads=threads, **(settings or {}))
        done += len(x0)
        solved += int((out["status"] == 1).sum())
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    # the 1-core figure SURVEY.md 8(d) asks for beside the all-core one (a short slice)
    n1, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < min(3.0, seconds / 3):
        out1 = cpu_solver.cpu_solve(params, x0[:256], ref[:256], u_prev[:256], nthreads=1, **(settings or {}))
        n1 += int((out1["status"] == 1).sum())
    dt1 = time.perf_counter() - t1
    # every core this process may use (SURVEY.md 8(d) "the host's cores"): the affinity mask capped by
    # the cgroup's CPU quota (on the GPU box the mask shows the whole node, 256 cores, while the job's
    # quota is 16: more threads than that only oversubscribe the quota)
    quota = cgroup_cpu_quota()
    all_threads = max(1, min(visible, int(np.ceil(quota)))) if quota else visible
    if all_threads == threads:  # the share above is already every usable core
        na, dta = solved, dt
    else:
        na, ta = 0, time.perf_counter()
        while True:
            outa = cpu_solver.cpu_solve(params, x0, ref, u_prev, nthreads=all_threads, **(settings or {}))
            na += int((outa["status"] == 1).sum())
            if time.perf_counter() - ta >= min(5.0, max(1.0, seconds / 2)):
                break
        dta = time.perf_counter() - ta
    return {
        "value": solved / dt,
        "unit": "QP/s",
        "cores": threads,
        "kind": "port",
        "threads": threads,
        "host_cores_visible": visible,
        "value_1core": n1 / dt1,
        "value_all_cores": na / dta,
        "threads_all_cores": all_threads,
        "cgroup_cpu_quota_cores": quota,
        "cpu_model": _cpu_model(),
        "sample": f"{done} QPs ({done // len(x0)} passes over this rank's batch) in {dt:.1f} s on {threads} "
                  f"OpenMP threads: the host's CPU share of this GPU (OMP_NUM_THREADS; {visible} cores are "
                  f"visible to the process, shared with the node's other GPUs); C restatement of the same "
                  f"ADMM+polish algorithm (oracle/mpcqp_cpu.c); value_1core: one thread on 256 QPs; "
                  f"value_all_cores: every core this process may use -- the {visible} visible cores capped by "
                  f"the cgroup CPU quota ({quota if quota else 'none'}) -- {all_threads} threads on the same "
                  f"batch ({dta:.1f} s{'; the same run as value' if all_threads == threads else ''})",
    }


def config5_swarm_sharded(ctx: DistContext, vehicles: int = 100) -> Optional[dict]:
    """BASELINE config 5 on `ctx.world` GPUs: the same swarm as config5_swarm, its vehicles sharded
    contiguously over the ranks (mpcqp.pipeline.swarm.run_swarm_sharded: every vehicle keeps its own
    seed, so it does exactly what it does on one GPU; one all_gather_object of the per-vehicle results
    at the end).  Timed between barriers, MAX over ranks; rank 0 then runs the whole swarm alone on its
    own GPU and compares vehicle for vehicle.  Returns the record on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    from mpcqp.pipeline.swarm import Swarm, run_swarm_sharded, shard_vehicles

    occ, starts, goals, mpc, planner = _config5_inputs(vehicles)
    lo, hi = shard_vehicles(vehicles, ctx.world, ctx.rank)
    sw = Swarm(occ, mpc, planner, map_resolution=0.8, max_vehicles=max(1, hi - lo), device=ctx.device,
               replan_distance=5.5, max_replans=2, fused=True)
    sw.run(starts[:4], goals[:4], seeds=np.arange(4), sim_steps=5)  # warm
    torch.cuda.synchronize(ctx.device)
    ctx.barrier()
    t0 = time.perf_counter()
    res = run_swarm_sharded(sw.run, starts, goals, np.arange(vehicles), rank=ctx.rank, world=ctx.world,
                            all_gather_object=dist.all_gather_object, check_every=50)
    torch.cuda.synchronize(ctx.device)
    ctx.barrier()
    T, _ = reduce_stats(ctx, time.perf_counter() - t0, [0.0])
    if ctx.rank != 0:
        return None
    one = Swarm(occ, mpc, planner, map_resolution=0.8, max_vehicles=vehicles, device=ctx.device,
                replan_distance=5.5, max_replans=2, fused=True)
    ref = one.run(starts, goals, seeds=np.arange(vehicles), check_every=50)
    same = (np.array_equal(res.steps, ref.steps) and np.array_equal(res.phase, ref.phase)
            and np.array_equal(res.replans, ref.replans)
            and all(np.array_equal(a, b) for a, b in zip(res.states, ref.states)))
    vsteps = int(res.steps.sum())
    return {
        "workload": f"config5: {vehicles} vehicles sharded over {ctx.world} ranks ({shard_vehicles(vehicles, ctx.world, 0)[1]} "
                    f"on rank 0), default inflated grid, N=15, replan trigger 5.5 px, <= 2 replans per vehicle",
        "n_gpus": ctx.world,
        "seconds": T,
        "vehicle_steps": vsteps,
        "vehicle_steps_per_s": vsteps / T,
        "goal_reached": int((res.phase == 1).sum()),
        "replans": int(res.replans.sum()),
        "identical_to_one_gpu_swarm": bool(same),
        "note": "end to end per rank (planning, references, tracking with replanning; fused loop) plus the "
                "all_gather_object of the results, between barriers, MAX over ranks; compared vehicle for "
                "vehicle with the whole swarm run on rank 0's GPU alone",
    }


def _config5_inputs(vehicles: int):
    from mpcqp.config import MPCConfig
    from mpcqp.planning.rrt_star import default_planner_parameters

    occ = np.load(ROOT / "rrt-mpc_amd" / "mpcqp" / "data" / "default_plan.npz")["occupancy"]
    rng = np.random.default_rng(5)
    free = np.argwhere(occ == 1)
    starts, goals = [], []
    while len(starts) < vehicles:  # start / goal pairs at least 30 px apart on free cells
        a, b = free[rng.integers(0, len(free), 2)]
        if np.hypot(*(a - b)) > 30:
            starts.append(a[::-1].astype(float))
            goals.append(b[::-1].astype(float))
    return occ, np.array(starts), np.array(goals), MPCConfig(horizon=15, sim_steps=300), default_planner_parameters()


def config5_swarm(vehicles: int = 100) -> dict:
    """BASELINE config 5 on one GPU (the N-GPU run shards the vehicles: config5_swarm_sharded): a swarm of
    `vehicles` on the default inflated grid -- batched RRT* plans, device references, the closed loop
    with the per-step replan trigger and replanning -- through the fused swarm loop
    (mpcqp_swarm_loop), timed end to end, and checked vehicle for vehicle against the graph-stepped
    swarm (mpcqp_swarm_run), whose per-step operations it fuses."""
    import torch
    from mpcqp.pipeline.swarm import Swarm

    occ, starts, goals, mpc, planner = _config5_inputs(vehicles)
    runs = {}
    for fused in (True, False):
        sw = Swarm(occ, mpc, planner, map_resolution=0.8, max_vehicles=vehicles,
                   device="cuda:0", replan_distance=5.5, max_replans=2, fused=fused)
        sw.run(starts[:4], goals[:4], seeds=np.arange(4), sim_steps=5)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = sw.run(starts, goals, seeds=np.arange(vehicles), check_every=50)
        torch.cuda.synchronize()
        runs[fused] = (time.perf_counter() - t0, res)
    dt, res = runs[True]
    ref = runs[False][1]
    same = (np.array_equal(res.steps, ref.steps) and np.array_equal(res.phase, ref.phase)
            and np.array_equal(res.replans, ref.replans)
            and all(np.array_equal(a, b) for a, b in zip(res.states, ref.states)))
    vsteps = int(res.steps.sum())
    return {
        "workload": f"config5: {vehicles} vehicles, default inflated grid, N=15, replan trigger 5.5 px, "
                    f"<= 2 replans per vehicle, 300 steps max",
        "seconds": dt,
        "vehicle_steps": vsteps,
        "vehicle_steps_per_s": vsteps / dt,
        "goal_reached": int((res.phase == 1).sum()),
        "replans": int(res.replans.sum()),
        "stepped_seconds": runs[False][0],
        "identical_to_stepped_swarm": bool(same),
        "timings": {k: round(v, 4) for k, v in res.timings.items()},
        "note": "end to end: planning, references, tracking with replanning (fused loop); the stepped "
                "graph-replay swarm timed beside it and compared vehicle for vehicle",
    }


def config1_closed_loop() -> dict:
    """BASELINE config 1: the default single-vehicle closed loop at horizon 10,
    100 control steps (the loop stops at the goal after ~65 solves), through the drop-in
    TrajectoryTracker.track (one B=1 GPU solve per step, the reference's call pattern,
    control_stage.py:100-150) and through the C restatement's solve on one core (checker leg)."""
    from types import SimpleNamespace

    from mpcqp import scenarios
    from mpcqp.config import MPCConfig, VizConfig
    from mpcqp.pipeline.control_stage import TrajectoryTracker

    sys.path.insert(0, str(ROOT / "oracle"))
    import cpu_solver
    import mpc_oracle as mo

    plan = scenarios.load_default_plan()
    path = [tuple(map(float, q)) for q in plan["path"]]
    mpc = MPCConfig(horizon=10, sim_steps=100)
    tracker = TrajectoryTracker(mpc, VizConfig())
    planning = SimpleNamespace(plan=SimpleNamespace(success=True, path=path))
    maps = SimpleNamespace(start=tuple(plan["start"]), goal=tuple(plan["goal"]))
    tracker.track(planning, maps, map_resolution=0.8, visualize=False)  # warm (workspace, graph)
    # each leg is a ~5 ms host-driven loop: the best of three runs, so one scheduler stall or
    # garbage collection does not set the number (the same rule for all three legs)
    gpu_s = None
    for _ in range(3):
        t0 = time.perf_counter()
        states = tracker.track(planning, maps, map_resolution=0.8, visualize=False).states
        dt = time.perf_counter() - t0
        gpu_s = dt if gpu_s is None else min(gpu_s, dt)

    # the same loop kept on the device: one vehicle of the fused fleet loop (mpcqp_fleet_loop, ONE
    # launch for the whole run: window, QP + relaxed retry, plant and goal test per step on the GPU)
    import torch
    from mpcqp.pipeline.fleet import FleetTracker

    # every leg solves with the B=1 drop-in's latency schedule (mpc_controller.latency_settings)
    from mpcqp.control.mpc_controller import latency_settings

    sched = latency_settings(10)
    ft = FleetTracker(mpc, map_resolution=0.8, max_vehicles=1, max_ref_len=len(plan["path"]) * 8 + 64,
                      device="cuda:0", fused=True, **sched)
    loop_s = setup_s = None
    for _ in range(4):  # warm, then the best of three
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ft.reset_from_plans([plan["path"]], np.asarray(plan["start"])[None], np.asarray(plan["goal"])[None])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        res = ft.run()
        t2 = time.perf_counter()
        if loop_s is None or t2 - t1 < loop_s:
            loop_s, setup_s = t2 - t1, t1 - t0
    loop_states = np.asarray(res.states[0])
    ft.close()

    params = mpc.to_parameters(0.8)
    from mpcqp.control.ref_builder import build_reference

    ref_g = build_reference(plan["path"], mpc.v_px_s, 10, mpc.dt)

    def c_loop(settings):
        def c_solve(p, state, window, u_prev):
            o = cpu_solver.cpu_solve(p, state[None], window[None], u_prev[None], nthreads=1, **settings)
            if int(o["status"][0]) not in (1, 2):
                return None, None, None
            return o["u0"][0], o["X"][0], o["U"][0]

        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            st = mo.track_loop(params, ref_g, plan["start"], float(plan["yaw0"]), plan["goal"], 100, c_solve)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best, st

    cpu_s, c_states = c_loop(sched)
    # the CPU's phase costs differ from the GPU's: its own faster schedule is the batch default
    cpu_default_s, c_default_states = c_loop({})
    dev = max(float(np.abs(np.asarray(states) - np.asarray(c_states)).max()), 0.0) \
        if len(states) == len(c_states) else None
    return {
        "workload": "config1: default plan, horizon 10, sim_steps 100, one vehicle",
        "solves": len(states),
        "gpu_b1_shim_s": gpu_s,
        "gpu_ms_per_step": 1e3 * gpu_s / max(1, len(states)),
        "gpu_device_loop_s": loop_s,
        "gpu_device_loop_setup_s": setup_s,
        "gpu_device_loop_ms_per_step": 1e3 * loop_s / max(1, len(loop_states)),
        "device_loop_steps": len(loop_states),
        "device_loop_max_state_diff_px": float(np.abs(loop_states - np.asarray(states)).max())
        if len(loop_states) == len(states) else None,
        "cpu_restatement_1core_s": cpu_s,
        "cpu_ms_per_step": 1e3 * cpu_s / max(1, len(c_states)),
        "cpu_ms_per_step_default_schedule": 1e3 * cpu_default_s / max(1, len(c_default_states)),
        "max_state_diff_px": dev,
        "polish_schedule": sched,
        "b1_path": "launch" if os.environ.get("MPCQP_B1_SERVER", "1") == "0" else "served",
        "note": "each leg the best of three runs after a warm one, all with the B=1 drop-in's latency "
                "polish schedule (polish_schedule; the batch default is tuned for a batch's slowest QP); "
                "gpu_ms_per_step: the drop-in TrajectoryTracker loop, one B=1 solve per step (b1_path: "
                "'served' = a request to the resident server wave, mpcqp_solve_served, the default; "
                "'launch' = one kernel launch + stream sync per solve, MPCQP_B1_SERVER=0); "
                "gpu_device_loop_ms_per_step: the same loop as one vehicle of the fused device loop "
                "(mpcqp_fleet_loop: one launch for the run, launch to results on the host; the "
                "reference build and fleet buffer setup are gpu_device_loop_setup_s)",
    }


SOLVER_SETTING_FIELDS = ("method", "rho", "sigma", "alpha", "eps_abs", "eps_rel", "adaptive_rho_tolerance", "max_iter",
                         "check_termination", "scaling", "adaptive_rho", "adaptive_rho_interval", "polish",
                         "polish_max_iter", "polish_from", "polish_attempt_max_iter", "polish_near", "reproducible")


def solver_settings(cparams) -> dict:
    """The solver settings of an ``mpcqp_params`` block (the fields after MPCParameters')."""
    return {k: getattr(cparams, k) for k in SOLVER_SETTING_FIELDS}


def settings_key(cparams) -> str:
    """Fingerprint of the solver settings a measurement ran with (keys the committed PMC passes)."""
    import hashlib

    return hashlib.sha256(json.dumps(solver_settings(cparams), sort_keys=True).encode()).hexdigest()[:16]


def lib_key() -> str:
    """Fingerprint of the kernel library the run loads (keys the committed PMC passes): its build id,
    the hash of the sources it was built from (mpcqp_build_id, __graft_entry__.source_hash)."""
    from mpcqp import _lib

    if hasattr(_lib.lib(), "mpcqp_build_id"):
        return _lib.build_id()[:16]
    import hashlib  # a development library without a build id (tools/ab_lib.py)

    return hashlib.sha256(Path(_lib.LIB_PATH).read_bytes()).hexdigest()[:16]


def method_label(cparams) -> str:
    """What ran, against the reference's OSQP call (mpc_controller.py:119-132: rho 0.1, alpha 1.6,
    eps 1e-3/1e-3, max_iter 60000, polish, adaptive_rho, OSQP defaults otherwise)."""
    s = solver_settings(cparams)
    if s["method"] != 0:
        return "newton (semismooth-Newton polish only; not the reference's OSQP call)"
    dev = []
    if s["scaling"] != 10:
        dev.append(f"scaling {s['scaling']} (OSQP default 10)")
    if s["polish"] and (s["polish_from"] > 0 or s["polish_near"] > 0):
        dev.append(f"early polish from ADMM iteration {s['polish_from']} / at {s['polish_near']:g}x the "
                   f"tolerances, <= {s['polish_attempt_max_iter']} passes per attempt (OSQP: one polish after ADMM)")
    dev.append(f"adaptive_rho_interval {s['adaptive_rho_interval']} (OSQP: timing-based)")
    ref = dict(rho=0.1, alpha=1.6, eps_abs=1e-3, eps_rel=1e-3, max_iter=60000, polish=1, adaptive_rho=1, sigma=1e-6)
    for k, v in ref.items():
        if s[k] != v:
            dev.append(f"{k} {s[k]:g} (reference {v:g})")
    return ("admm+polish: OSQP's algorithm with the reference's settings (rho 0.1, alpha 1.6, eps 1e-3/1e-3, "
            "max_iter 60000, polish, adaptive rho); deviations: " + "; ".join(dev))


def load_pmc_traffic(N: int, batch: int, skey: str, lkey: str) -> Tuple[Optional[dict], Optional[str]]:
    """This workload's entry of the committed rocprofv3 PMC summary (HBM bytes, SQ counters) when it
    was measured with the same solver settings and the same kernel library; else (None, reason)."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None, "no committed PMC summary (profiles/pmc_traffic.json)"
    try:
        e = json.loads(p.read_text()).get(f"N{N}_B{batch}")
    except Exception as exc:  # pragma: no cover
        return None, f"unreadable PMC summary: {exc}"
    if not e:
        return None, f"no PMC entry for N={N}, B={batch}"
    if e.get("settings_key") != skey:
        return None, f"PMC entry measured with other solver settings ({e.get('settings_key')} != {skey})"
    if e.get("lib_key") != lkey:
        return None, f"PMC entry measured with another kernel library ({e.get('lib_key')} != {lkey})"
    return e, None


OSQP_SETTINGS = {"scaling": 10, "polish_from": 0, "polish_near": 0.0}


def osqp_settings_leg(params, x0, ref, u_prev, steps: int, warmup: int, device, method: str, extra: dict,
                      check: int) -> Callable[[], dict]:
    """The same batch with OSQP's own defaults where this build's differ (10 Ruiz passes, one polish
    after ADMM stops; mpc_controller.py:119-132 sets nothing else), timed like the headline leg
    (events on the launch stream around each step's solve launch), spot-checked the same way.
    Runs its GPU part now and returns the function that builds its record (host copies and the
    spot check), so the caller can run its GPU legs back to back and check afterwards."""
    import torch

    from mpcqp import _lib
    from mpcqp.control.mpc_controller import BatchedMPCController

    B, N = len(x0), int(params.horizon)
    sett = {**extra, **OSQP_SETTINGS}
    ctrl = BatchedMPCController(params, max(1, B), device=device, method=method, **sett)
    try:
        x0_t, ref_t, up_t = (torch.from_numpy(a).to(device) for a in (x0, ref, u_prev))
        L = _lib.lib()
        stream = torch.cuda.current_stream(device)
        s = ctypes.c_void_p(stream.cuda_stream)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]

        def step(k: int) -> None:
            if k >= 0:
                ev[k][0].record(stream)
            _lib.check(L.mpcqp_build(ctrl._ws, B, x0_t.data_ptr(), ref_t.data_ptr(), up_t.data_ptr(), s), "build")
            _lib.check(L.mpcqp_solve(ctrl._ws, B, ctrl._u0.data_ptr(), ctrl._X.data_ptr(), ctrl._U.data_ptr(),
                                     ctrl._status.data_ptr(), ctrl._iters.data_ptr(), ctrl._active.data_ptr(), s),
                       "solve")
            if k >= 0:
                ev[k][1].record(stream)

        elapsed = timed_steps(step, steps, warmup, DistContext(), lambda: torch.cuda.synchronize(device))
    except BaseException:
        ctrl.close()
        raise

    def finish() -> dict:
        try:
            return _osqp_record(ctrl, ev, elapsed, steps, params, x0, ref, u_prev, check, sett)
        finally:
            ctrl.close()

    return finish


def _osqp_record(ctrl, ev, elapsed, steps, params, x0, ref, u_prev, check, sett) -> dict:
    B, N = len(x0), int(params.horizon)
    k2_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    status = ctrl._status[:B].cpu().numpy()
    iters = ctrl._iters[:B].cpu().numpy()
    flops = qp_flops(N, iters, scaling=int(ctrl._cparams.scaling), check=int(ctrl._cparams.check_termination))
    tf = float(flops.sum()) / (k2_ms * 1e-3) / 1e12
    out = {
        "value": float((status == 1).sum()) * steps / elapsed,
        "unit": "QP/s",
        "ms_per_step": 1e3 * elapsed / steps,
        "k_solve_ms": k2_ms,
        "method": method_label(ctrl._cparams),
        "solver_settings": solver_settings(ctrl._cparams),
        "solved_fraction": float((status == 1).mean()),
        "iters_mean": {"admm": float(iters[:, 0].mean()), "polish": float(iters[:, 1].mean())},
        "roofline": {"bound": "fp64_valu", "achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": tf / FP64_PEAK_TFLOPS},
        "note": "the headline batch under OSQP's defaults where this build's defaults differ (scaling 10, "
                "polish once after ADMM); same timing rule as the headline line; run before the headline "
                "(its GPU part), checked after it",
    }
    if check > 0:
        idx = np.unique(np.linspace(0, B - 1, min(B, check)).astype(int))
        out["rel_err"] = spot_check(params, x0, ref, u_prev, ctrl._U[:B].cpu().numpy(),
                                    ctrl._active[:B].cpu().numpy(), status, idx, iters, settings=sett)
    return out


def pipelined_leg(params, x0, ref, u_prev, steps: int, warmup: int, device, method: str,
                  extra: dict, streams: int = 2) -> Callable[[object], dict]:
    """The headline batch solved `steps` times with step k on stream k % `streams` (each stream its own
    workspace and outputs), so one batch's dispatch tail -- its slowest QPs, DESIGN.md §5 -- overlaps
    the next batch's start.  Reported beside `value`, never as it: every step is still one whole batch
    with its own build and solve, but `streams` batches may be in flight (a serving front end with
    independent requests; a closed loop whose next batch needs this one's u0 cannot do this).  Runs
    its GPU part now; the returned function takes the headline's U and builds the record."""
    import torch

    from mpcqp import _lib
    from mpcqp.control.mpc_controller import BatchedMPCController

    B = len(x0)
    ctrls = [BatchedMPCController(params, max(1, B), device=device, method=method, **extra) for _ in range(streams)]
    try:
        x0_t, ref_t, up_t = (torch.from_numpy(a).to(device) for a in (x0, ref, u_prev))
        L = _lib.lib()
        strs = [torch.cuda.Stream(device) for _ in range(streams)]
        cur = torch.cuda.current_stream(device)
        for st in strs:  # the inputs were written on the current stream
            st.wait_stream(cur)

        issued = [0]  # warmup steps rotate over the streams too

        def step(k: int) -> None:
            j = issued[0] % streams
            issued[0] += 1
            c, st = ctrls[j], strs[j]
            s = ctypes.c_void_p(st.cuda_stream)
            _lib.check(L.mpcqp_build(c._ws, B, x0_t.data_ptr(), ref_t.data_ptr(), up_t.data_ptr(), s), "build")
            _lib.check(L.mpcqp_solve(c._ws, B, c._u0.data_ptr(), c._X.data_ptr(), c._U.data_ptr(),
                                     c._status.data_ptr(), c._iters.data_ptr(), c._active.data_ptr(), s), "solve")

        elapsed = timed_steps(step, steps, max(warmup, streams), DistContext(),
                              lambda: torch.cuda.synchronize(device))
    except BaseException:
        for c in ctrls:
            c.close()
        raise

    def finish(U_ref) -> dict:
        try:
            solved = float((ctrls[0]._status[:B] == 1).sum().item())
            same = all(torch.equal(c._U[:B], U_ref) for c in ctrls)
            return {
                "value": solved * steps / elapsed,
                "unit": "QP/s",
                "streams": streams,
                "ms_per_step": 1e3 * elapsed / steps,
                "identical_to_headline": bool(same),
                "note": f"the headline batch, step k on stream k % {streams}: consecutive batches overlap, so one "
                        "batch's slowest QPs share the GPU with the next batch's start; same timing rule as "
                        "the headline line (K steps between synchronizations); not the headline value, "
                        "which runs one batch at a time; run before the headline, compared with it after",
            }
        finally:
            for c in ctrls:
                c.close()

    return finish


def strong_leg(ctx: DistContext, steps: int, warmup: int, method: str, extra: dict, total: int = 16384,
               config: str = "config4", check: int = 64, batch=None) -> Callable[[], Optional[dict]]:
    """BASELINE config 4 as strong scaling: a fixed global batch (16384 Monte-Carlo start poses, N = 30)
    split contiguously over the ranks, timed like the headline (warmup, then `steps` steps between
    barriers + device syncs, MAX over ranks), the per-QP results gathered to rank 0 afterwards and
    spot-checked there.  Every world size runs it, N = 1 included, so the driver's per-N lines carry
    the strong-scaling curve beside the weak headline.  Runs its GPU part now and returns the function
    (collective: every rank calls it) that gathers, checks and returns the record on rank 0."""
    import torch

    from mpcqp import _lib
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    batch = batch if batch is not None else make_global_batch(config, total)
    lo, hi = shard_bounds(total, ctx.world, ctx.rank)
    counts = shard_counts(total, ctx.world)
    B = hi - lo
    params = MPCConfig(horizon=batch.horizon).to_parameters(0.8)
    ctrl = BatchedMPCController(params, max(1, B), device=ctx.device, method=method, **extra)
    try:
        x0_t, ref_t, up_t = (torch.from_numpy(a[lo:hi]).to(ctx.device) for a in (batch.x0, batch.ref, batch.u_prev))
        L = _lib.lib()
        stream = torch.cuda.current_stream(ctx.device)
        s = ctypes.c_void_p(stream.cuda_stream)

        def step(k: int) -> None:
            _lib.check(L.mpcqp_build(ctrl._ws, B, x0_t.data_ptr(), ref_t.data_ptr(), up_t.data_ptr(), s), "build")
            _lib.check(L.mpcqp_solve(ctrl._ws, B, ctrl._u0.data_ptr(), ctrl._X.data_ptr(), ctrl._U.data_ptr(),
                                     ctrl._status.data_ptr(), ctrl._iters.data_ptr(), ctrl._active.data_ptr(), s),
                       "solve")

        elapsed = timed_steps(step, steps, warmup, ctx, lambda: torch.cuda.synchronize(ctx.device))
    except BaseException:
        ctrl.close()
        raise

    def finish() -> Optional[dict]:
        try:
            status = ctrl._status[:B]
            rank_s = gather_scalar(ctx, elapsed)
            T, (solved,) = reduce_stats(ctx, elapsed, [float((status == 1).sum().item())])
            g = {k: gather_rows(ctx, t[:B], counts).cpu().numpy() for k, t in
                 (("status", ctrl._status), ("U", ctrl._U), ("active", ctrl._active))}
            if ctx.rank != 0:
                return None
            out = {
                "metric": f"MPC QP solves/s (horizon={batch.horizon}, global batch={total}), strong scaling",
                "workload": batch.name,
                "value": solved * steps / T,
                "unit": "QP/s",
                "n_gpus": ctx.world,
                "scaling": "strong",
                "global_batch": total,
                "batch_per_gpu": counts,
                "ms_per_step": 1e3 * T / steps,
                # each rank's own elapsed time per step (the line's ms_per_step is their MAX): shard imbalance
                "rank_ms_per_step": [1e3 * e / steps for e in rank_s],
                "steps": steps,
                "warmup": warmup,
                "solved_fraction": solved / total,
                "note": "BASELINE config 4: the fixed global batch split over the ranks, the same timing rule as the "
                        "headline (barriers + device syncs around the K steps, MAX over ranks); no data-path "
                        "collective, one gather of the results after timing; run before the headline (its GPU "
                        "part), gathered and checked after it",
            }
            if check > 0:
                idx = np.unique(np.linspace(0, total - 1, min(total, check)).astype(int))
                out["rel_err"] = spot_check(params, batch.x0, batch.ref, batch.u_prev, g["U"], g["active"],
                                            g["status"], idx, settings=extra)
                out["rel_err"]["gathered_qps"] = int(len(g["status"]))
            return out
        finally:
            ctrl.close()

    return finish


# ------------------------------------------------------------------ main
def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # steady state: ~100 untimed steps bring the GPU to its sustained clocks (20 timed after 3 warm
    # steps read ~8 % low: tools/diag/gpu_steps_warmup.sh); the whole default run still takes seconds
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", default="config3", choices=sorted(DEFAULT_BATCH))
    ap.add_argument("--batch", type=int, default=0, help="QPs per GPU, weak scaling (default: the config's)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: a fixed global batch split over the ranks (e.g. 16384 for config 4)")
    ap.add_argument("--horizon", type=int, default=0, help="the config's generator at another horizon N")
    ap.add_argument("--method", default="admm", choices=["admm", "newton"])
    ap.add_argument("--polish-from", type=int, default=None,
                    help="ADMM iteration of the first early polish attempt (default: the library's; 0 = off)")
    ap.add_argument("--polish-near", type=float, default=None,
                    help="residual/tolerance ratio that triggers an early polish (default: the library's; 0 = off)")
    ap.add_argument("--pairing", default="auto", choices=["auto", "on", "off"],
                    help="two QPs per wave for N <= 15 (mpcqp_set_pairing; the same results bit for bit)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="development: override a solver setting of mpcqp_params (repeatable)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length (0 = skip)")
    ap.add_argument("--check-sample", type=int, default=512, help="QPs of the gathered result rank 0 checks")
    ap.add_argument("--event-every", type=int, default=4,
                    help="HIP event pair around every K-th timed step (the kernel time is their mean): a pair "
                         "costs ~7 us of stream time per step it brackets (tools/diag/gpu_event_cost.sh)")
    ap.add_argument("--no-config1", action="store_true", help="skip the config-1 closed-loop line")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 swarm line")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the config-4 strong-scaling leg (16384 QPs, N = 30, split over the ranks)")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the leg that overlaps consecutive batches on two streams")
    ap.add_argument("--no-osqp-settings", action="store_true",
                    help="skip the leg that reruns the batch under OSQP's own scaling / polish defaults")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only to rehearse "
                         "several ranks on one GPU)")
    args = ap.parse_args()
    bad = world_mismatch(args.gpus)
    if bad:
        print(f"bench.py: {bad}", file=sys.stderr)
        return 2
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` on its own: start the N ranks (before anything touches the GPU)
        return launch_ranks(args.gpus, sys.argv[1:])

    import torch

    ctx = DistContext.from_env(args.backend)
    world, rank, device = ctx.world, ctx.rank, ctx.device

    from mpcqp import _lib
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    strong = args.global_batch > 0
    per_gpu = args.batch or DEFAULT_BATCH[args.config]
    total = args.global_batch if strong else per_gpu * world
    batch = make_global_batch(args.config, total, args.horizon)
    N, name = batch.horizon, batch.name
    lo, hi = shard_bounds(total, world, rank)
    counts = shard_counts(total, world)
    B = hi - lo
    x0, ref, u_prev = batch.x0[lo:hi], batch.ref[lo:hi], batch.u_prev[lo:hi]
    params = MPCConfig(horizon=N).to_parameters(0.8)
    extra = {} if args.polish_from is None else {"polish_from": args.polish_from}
    if args.polish_near is not None:
        extra["polish_near"] = args.polish_near
    for kv in args.set:
        k, v = kv.split("=", 1)
        extra[k] = float(v) if "." in v or "e" in v else int(v)
    ctrl = BatchedMPCController(params, max(1, B), device=device, method=args.method, pairing=args.pairing, **extra)
    x0_t = torch.from_numpy(x0).to(device)
    ref_t = torch.from_numpy(ref).to(device)
    up_t = torch.from_numpy(u_prev).to(device)
    L = _lib.lib()
    stream = torch.cuda.current_stream(device)
    s = ctypes.c_void_p(stream.cuda_stream)
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    # K1 is fused into the solve kernel (N <= 32, fast mode, no debug state): mpcqp_build enqueues
    # nothing, so one event pair brackets the step's only kernel (a middle event would add its own
    # ~5 us packet to every step); otherwise k_build and k_solve are timed apart
    fused = N < _lib.WIDE_MIN_HORIZON and not extra.get("reproducible", 0) and not extra.get("debug_state", 0)

    def step(k: int) -> None:
        ev = events[k] if k >= 0 and k % args.event_every == 0 else None
        if ev is not None:
            ev[0].record(stream)
        _lib.check(L.mpcqp_build(ctrl._ws, B, x0_t.data_ptr(), ref_t.data_ptr(), up_t.data_ptr(), s), "build")
        if ev is not None and not fused:
            ev[1].record(stream)
        _lib.check(L.mpcqp_solve(ctrl._ws, B, ctrl._u0.data_ptr(), ctrl._X.data_ptr(), ctrl._U.data_ptr(),
                                 ctrl._status.data_ptr(), ctrl._iters.data_ptr(), ctrl._active.data_ptr(), s),
                   "solve")
        if ev is not None:
            ev[2].record(stream)

    # The secondary legs (OSQP settings and pipelined on one GPU; config 4 strong scaling at every world
    # size) run their GPU parts first, back to back and straight into the headline's warmup; their host
    # work (copies, gathers, spot checks) waits until after the headline.  Together they are ~35 ms of
    # GPU work, more than the MI355X takes to reach its sustained clock from idle (a step
    # takes 203 -> 188 us over its first ~80 launches; 20 steps after 5 warm ones read 8 % low,
    # profiles/r06/warmup_matrix.txt), so the headline's K steps run at the clock the GPU holds under
    # load rather than inside its ramp.  The line records the order (leg_order).
    headline = args.config == "config3" and not args.horizon and not strong
    strong_batch = make_global_batch("config4", 16384) if headline and not args.no_strong else None
    pre_legs = {}
    if world == 1 and not args.no_osqp_settings:
        pre_legs["osqp_settings"] = osqp_settings_leg(params, x0, ref, u_prev, args.steps, args.warmup, device,
                                                      args.method, extra, min(args.check_sample, 256))
    if world == 1 and not args.no_pipelined:
        pre_legs["pipelined"] = pipelined_leg(params, x0, ref, u_prev, args.steps, args.warmup, device,
                                              args.method, extra)
    if strong_batch is not None:  # every rank (collectives in its record step, after the headline)
        pre_legs["strong_config4"] = strong_leg(ctx, args.steps, args.warmup, args.method, extra, batch=strong_batch)
    elapsed = timed_steps(step, args.steps, args.warmup, ctx, lambda: torch.cuda.synchronize(device))
    timed = events[::args.event_every]
    if fused:
        k1_ms = 0.0
        k2_ms = float(np.mean([e[0].elapsed_time(e[2]) for e in timed]))
    else:
        k1_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in timed]))
        k2_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in timed]))

    status = ctrl._status[:B].cpu().numpy()
    iters = ctrl._iters[:B].cpu().numpy()
    flops = qp_flops(N, iters, scaling=int(ctrl._cparams.scaling), check=int(ctrl._cparams.check_termination))
    rank_s = gather_scalar(ctx, elapsed)
    T, (solved_all, flops_all, admm_all, pol_all) = reduce_stats(
        ctx, elapsed, [float((status == 1).sum()), float(flops.sum()), float(iters[:, 0].sum()),
                       float(iters[:, 1].sum())])
    # end-of-run gather of the per-QP results (u0, status, U, active) to every rank
    g = {k: gather_rows(ctx, t[:B], counts) for k, t in
         (("u0", ctrl._u0), ("status", ctrl._status), ("U", ctrl._U), ("active", ctrl._active),
          ("iters", ctrl._iters))}
    g = {k: v.cpu().numpy() for k, v in g.items()}

    if rank == 0:
        value = solved_all * args.steps / T
        ms_per_step = 1000.0 * T / args.steps
        achieved_tf = float(flops.sum()) / (k2_ms * 1e-3) / 1e12  # rank-0 K2 launch, algorithmic flops
        hbm_gbs = total * qp_bytes(N) / (ms_per_step * 1e-3) / 1e9
        skey, lkey = settings_key(ctrl._cparams), lib_key()
        pmc, pmc_reason = load_pmc_traffic(N, B, skey, lkey)
        pmc = pmc or {}
        traffic = pmc.get("k_solve_hbm_bytes_per_launch")
        hw_flops = (pmc.get("k_solve_sq") or {}).get("hw_fp64_flops_per_launch")
        metric = BASELINE_METRIC if (args.config, N, per_gpu, strong) == ("config3", 20, 4096, False) else \
            f"MPC QP solves/s (horizon={N}, {'global batch' if strong else 'batch per GPU'}={total if strong else per_gpu})"
        out = {
            "metric": metric,
            "value": value,
            "unit": "QP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            # each rank's own elapsed time per step (ms_per_step is their MAX): shard imbalance
            "rank_ms_per_step": [1e3 * e / args.steps for e in rank_s],
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: BASELINE config inputs derived from the reference's default RRT* tree "
                    "(tests/golden/gen_golden.py), no external dataset",
            "config": {
                "workload": name,
                "config": args.config,
                "batch_per_gpu": B,
                "global_batch": total,
                "horizon": N,
                "nx": 4,
                "nu": 2,
                "method": method_label(ctrl._cparams),
                "solver_settings": solver_settings(ctrl._cparams),
                # two QPs per wave (mpcqp_set_pairing): only for N <= 15, AUTO past 8 waves per CU
                "pairing": {"mode": args.pairing, "applied": bool(
                    N <= 15 and not extra.get("reproducible", 0) and not extra.get("debug_state", 0) and (
                        args.pairing == "on" or (args.pairing == "auto" and
                                                 B > 8 * torch.cuda.get_device_properties(device).multi_processor_count)))},
                "parallelism": f"dp{world} (independent contiguous shards, {'strong' if strong else 'weak'})",
                "build_id": _lib.build_id() if hasattr(L, "mpcqp_build_id") else None,
            },
            "solved_fraction": solved_all / total,
            "iters_mean": {"admm": admm_all / total, "polish": pol_all / total},
            "kernel_ms": {"mpcqp_build": k1_ms, "k_solve": k2_ms},
            # HIP event pairs on the launch stream around every event_every-th timed step
            "kernel_timing": {"event_pairs": len(timed), "event_every": args.event_every},
            "roofline": {
                "bound": "fp64_valu",
                "achieved": achieved_tf,
                "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved_tf / FP64_PEAK_TFLOPS,
                "traffic": traffic,
                "kernel": "k_solve",
                # the hardware's own count (SQ_INSTS_VALU_FLOPS_FP64, committed PMC pass) over this launch time
                "hw_flops_per_launch": hw_flops,
                "hw_frac": hw_flops / (k2_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS if hw_flops else None,
                # the PMC entry counts only when measured with these settings and this library
                "pmc_key": {"settings": skey, "lib": lkey},
                "pmc_null_reason": pmc_reason,
                "note": "FP64 VALU roof (MI355X FP64 vector peak 78.6 TF; no MFMA is issued: f64 MFMA has "
                        "the same peak and the per-QP matrices are <= 62x62). k_solve is a latency-bound "
                        "FP64 VALU kernel. Flops = bench.qp_flops (as implemented, counted per QP from the "
                        "kernel's iteration counters) / mean k_solve event time on the launch stream "
                        "(event pairs around every event_every-th timed step: kernel_timing).",
            },
            "hbm_roofline": {
                "achieved": hbm_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": hbm_gbs / HBM_PEAK_GBS,
                "bytes_per_qp": qp_bytes(N),
                "note": "compulsory f64 I/O per QP over the whole step; not the binding roof",
            },
        }
        # checker leg: the gathered global result against the C restatement on a strided sample
        if args.check_sample > 0:
            idx = np.unique(np.linspace(0, total - 1, min(total, args.check_sample)).astype(int))
            out["rel_err"] = spot_check(params, batch.x0, batch.ref, batch.u_prev, g["U"], g["active"],
                                        g["status"], idx, g["iters"], settings=extra)
            out["rel_err"]["gathered_qps"] = int(len(g["status"]))
            out["rel_err"]["gathered_solved"] = int((g["status"] == 1).sum())
    # legs every rank takes part in (collectives inside): config 4 as strong scaling at every world size
    # (its GPU part ran before the headline), config 5 sharded by vehicle past one GPU
    if "strong_config4" in pre_legs:
        rec = pre_legs["strong_config4"]()
        if rank == 0:
            out["strong_config4"] = rec
    if headline and world > 1 and not args.no_config5:
        rec = config5_swarm_sharded(ctx)
        if rank == 0:
            out["config5"] = rec
    if rank == 0:
        if "pipelined" in pre_legs:
            out["pipelined"] = pre_legs["pipelined"](ctrl._U[:B])
        if "osqp_settings" in pre_legs:
            out["osqp_settings"] = pre_legs["osqp_settings"]()
        out["leg_order"] = list(pre_legs) + ["headline"]
        if world == 1 and args.cpu_seconds > 0:
            out["cpu_baseline"] = cpu_baseline(params, x0, ref, u_prev, args.cpu_seconds, settings=extra)
        if world == 1 and not args.no_config1:
            out["config1"] = config1_closed_loop()
        if world == 1 and not args.no_config5 and args.config == "config3" and not args.horizon:
            out["config5"] = config5_swarm()
        if world == 1:
            print(json.dumps(out), flush=True)
    ctx.barrier()
    ctrl.close()
    ctx.close()
    if rank == 0 and world > 1:
        # the N-rank line carries the CPU baseline too: rank 0 times it after every rank's GPU legs and
        # collectives are over (the other ranks are leaving, so it does not share their host cores)
        if args.cpu_seconds > 0:
            out["cpu_baseline"] = cpu_baseline(params, x0, ref, u_prev, args.cpu_seconds, settings=extra)
            out["cpu_baseline"]["note"] = (f"measured on rank 0 after the {world} ranks' timed legs: the host CPU "
                                           f"share of one GPU (threads) and one core, on rank 0's shard")
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
