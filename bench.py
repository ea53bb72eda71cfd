#!/usr/bin/env python3
"""Benchmark: batched bicycle-MPC QP solves/s on MI355X (BASELINE.json metric).

One "step" = one pass of the hot path over one batch resident in HBM:
K1 ``k_build`` (unwrap + linearize) + K2 ``k_solve`` (condense + ADMM/OSQP + polish)
for every QP of the batch.  Default workload = BASELINE config 3 (B=4096 randomised
RRT*-branch references, horizon 20) per GPU; with N GPUs each rank solves its own
contiguous shard of a 4096*N batch (weak scaling, no data-path collective).

    python bench.py --gpus 1 --steps 20 --warmup 3
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints ONE JSON line on rank 0 (driver contract; roofline + cpu_baseline objects).
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

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "rrt-mpc_amd"))
sys.path.insert(0, str(ROOT))

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 dense (vector == matrix), AMD spec
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md


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


def make_batch(config: str, batch_per_gpu: int, world: int, rank: int):
    from mpcqp import scenarios

    total = batch_per_gpu * world
    if config == "config2":
        b = scenarios.config2(total)
    elif config == "config3":
        b = scenarios.config3(total)
    elif config == "config4":
        b = scenarios.config4(total)
    else:
        raise SystemExit(f"unknown config {config}")
    sl = slice(rank * batch_per_gpu, (rank + 1) * batch_per_gpu)
    return b.x0[sl], b.ref[sl], b.u_prev[sl], b.horizon, b.name


BASELINE_METRIC = "MPC QP solves/s (horizon=20, batch=4096) @1/2/4/8 GPU; rel-err vs OSQP"


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(params, x0, ref, u_prev, seconds: float, gpu_U=None, gpu_active=None):
    """The C restatement (oracle/, kind "port") on the host cores, bounded sample.

    As the checker, it also gives the GPU batch's rel-err: the C restatement's polish ends at
    the exact optimum, which is the OSQP+polish optimum of the reference (a strictly convex QP)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import cpu_solver

    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count() or 1
    threads = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)), 16))
    cpu_solver.cpu_solve(params, x0[:64], ref[:64], u_prev[:64], nthreads=threads)  # warm (build + page-in)
    done, t0 = 0, time.perf_counter()
    solved = 0
    while True:
        out = cpu_solver.cpu_solve(params, x0, ref, u_prev, nthreads=threads)
        done += len(x0)
        solved += int((out["status"] == 1).sum())
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    # the 1-core figure SURVEY.md 8(d) asks for beside the all-core one (a short slice)
    n1, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < min(3.0, seconds / 3):
        out1 = cpu_solver.cpu_solve(params, x0[:256], ref[:256], u_prev[:256], nthreads=1)
        n1 += int((out1["status"] == 1).sum())
    dt1 = time.perf_counter() - t1
    parity = None
    if gpu_U is not None:
        Uc = out["U"]
        parity = {
            "vs": "exact optimum (C restatement's polish; = the reference's OSQP+polish optimum)",
            "qps": int(len(Uc)),
            "max_rel_err_U": float(np.max(np.abs(gpu_U - Uc).reshape(len(Uc), -1).max(axis=1)
                                          / np.maximum(1.0, np.abs(Uc).reshape(len(Uc), -1).max(axis=1)))),
            "active_set_mismatches": int((gpu_active != out["active"]).any(axis=1).sum()),
        }
    return parity, {
        "value": solved / dt,
        "unit": "QP/s",
        "cores": threads,
        "kind": "port",
        "value_1core": n1 / dt1,
        "cpu_model": _cpu_model(),
        "sample": f"{done} QPs ({done // len(x0)} passes over this rank's batch) in {dt:.1f} s, "
                  f"C restatement of the same ADMM+polish algorithm (oracle/mpcqp_cpu.c, OpenMP), "
                  f"host {platform.processor() or platform.machine()}",
    }


def load_pmc_traffic(N: int, batch: int):
    """This workload's entry of the committed rocprofv3 PMC summary (HBM bytes, SQ counters), if present."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get(f"N{N}_B{batch}") or None
    except Exception:
        return None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="config3", choices=["config2", "config3", "config4"])
    ap.add_argument("--batch", type=int, default=0, help="QPs per GPU (default: the config's)")
    ap.add_argument("--method", default="admm", choices=["admm", "newton"])
    ap.add_argument("--polish-from", type=int, default=None,
                    help="ADMM iteration of the first early polish attempt (default: the library's; 0 = off)")
    ap.add_argument("--polish-near", type=float, default=None,
                    help="residual/tolerance ratio that triggers an early polish (default: the library's; 0 = off)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="development: override a solver setting of mpcqp_params (repeatable)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length (0 = skip)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo only to rehearse "
                         "several ranks on one GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; ranks beyond the visible devices wrap (rehearsal on one GPU)
    dev_index = local_rank % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_index)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")
    device = torch.device("cuda", dev_index)
    torch.cuda.set_device(device)

    from mpcqp import _lib
    from mpcqp.config import MPCConfig
    from mpcqp.control.mpc_controller import BatchedMPCController

    default_batch = {"config2": 1024, "config3": 4096, "config4": 16384}[args.config]
    B = args.batch or default_batch
    x0, ref, u_prev, N, name = make_batch(args.config, B, world, rank)
    params = MPCConfig(horizon=N).to_parameters(0.8)
    extra = {} if args.polish_from is None else {"polish_from": args.polish_from}
    if args.polish_near is not None:
        extra["polish_near"] = args.polish_near
    for kv in args.set:
        k, v = kv.split("=", 1)
        extra[k] = float(v) if "." in v or "e" in v else int(v)
    ctrl = BatchedMPCController(params, B, device=device, method=args.method, **extra)
    x0_t = torch.from_numpy(x0).to(device)
    ref_t = torch.from_numpy(ref).to(device)
    up_t = torch.from_numpy(u_prev).to(device)
    L = _lib.lib()
    stream = torch.cuda.current_stream(device)
    s = ctypes.c_void_p(stream.cuda_stream)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        _lib.check(L.mpcqp_build(ctrl._ws, B, x0_t.data_ptr(), ref_t.data_ptr(), up_t.data_ptr(), s), "build")
        if ev is not None:
            ev[1].record(stream)
        _lib.check(L.mpcqp_solve(ctrl._ws, B, ctrl._u0.data_ptr(), ctrl._X.data_ptr(), ctrl._U.data_ptr(),
                                 ctrl._status.data_ptr(), ctrl._iters.data_ptr(), ctrl._active.data_ptr(), s),
                   "solve")
        if ev is not None:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    k1_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in events]))
    k2_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in events]))

    status = ctrl._status[:B].cpu().numpy()
    iters = ctrl._iters[:B].cpu().numpy()
    solved = int((status == 1).sum())
    flops = qp_flops(N, iters)
    stats = torch.tensor([elapsed, float(solved), float(flops.sum()), float(iters[:, 0].sum()),
                          float(iters[:, 1].sum())], dtype=torch.float64, device=device)
    if world > 1:
        tmax = stats[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        rest = stats[1:].clone()
        dist.all_reduce(rest, op=dist.ReduceOp.SUM)
        stats = torch.cat([tmax, rest])
    T, solved_all, flops_all, admm_all, pol_all = (float(v) for v in stats.cpu().tolist())

    if rank == 0:
        value = solved_all * args.steps / T
        ms_per_step = 1000.0 * T / args.steps
        achieved_tf = float(flops.sum()) / (k2_ms * 1e-3) / 1e12  # rank-0 K2 launch, algorithmic flops
        hbm_gbs = B * qp_bytes(N) / (ms_per_step * 1e-3) / 1e9
        pmc = load_pmc_traffic(N, B) or {}
        traffic = pmc.get("k_solve_hbm_bytes_per_launch")
        hw_flops = (pmc.get("k_solve_sq") or {}).get("hw_fp64_flops_per_launch")
        metric = BASELINE_METRIC if (args.config, N, B) == ("config3", 20, 4096) else \
            f"MPC QP solves/s (horizon={N}, batch={B} per GPU)"
        out = {
            "metric": metric,
            "value": value,
            "unit": "QP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: BASELINE config 3 inputs derived from the reference's default RRT* tree "
                    "(tests/golden/gen_golden.py), no external dataset",
            "config": {
                "workload": name,
                "config": args.config,
                "batch_per_gpu": B,
                "global_batch": B * world,
                "horizon": N,
                "nx": 4,
                "nu": 2,
                "method": "admm+polish (OSQP algorithm, reference settings)" if args.method == "admm"
                else "newton (polish only)",
                "parallelism": f"dp{world} (independent shards)",
            },
            "solved_fraction": solved_all / (B * world),
            "iters_mean": {"admm": admm_all / (B * world), "polish": pol_all / (B * world)},
            "kernel_ms": {"k_build": k1_ms, "k_solve": k2_ms},
            "roofline": {
                "bound": "mfma",
                "achieved": achieved_tf,
                "peak": FP64_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved_tf / FP64_PEAK_TFLOPS,
                "traffic": traffic,
                "kernel": "k_solve",
                # the hardware's own count (SQ_INSTS_VALU_FLOPS_FP64, committed PMC pass) over this launch time
                "hw_flops_per_launch": hw_flops,
                "hw_frac": hw_flops / (k2_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS if hw_flops else None,
                "note": "FP64 compute roof (MI355X FP64 vector peak == FP64 matrix peak); k_solve is a "
                        "latency-bound FP64 VALU kernel. Flops = bench.qp_flops (as implemented, counted "
                        "per QP from the kernel's iteration counters) / mean k_solve event time.",
            },
            "hbm_roofline": {
                "achieved": hbm_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": hbm_gbs / HBM_PEAK_GBS,
                "bytes_per_qp": qp_bytes(N),
                "note": "compulsory f64 I/O per QP over the whole step (K1+K2); not the binding roof",
            },
        }
        if world == 1 and args.cpu_seconds > 0:
            out["rel_err"], out["cpu_baseline"] = cpu_baseline(
                params, x0, ref, u_prev, args.cpu_seconds, ctrl._U[:B].cpu().numpy(), ctrl._active[:B].cpu().numpy())
        print(json.dumps(out), flush=True)
    ctrl.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
