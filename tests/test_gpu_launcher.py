"""`bench.py --gpus 2` end to end on one GPU: the script starts its two ranks itself (gloo instead of
RCCL, both ranks on cuda:0, as the rehearsal in DESIGN.md §7), each solves its 4096-QP shard of the
8192-QP weak batch, the strong-scaling config-4 leg splits its 16,384 QPs over the two ranks, and
rank 0 prints one line for the whole job with the gathered results checked against the C
restatement; the line carries each rank's step time and the CPU baseline (timed on rank 0 after the
GPU legs)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_two_ranks_on_one_gpu():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "3",
                        "--warmup", "1", "--cpu-seconds", "1", "--no-config1", "--no-config5", "--check-sample", "64"],
                       cwd=str(ROOT), env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # one line for the whole job (rank 0)
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 8192 and d["config"]["batch_per_gpu"] == 4096
    assert d["solved_fraction"] == 1.0
    re_ = d["rel_err"]
    assert re_["gathered_qps"] == 8192 and re_["gathered_solved"] == 8192
    assert re_["active_set_mismatches"] == 0 and re_["status_mismatches"] == 0
    assert re_["max_rel_err_U"] < 1e-8
    s = d["strong_config4"]
    assert s["n_gpus"] == 2 and s["scaling"] == "strong" and s["batch_per_gpu"] == [8192, 8192]
    assert s["solved_fraction"] == 1.0
    # the N-rank line is self-contained: each rank's own step time beside the MAX, and the CPU baseline
    for rec in (d, s):
        assert len(rec["rank_ms_per_step"]) == 2
        assert abs(max(rec["rank_ms_per_step"]) - rec["ms_per_step"]) <= 1e-6 * rec["ms_per_step"] + 1e-9
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["value_1core"] > 0 and cb["cores"] >= 1 and "rank 0" in cb["note"]
