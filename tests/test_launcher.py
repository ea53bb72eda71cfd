"""bench.py --gpus N without torch.distributed.run: the parent starts the N ranks itself (before any
GPU call), relays rank 0's JSON line and fails when a rank fails; a WORLD_SIZE that disagrees with
--gpus is refused.  CPU only: the ranks are a gloo stand-in (tests/_rank_stub.py)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
STUB = str(ROOT / "tests" / "_rank_stub.py")


def test_world_mismatch():
    import bench

    assert bench.world_mismatch(2, {}) is None
    assert bench.world_mismatch(2, {"WORLD_SIZE": "2"}) is None
    msg = bench.world_mismatch(8, {"WORLD_SIZE": "1"})
    assert msg and "--gpus 8" in msg and "WORLD_SIZE=1" in msg


def test_launch_command_is_the_drivers():
    import bench

    cmd = bench.rank_launch_cmd(4, ["--gpus", "4", "--steps", "3"], script="x.py", port=29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    assert cmd[-5:] == ["x.py", "--gpus", "4", "--steps", "3"]


@pytest.mark.timeout(180)
def test_launch_ranks_relays_rank0_line(capfd):
    import bench

    rc = bench.launch_ranks(3, ["--gpus", "3", "--backend", "gloo"], script=STUB)
    out = capfd.readouterr().out
    assert rc == 0, out
    lines = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    rec = lines[0]
    assert rec["world"] == 3 and rec["rank_sum"] == 1 + 2 + 3 and rec["master_addr"] == "127.0.0.1"
    assert rec["argv"] == ["--gpus", "3", "--backend", "gloo"]


@pytest.mark.timeout(180)
def test_launch_ranks_fails_when_a_rank_fails(capfd):
    import bench

    rc = bench.launch_ranks(2, ["--fail-rank", "1"], script=STUB)
    capfd.readouterr()
    assert rc != 0


@pytest.mark.timeout(120)
def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3"], env=env, capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
