"""Test configuration: import paths, the ``gpu`` marker and shared fixtures."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "rrt-mpc_amd", ROOT / "oracle", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmpcqp.so on the device)")


def load_golden(name: str) -> dict:
    with np.load(GOLDEN / name, allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test without a visible GPU (no CPU fallback exists)")
    import __graft_entry__ as g

    if not g.LIB.exists():  # the snapshot normally carries the in-tree build
        g.build_library()
    return torch.device("cuda:0")
