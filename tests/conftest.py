"""Shared pytest setup: repo root on sys.path, the `gpu` marker, golden loaders."""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device) and libctr_hip.so")


def load_golden(name: str):
    p = GOLDEN / name
    if p.suffix == ".json":
        return json.loads(p.read_text())
    return np.load(p, allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no ROCm device is visible")
    from rl_ctr_prediction_amd._lib import lib
    lib.load()  # the HIP library must load: no fallback
    return torch.device("cuda:0")
