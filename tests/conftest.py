"""Shared pytest configuration: markers, repo paths and fixture loaders."""
from __future__ import annotations

import importlib
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
PKG_NAME = "problem-recommender-system-using-kgat-in-codeforces_amd"

if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def load_pkg():
    """Import the product package (its directory name is not an identifier)."""
    return importlib.import_module(PKG_NAME)


def golden(name: str) -> dict[str, np.ndarray]:
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


KGAT_CASES = ["L1_d64", "L2_d64", "L3_d64", "L3_d128"]


@pytest.fixture(params=KGAT_CASES)
def kgat_case(request):
    return request.param, golden("kgat_" + request.param)
