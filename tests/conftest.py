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


def c1_inputs(g: dict):
    """(U, E, interactions, triplets, train dict, test dict, eval users) of the C1 (--sm shaped) fixture."""
    U, E = int(g["user_num"]), int(g["entity_num"])
    inter = g["interactions"].astype(np.int64)
    trip = g["triplets"].astype(np.int64)
    in_test = np.unpackbits(g["test_mask"])[:len(inter)].astype(bool)
    train, test = {u: [] for u in range(U)}, {u: [] for u in range(U)}
    for (u, i), t in zip(inter.tolist(), in_test.tolist()):
        (test if t else train)[u].append(i)
    train = {u: sorted(v) for u, v in train.items()}
    test = {u: sorted(v) for u, v in test.items()}
    return U, E, inter, trip, train, test, g["eval_users"]


def assert_topk_with_ties(got: np.ndarray, ref: np.ndarray, ref_top_scores: np.ndarray, tol: float = 1e-5) -> int:
    """Top-k rows equal, except where the order of near-equal scores is unspecified (the reference's
    torch.sort / topk): at a row's first differing position j the reference's score must lie within
    tol of a neighbouring rank's (ref_top_scores: its top-(k+1) values).  Returns the excused row count."""
    excused = 0
    for r in np.nonzero((got != ref).any(1))[0]:
        j = int(np.nonzero(got[r] != ref[r])[0][0])
        v = ref_top_scores[r]
        near = min(abs(v[j] - v[j + 1]), abs(v[j] - v[j - 1]) if j else np.inf)
        assert near < tol, (r, j, got[r], ref[r], near)
        excused += 1
    return excused


def assert_metrics_with_ties(got: dict, g: dict, k: int, ref_top_scores: np.ndarray, tol: float = 1e-5) -> None:
    """Per-user precision / recall / nDCG@k equal the reference's, except near-tie rows (as above)."""
    for m in ("precision", "recall", "ndcg"):
        a, b = np.asarray(got[m]), g[f"metrics/{k}/{m}"]
        for r in np.nonzero(~np.isclose(a, b, rtol=1e-5, atol=1e-7, equal_nan=True))[0]:
            assert np.abs(np.diff(ref_top_scores[r])).min() < tol, (m, r, a[r], b[r])
