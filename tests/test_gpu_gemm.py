"""kgat_gemm_f32 (csrc/gemm.hip, the hand-written fp32 MFMA GEMM of the wide layers) against an fp64
torch reference of the same product: every transpose combination, ragged M / N / K (tile edges,
K not a multiple of the 16-deep stage), batches and accumulation.  fp32 tolerance: the MFMA is an
exact fp32 fma chain, so |error| <= ~K * 2^-23 * max|a| max|b| -- asserted at 2e-6 * K."""
from __future__ import annotations

import ctypes

import pytest
import torch

from tests.conftest import load_pkg

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return __import__(load_pkg().__name__ + "._lib", fromlist=["_lib"])


def _gemm(lib, ta, tb, A, B, C, M, N, K, batch, acc):
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    lib.call("kgat_gemm_f32", int(ta), int(tb), M, N, K, A.data_ptr(), A.shape[-1], A[0].numel(), B.data_ptr(),
             B.shape[-1], B[0].numel(), C.data_ptr(), C.shape[-1], C[0].numel(), batch, int(acc), st)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K,batch", [(1, 4, 4, 1), (130, 132, 20, 1), (257, 100, 260, 2), (4096, 256, 256, 1),
                                         (256, 260, 4099, 3), (64, 64, 1, 1)])
def test_gemm_matches_fp64(lib, ta, tb, M, N, K, batch):
    if (ta and M % 4) or (not tb and N % 4) or (not ta and K % 4) or (tb and K % 4):
        pytest.skip("contiguous dimension must be a multiple of 4")
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + K)
    A = torch.rand(batch, *((K, M) if ta else (M, K)), device=DEV, generator=g) * 2 - 1
    B = torch.rand(batch, *((N, K) if tb else (K, N)), device=DEV, generator=g) * 2 - 1
    C0 = torch.rand(batch, M, N, device=DEV, generator=g)
    ref = torch.matmul((A.transpose(1, 2) if ta else A).double(), (B.transpose(1, 2) if tb else B).double())
    for acc in (False, True):
        C = C0.clone()
        _gemm(lib, ta, tb, A, B, C, M, N, K, batch, acc)
        want = ref + C0.double() if acc else ref
        err = (C.double() - want).abs().max().item()
        assert err <= 2e-6 * max(K, 1) + 1e-6, (acc, err)


def test_gemm_deterministic_and_rejects_bad_layouts(lib):
    A = torch.randn(1, 1000, 64, device=DEV)
    B = torch.randn(1, 48, 64, device=DEV)
    C1 = torch.empty(1, 1000, 48, device=DEV)
    C2 = torch.empty_like(C1)
    _gemm(lib, False, True, A, B, C1, 1000, 48, 64, 1, False)
    _gemm(lib, False, True, A, B, C2, 1000, 48, 64, 1, False)
    assert torch.equal(C1, C2)
    st = ctypes.c_void_p(0)
    bad = lib.lib().kgat_gemm_f32(0, 1, 1000, 48, 62, A.data_ptr(), 62, 0, B.data_ptr(), 62, 0, C1.data_ptr(), 48, 0,
                                  1, 0, st)
    assert bad != 0  # K not a multiple of 4 along the contiguous dimension
