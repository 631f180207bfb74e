"""Run the wide (GEMM) bi-interaction forward + backward once and save every output (launched by
tests/test_gpu_parity.py::test_dual_gemm_bit_identical_to_separate with KGAT_DUAL_GEMM=0 / 1: the
dual-GEMM launches vs the separate GEMM + um / dxs passes)."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.conftest import load_pkg  # noqa: E402


def main() -> None:
    out_path = sys.argv[1]
    pkg = load_pkg()
    kernels = sys.modules[pkg.__name__ + ".kernels"]
    res = {}
    for din, dout, n in ((256, 256, 70000 + 13), (256, 128, 3000 + 5), (128, 128, 5000 + 3)):
        g = torch.Generator().manual_seed(din + dout)
        X, S = torch.randn(n, din, generator=g), torch.randn(n, din, generator=g)
        W1, W2 = torch.randn(dout, din, generator=g) * 0.1, torch.randn(dout, din, generator=g) * 0.1
        b1, b2 = torch.randn(dout, generator=g) * 0.1, torch.randn(dout, generator=g) * 0.1
        dv = [t.cuda() for t in (X, S, W1, b1, W2, b2)]
        st = kernels.BiState(n, "cuda", din, dout, kind="gemm")
        H = kernels.biinter_fwd(*dv, dropout_p=0.1, seed=5, state=st)
        P1, P2, nrm = (t.clone() for t in st.gemm_views())
        dH = torch.randn(n, dout, generator=g).cuda()
        got = kernels.biinter_bwd(dv[0], dv[1], dH, *dv[2:], dropout_p=0.1, seed=5, H=H, state=st)
        key = f"{din}x{dout}"
        for name, t in zip(("H", "P1", "P2", "norm", "dXd", "dS", "dW1", "db1", "dW2", "db2"),
                           (H, P1, P2, nrm, *got)):
            res[f"{key}_{name}"] = t.detach().cpu().numpy()
    np.savez(out_path, **res)
    print("dual gemm worker ok", os.environ.get("KGAT_DUAL_GEMM"), flush=True)


if __name__ == "__main__":
    main()
