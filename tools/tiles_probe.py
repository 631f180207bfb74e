"""Probe of the row-set bi-interaction forward (kgat_biinter_fwd_tiles_f32) at C2: the first hop F + N(F) of a
256-pair batch (host-marked from the CSR), an empty set, the batch rows F alone, and every row, against the
whole-table launch -- how much of the frontier step's tile launch is the member tiles' math and how much is
the walk over the bitmap.

    python tools/tiles_probe.py [hop,batch,empty,all]

KGAT_TL_OLD=1 selected the round-5 grid-stride walk during the round-6 A/B (the switch is gone from the
library; both legs now run the chunked kernel).  The event timings of small sets are host-bound (~13 us per call of Python checks); under
`rocprofv3 --kernel-trace --stats` with one set per run the kernel durations are the measurement.
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
PKG = "problem-recommender-system-using-kgat-in-codeforces_amd"


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def bitmap(n, members):
    b = np.zeros((n + 31) // 32, np.uint32)
    m = np.unique(members)
    np.bitwise_or.at(b, m >> 5, (np.uint32(1) << (m & 31).astype(np.uint32)))
    return torch.from_numpy(b.view(np.int32)).cuda()


WANT = sys.argv[1].split(",") if len(sys.argv) > 1 else ["hop", "batch", "empty", "all"]
DIMS = [(64, 64), (64, 32)]


def main():
    graph = importlib.import_module(PKG + ".graph")
    K = importlib.import_module(PKG + ".kernels")
    U, E, inter, trip = graph.synthetic_ckg(1_000_000, 10_000_000, seed=2024)
    lay = graph.build_layout(U, E, inter, trip)
    n = lay.n_nodes
    rng = np.random.default_rng(7)
    users = rng.integers(0, U, 256)
    items = np.concatenate([inter[rng.integers(0, len(inter), 256), 1], rng.integers(0, int(E * 0.1), 256)]) + U
    F = np.unique(np.concatenate([users, items]))
    rp, col = lay.rowptr, lay.col
    nbr = np.concatenate([col[rp[r]:rp[r + 1]] for r in F])
    H1 = np.unique(np.concatenate([F, nbr]))
    tiles = lambda s: int(np.unique(s >> 4).size)
    quads = lambda s: int(np.unique(s >> 2).size)
    out = {"F_rows": int(F.size), "F_tiles": tiles(F), "F_quads": quads(F), "hop_rows": int(H1.size),
           "hop_tiles": tiles(H1), "hop_quads": quads(H1), "all_tiles": (n + 15) // 16}
    torch.manual_seed(0)
    for din, dout in DIMS:
        X = torch.randn(n, din, device="cuda")
        S = torch.randn(n, din, device="cuda")
        W1, W2 = torch.randn(dout, din, device="cuda") * 0.1, torch.randn(dout, din, device="cuda") * 0.1
        b1, b2 = torch.randn(dout, device="cuda"), torch.randn(dout, device="cuda")
        H = torch.empty(n, dout, device="cuda")
        st = K.make_state(n, din, dout, X.device)
        res = {}
        sets = (("hop", H1), ("batch", F), ("empty", np.zeros(0, np.int64)), ("all", np.arange(n)))
        for name, mem in [x for x in sets if x[0] in WANT]:
            bits = bitmap(n, mem.astype(np.int64))
            outs = []
            for old in ("1", "0", "1", "0"):  # interleaved: the grid-stride walk (KGAT_TL_OLD=1) vs chunks
                os.environ["KGAT_TL_OLD"] = old
                H.zero_(); st.norm.zero_(); st.mask.zero_()
                K.biinter_fwd_tiles(X, S, W1, b1, W2, b2, 0.1, 5, H, bits, state=st)
                outs.append((H.clone(), st.norm.clone(), st.mask.clone()))
                res[f"{name}_{'walk' if old == '1' else 'chunks'}"] = round(
                    timeit(lambda: K.biinter_fwd_tiles(X, S, W1, b1, W2, b2, 0.1, 5, H, bits, state=st)), 1)
            res[f"{name}_bit_identical"] = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
        os.environ.pop("KGAT_TL_OLD", None)
        out[f"{din}->{dout}"] = res
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
