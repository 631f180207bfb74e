"""Microbench of the CF step's fused table update (layer-0 masked A^T product + table Adam,
kgat_spmm_csr_masked_adam_f32) at C2 on a real hop set: the model runs a few train-mode CF steps,
then the pending update of one more backward is launched --reps times on copies of p / m / v
(HIP events), beside the dense Adam pass over the same table.  The synthetic graph and layout are
cached in /tmp, so variant runs (library env switches, one process each) skip the host build:
    python tools/bench_tu.py [--reps 20] [--tag name]
Prints one JSON line: avg / min launch ms of the fused update and of adam_multi."""
from __future__ import annotations

import argparse
import dataclasses
import importlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
PKG = "problem-recommender-system-using-kgat-in-codeforces_amd"
CACHE = Path(os.environ.get("TMPDIR", "/tmp")) / "kgat_tu_c2_cache.npz"


def load_graph(graph_mod):
    if CACHE.exists():
        z = np.load(CACHE)
        f = {k: z[k] for k in z.files}
        lay = graph_mod.GraphLayout(n_nodes=int(f.pop("n_nodes")), rel_order=[int(x) for x in f.pop("rel_order")],
                                    **{k: f[k] for k in ("heads", "rels", "tails", "edge_vals", "rowptr", "col",
                                                         "val", "slot")})
        return int(f["U"]), int(f["E"]), f["inter"], lay
    U, E, inter, trip = graph_mod.synthetic_ckg(1_000_000, 10_000_000, seed=2024)
    lay = graph_mod.build_layout(U, E, inter, trip)
    d = dataclasses.asdict(lay)
    d["rel_order"] = np.asarray(d["rel_order"])
    np.savez(CACHE, U=U, E=E, inter=inter, **d)
    return U, E, inter, lay


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    pkg = importlib.import_module(PKG)
    graph_mod = importlib.import_module(PKG + ".graph")
    K = importlib.import_module(PKG + ".kernels")
    dev = torch.device("cuda:0")
    t0 = time.perf_counter()
    U, E, inter, lay = load_graph(graph_mod)
    torch.manual_seed(2024)
    model = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), cf_embedding_dim=64,
                                  kg_embedding_dim=64, layer_size=[64, 32], message_dropout=[0.1, 0.1]))
    model.attach_graph(lay, dev)
    model.train()
    model.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    model.fuse_table_update = True
    rng = np.random.default_rng(7)
    order = np.argsort(inter[:, 0], kind="stable")
    su = inter[order]
    ustart = np.searchsorted(su[:, 0], np.arange(U + 1))
    have = np.nonzero(np.diff(ustart) > 0)[0]

    def batch():
        u = rng.choice(have, 256, replace=False)
        k = ustart[u] + (rng.random(256) * (ustart[u + 1] - ustart[u])).astype(np.int64)
        return [torch.from_numpy(x.astype(np.int64)).to(dev) for x in (u, su[k, 1], rng.integers(0, E // 10, 256))]

    for _ in range(3):
        loss = model(*batch(), mode=pkg.KGATMode.TRAIN_CF)
        loss.backward()
        model.update_cf_weights()
    loss = model(*batch(), mode=pkg.KGATMode.TRAIN_CF)
    loss.backward()
    tu = model._table_update
    graph, src_map, Xc, Yc, rank = tu.pending
    p = tu.param.data.clone()
    m = torch.rand_like(p) * 1e-3
    v = torch.rand_like(p) * 1e-6
    n_hop = int((src_map >= 0).sum())

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        return sum(ms) / len(ms), min(ms)

    # bits of one launch from these inputs (equal across same-bits variants)
    p1, m1, v1 = p.clone(), m.clone(), v.clone()
    K.spmm_masked_adam(graph, src_map, Xc, Yc, rank, p1, m1, v1, 1e-4, 0.9, 0.999, 0.03, 1e-8)
    digest = [int(t.view(torch.int32).to(torch.int64).sum()) for t in (p1, m1, v1)]
    del p1, m1, v1
    fused = timeit(lambda: K.spmm_masked_adam(graph, src_map, Xc, Yc, rank, p, m, v, 1e-4, 0.9, 0.999, 0.03, 1e-8))
    parts = {}
    if os.environ.get("TU_PARTS"):
        import ctypes
        lib = importlib.import_module(PKG + "._lib")
        csr = graph.AT
        desc = csr.descriptor()
        ws = torch.empty(max(1, csr.n_seg * 64), dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        for k in (1, 2):
            parts[f"part{k}_avg_ms"], parts[f"part{k}_min_ms"] = timeit(lambda: lib.call(
                "kgat_spmm_csr_masked_adam_part_f32", ctypes.byref(desc), src_map.data_ptr(), Xc.data_ptr(),
                Xc.stride(0), Yc.data_ptr() if Yc is not None else None, Yc.stride(0) if Yc is not None else 0, 0,
                rank.data_ptr() if rank is not None else None, p.data_ptr(), m.data_ptr(), v.data_ptr(), 64, 64, 1e-4,
                0.9, 0.999, 0.03, 1e-8, None, k, ws.data_ptr(), ws.numel(), st))
    g = torch.randn_like(p)
    dense = timeit(lambda: K.adam_multi([(p.view(-1), g.view(-1), m.view(-1), v.view(-1), 1e-4, 0.03)], 0.9, 0.999,
                                        1e-8))
    tu.discard()
    print(json.dumps({"tag": a.tag, "env": {k: e for k, e in os.environ.items() if k.startswith("KGAT_")},
                      "n_hop": n_hop, "digest": digest, "fused_avg_ms": fused[0], "fused_min_ms": fused[1], "adam_avg_ms": dense[0],
                      "adam_min_ms": dense[1], **parts, "setup_s": round(time.perf_counter() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
