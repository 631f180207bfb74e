"""CPU-only checks of the product host code and the C-ABI library boundary.

No GPU compute is launched here: the library is only loaded and its host-side
helper (kgat_csr_plan) called.
"""
from __future__ import annotations

import ctypes
import re

import numpy as np
import pytest
import torch

from oracle import kgat_cpu as K
from tests.conftest import ROOT, golden, load_pkg

pkg = load_pkg()
graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])
_lib = __import__(pkg.__name__ + "._lib", fromlist=["_lib"])


def test_header_symbols_are_bound_and_exported():
    header = (ROOT / "include" / "kgat_hip.h").read_text()
    declared = set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]*?\b(kgat_\w+)\s*\(", header, re.M))
    bound = set(_lib.exported_symbols())
    assert declared == bound, (declared ^ bound)
    lib = _lib.lib()
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.kgat_version() >= 1
    assert b"invalid" in lib.kgat_strerror(1001)


def test_masked_adam_block_rejects_bad_arguments():
    """kgat_spmm_csr_masked_adam_block_f32 validates before it touches the device: a negative yc_row0
    and a null table are refused with KGAT_ERR_INVALID (host-side checks only)."""
    lib = _lib.lib()
    desc = _lib.CSR()
    fake = ctypes.c_void_p(16)  # never dereferenced: the argument checks fail first
    args = dict(row0=0, p=fake)

    def call(**kw):
        a = {**args, **kw}
        return lib.kgat_spmm_csr_masked_adam_block_f32(ctypes.byref(desc), fake, fake, 64, None, 0, a["row0"], None,
                                                       a["p"], fake, fake, 64, 64, 1e-3, 0.9, 0.999, 1.0, 1e-8, None,
                                                       None, 0, None)
    invalid = 1001
    assert b"invalid" in lib.kgat_strerror(invalid)
    assert call(row0=-1) == invalid
    assert call(p=None) == invalid


@pytest.mark.parametrize("case", ["L1_d64", "L2_d64", "L3_d128"])
def test_layout_matches_reference_preprocess(case):
    g = golden("kgat_" + case)
    U, E = int(g["user_num"]), int(g["entity_num"])
    lay = graph.build_layout(U, E, g["interactions"], g["triplets"])
    assert lay.rel_order == g["adjacency_relations"].tolist()
    np.testing.assert_array_equal(lay.heads, g["kg_heads"])
    np.testing.assert_array_equal(lay.rels, g["kg_rels"])
    np.testing.assert_array_equal(lay.tails, g["kg_tails"])
    np.testing.assert_allclose(lay.edge_vals, g["kg_vals"], rtol=1e-6)
    rows, cols, vals = lay.coo()
    np.testing.assert_array_equal(np.vstack([rows, cols]), g["A_idx"])
    np.testing.assert_allclose(vals, g["A_val"], rtol=1e-6)
    # CSR slot of every edge points at its (head, tail) entry
    assert np.all(rows[lay.slot] == lay.heads) and np.all(cols[lay.slot] == lay.tails)


def test_degree_weights_match_oracle():
    g = golden("kgat_L2_d64")
    n = int(g["user_num"]) + int(g["entity_num"])
    h, r, t = g["kg_heads"], g["kg_rels"], g["kg_tails"]
    w = graph.degree_weights(h, t, r, n)
    for rel in np.unique(r):
        sel = r == rel
        hh, tt = torch.from_numpy(h[sel]), torch.from_numpy(t[sel])
        dh = torch.bincount(hh, minlength=n)
        dt = torch.bincount(tt, minlength=n)
        ref = 1.0 / (torch.log1p(dh[hh]) + torch.log1p(dt[tt]))
        np.testing.assert_allclose(w[sel], ref.numpy(), rtol=1e-6)


def test_long_row_plan_matches_c_helper():
    rng = np.random.default_rng(0)
    deg = rng.integers(0, 40, 5000)
    deg[rng.integers(0, 5000, 30)] = rng.integers(300, 5000, 30)
    rowptr = np.zeros(deg.size + 1, np.int64)
    np.cumsum(deg, out=rowptr[1:])
    lr, off, sr, sb = graph.long_row_plan(rowptr, 256, 512)
    lib = _lib.lib()
    nl, ns = ctypes.c_int32(), ctypes.c_int32()
    rp = np.ascontiguousarray(rowptr)
    assert lib.kgat_csr_plan(rp.ctypes.data, deg.size, 256, 512, ctypes.byref(nl), ctypes.byref(ns),
                             None, None, None, None) == 0
    assert (nl.value, ns.value) == (lr.size, sr.size)
    a, b = np.zeros(nl.value, np.int32), np.zeros(nl.value + 1, np.int32)
    c, d = np.zeros(ns.value, np.int32), np.zeros(ns.value, np.int64)
    assert lib.kgat_csr_plan(rp.ctypes.data, deg.size, 256, 512, ctypes.byref(nl), ctypes.byref(ns),
                             a.ctypes.data, b.ctypes.data, c.ctypes.data, d.ctypes.data) == 0
    for x, y in ((a, lr), (b, off), (c, sr), (d, sb)):
        np.testing.assert_array_equal(x, y)
    # segments tile every long row exactly
    for i, r in enumerate(lr):
        begs = sb[off[i]:off[i + 1]]
        assert begs[0] == rowptr[r] and np.all(np.diff(begs) == 512) and begs[-1] < rowptr[r + 1]


def _plan_cols_loops(rowptr, col, T, seg_len, col_block, min_piece):
    """Pure-Python statement of kgat_csr_plan_cols' cut rule (small cases only)."""
    lr, off, sr, sb = [], [0], [], []
    for r in range(rowptr.size - 1):
        a, b = int(rowptr[r]), int(rowptr[r + 1])
        if b - a <= T:
            continue
        lr.append(r)
        s = a
        for i in range(a + 1, b):
            if i - s >= seg_len or (col[i] // col_block != col[i - 1] // col_block and i - s >= min_piece):
                sr.append(r)
                sb.append(s)
                s = i
        sr.append(r)
        sb.append(s)
        off.append(len(sr))
    return [np.array(x, dt) for x, dt in ((lr, np.int32), (off, np.int32), (sr, np.int32), (sb, np.int64))]


@pytest.mark.parametrize("col_block,min_piece", [(64, 8), (1000, 32), (1 << 30, 32)])
def test_long_row_plan_cols(col_block, min_piece):
    """kgat_csr_plan_cols == its loop statement; segments tile each long row, hold <= seg_len entries and
    cross no col_block boundary once they hold min_piece; an unreachable col_block is kgat_csr_plan's plan."""
    rng = np.random.default_rng(col_block)
    deg = rng.integers(0, 40, 3000)
    deg[rng.integers(0, 3000, 25)] = rng.integers(300, 3000, 25)
    rowptr = np.zeros(deg.size + 1, np.int64)
    np.cumsum(deg, out=rowptr[1:])
    col = np.concatenate([np.sort(rng.choice(20000, d, replace=False)) for d in deg]).astype(np.int32)
    got = graph.long_row_plan_cols(rowptr, col, 256, 512, col_block, min_piece)
    want = _plan_cols_loops(rowptr, col, 256, 512, col_block, min_piece)
    for x, y in zip(got, want):
        np.testing.assert_array_equal(x, y)
    lr, off, sr, sb = got
    for i, r in enumerate(lr):
        begs = np.r_[sb[off[i]:off[i + 1]], rowptr[r + 1]]
        assert begs[0] == rowptr[r] and np.all(np.diff(begs) >= 1) and np.all(np.diff(begs) <= 512)
    if col_block >= 1 << 30:
        for x, y in zip(got, graph.long_row_plan(rowptr, 256, 512)):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("n_seg", [0, 1, 5, 37, 64, 1001])
def test_seg_launch_order_matches_c_helper(n_seg):
    """kgat_csr_seg_order == graph.seg_launch_order; a permutation of the segments (padding = n_seg);
    the slots of blocks sharing an XCD (b % 8) hold one contiguous run of the column-sorted list."""
    rng = np.random.default_rng(n_seg)
    col = rng.integers(0, 1 << 20, 4096).astype(np.int32)
    seg_beg = rng.integers(0, col.size, n_seg).astype(np.int64)
    order = graph.seg_launch_order(col, seg_beg)
    nb = (n_seg + 3) // 4
    assert order.dtype == np.int32 and order.size == 4 * nb
    c = np.zeros(max(4 * nb, 1), np.int32)
    assert _lib.lib().kgat_csr_seg_order(col.ctypes.data, seg_beg.ctypes.data, n_seg, c.ctypes.data) == 0
    np.testing.assert_array_equal(c[:order.size], order)
    real = order[order < n_seg]
    np.testing.assert_array_equal(np.sort(real), np.arange(n_seg))
    assert np.count_nonzero(order == n_seg) == 4 * nb - n_seg
    by_col = np.argsort(col[seg_beg], kind="stable")
    run = []
    for x in range(8):
        for b in range(x, nb, 8):
            run.extend(order[4 * b:4 * b + 4].tolist())
    np.testing.assert_array_equal(np.array([s for s in run if s < n_seg], np.int64), by_col)


def test_synthetic_ckg_shape():
    U, E, inter, trip = graph.synthetic_ckg(20000, 200000, seed=1)
    assert U == 2000 and E == 18000
    assert inter.shape[1] == 2 and trip.shape[1] == 3
    assert inter[:, 0].max() < U and inter[:, 1].max() < int(E * 0.1)
    assert len(np.unique(inter[:, 0] * E + inter[:, 1])) == len(inter)
    assert set(np.unique(trip[:, 1]).tolist()) <= {0, 1, 2, 3}
    lay = graph.build_layout(U, E, inter, trip)
    assert lay.nnz == 2 * (len(inter) + len(trip))  # every relation has its inverse, no collisions


def test_model_init_matches_reference_rng():
    """Same creation order => the same initial weights as the reference under one seed."""
    g = golden("kgat_L3_d64")
    U, E = int(g["user_num"]), int(g["entity_num"])
    torch.manual_seed(2024)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(g["adjacency_relations"]),
                              layer_size=[64, 32, 16]))
    sd = m.state_dict()
    for k, v in sd.items():
        if v.is_sparse:
            continue
        np.testing.assert_array_equal(v.numpy(), g["init/" + k], err_msg=k)
    assert set(k for k in sd if not sd[k].is_sparse) == {k[5:] for k in g if k.startswith("init/")}


def test_model_refuses_cpu():
    g = golden("kgat_L1_d64")
    U, E = int(g["user_num"]), int(g["entity_num"])
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=10, layer_size=[64]))
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, dtype=torch.long), torch.zeros(2, dtype=torch.long), torch.zeros(2, dtype=torch.long),
          mode=pkg.KGATMode.TRAIN_CF)


def test_oracle_layout_agrees_with_product_layout():
    g = golden("kgat_L3_d128")
    U, E = int(g["user_num"]), int(g["entity_num"])
    lay = graph.build_layout(U, E, g["interactions"], g["triplets"])
    blocks, rel_ids = K.adjacency_blocks(U, [0, 1, 2, 3], g["interactions"], g["triplets"])
    A = K.initial_attentive(U + E, K.normalized_blocks(U + E, blocks))
    np.testing.assert_allclose(lay.coo()[2], A.values().numpy(), rtol=1e-6)


def test_nfm_init_matches_reference_rng():
    g = golden("nfm_h3_d64")
    torch.manual_seed(2024)
    m = pkg.NFM(pkg.NFMArgs(user_num=int(g["user_num"]), item_num=int(g["item_num"]), entity_num=int(g["entity_num"]),
                            embedding_dim=int(g["dim"]), hidden_dim=g["hidden"].tolist()))
    sd = m.state_dict()
    assert set(sd) == {k[5:] for k in g if k.startswith("init/")}
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), g["init/" + k], err_msg=k)


def test_eval_csr_helper_sorts_and_dedups():
    ev = pkg.evaluation
    ptr, idx = ev._csr([[5, 1, 5, 3], [], [2]], "cpu", unique=True)
    assert ptr.tolist() == [0, 3, 3, 4] and idx.tolist() == [1, 3, 5, 2] and idx.dtype == torch.int32
    ptr, idx = ev._csr([[], []], "cpu")
    assert ptr.tolist() == [0, 0, 0] and idx.numel() == 1


def test_reference_checkpoints_load_into_product_models():
    """kgat.pth / nfm.pth in the reference's format (main.py:197-231, NFM/main.py:186-220) load with the
    safe loader and match our state_dict keys and shapes (including the sparse attentive_matrix)."""
    g = golden("kgat_L2_d64")
    ck = torch.load(ROOT / "tests" / "golden" / "kgat_L2_d64_ckpt.pth", map_location="cpu", weights_only=True)
    sd = ck["model_state_dict"]
    m = pkg.KGAT(pkg.KGATArgs(user_num=int(g["user_num"]), entity_num=int(g["entity_num"]),
                              relation_num=len(g["adjacency_relations"]), layer_size=[64, 32]))
    own = m.state_dict()
    assert set(sd) == set(own)
    for k in sd:
        assert sd[k].shape == own[k].shape and sd[k].is_sparse == own[k].is_sparse, k
    m.load_state_dict(sd)
    assert m.attentive_matrix.data._nnz() == sd["attentive_matrix"]._nnz()
    gn = golden("nfm_h3_d64")
    ckn = torch.load(ROOT / "tests" / "golden" / "nfm_h3_d64_ckpt.pth", map_location="cpu", weights_only=True)
    n = pkg.NFM(pkg.NFMArgs(user_num=int(gn["user_num"]), item_num=int(gn["item_num"]),
                            entity_num=int(gn["entity_num"]), embedding_dim=int(gn["dim"]),
                            hidden_dim=gn["hidden"].tolist()))
    n.load_state_dict(ckn["model_state_dict"])


def test_nfm_feature_matrix_matches_reference_construction():
    """NFMBatcher's item feature CSR (built on the host, NFM/preprocess.py:150-193) equals the
    reference's coo_matrix(...).tocsr(): item one-hots plus problem-headed triplet tails, duplicates summed."""
    rng = np.random.default_rng(3)
    I, E = 25, 70
    heads, tails = rng.integers(0, I, 120), rng.integers(I, E, 120)
    b = pkg.NFMBatcher(10, I, E, heads, tails, {0: [1, 2]}, "cpu")
    want = K.nfm_feature_matrix(I, E, heads, tails)
    want.sum_duplicates()
    want.sort_indices()
    np.testing.assert_array_equal(b.feature_rowptr.numpy(), want.indptr)
    np.testing.assert_array_equal(b.feature_col.numpy(), want.indices)
    np.testing.assert_array_equal(b.feature_val.numpy(), want.data.astype(np.float32))
    with pytest.raises(IndexError):
        pkg.NFMBatcher(10, I, E, [I], [I], {0: [1]}, "cpu")


def test_driver_dataset_split_and_early_stopping():
    """driver.py (make train / predict / recommend): the Codeforces-shaped synthetic dataset keeps the
    reference's KG layout and the per-user 80/20 then 90/10 split is disjoint and complete
    (preprocess.py:55-111, 608-614); early_stopping follows main.py:173-195."""
    import importlib
    import math
    drv = importlib.import_module(load_pkg().__name__ + ".driver")
    inter, trip, E = drv.synthetic_codeforces(users=40, problems=300, contests=50, tags=10, ratings=8,
                                              per_user=(10, 60), seed=3)
    assert E == 300 + 50 + 6 + 10 + 8
    assert set(np.unique(trip[:, 1]).tolist()) <= {0, 1, 2, 3}
    assert np.all(trip[trip[:, 1] == 2, 2] >= 300) and np.all(trip[trip[:, 1] == 3, 0] >= 300)
    assert np.unique(inter, axis=0).shape[0] == inter.shape[0]
    tr, va, te = drv.split_interactions(inter, 40, seed=3)
    assert tr.shape[0] + va.shape[0] + te.shape[0] == inter.shape[0]
    for u in range(40):
        a, b, c = (set(x[x[:, 0] == u, 1].tolist()) for x in (tr, va, te))
        n = int((inter[:, 0] == u).sum())
        assert not (a & b or a & c or b & c) and len(c) == math.ceil(0.2 * n)  # sklearn's sizes
    assert drv.early_stopping([0.1, 0.2] + [0.1] * 9) == (0.2, False)
    assert drv.early_stopping([0.1, 0.2] + [0.1] * 10) == (0.2, True)


def test_step_loss_plain_backward_takes_the_direct_path():
    """model._StepLoss: a plain ``loss.backward()`` calls the node's ``fast_backward`` (no autograd engine);
    a scaled loss, ``retain_graph`` or a leaf with gradient hooks goes through the engine and the node's
    ordinary backward; either way a second backward of the same loss raises."""
    model = __import__(load_pkg().__name__ + ".model", fromlist=["model"])
    calls = []

    def fast(ctx):
        if any(getattr(p, "_post_accumulate_grad_hooks", None) for p in ctx.leaves):
            ctx.fast_backward = fast
            raise model._UseEngine
        calls.append("fast")
        ctx.done = True
        ctx.leaves[0].grad = torch.full((3,), 2.0)

    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            ctx.leaves, ctx.done, ctx.fast_backward = (x,), False, fast
            return (2 * x).sum().as_subclass(model._StepLoss)

        @staticmethod
        def backward(ctx, g):
            ctx.fast_backward = None
            if ctx.done:
                raise RuntimeError("Trying to backward through the graph a second time")
            ctx.done = True
            calls.append("engine")
            return g * 2 * torch.ones(3)

    x = torch.ones(3, requires_grad=True)
    loss = F.apply(x)
    assert isinstance(loss, model._StepLoss) and float(loss) == 6.0
    assert type(loss + 1) is torch.Tensor  # every other operation sees a plain tensor
    loss.backward()
    assert calls == ["fast"] and torch.equal(x.grad, torch.full((3,), 2.0))
    with pytest.raises(RuntimeError):
        loss.backward()
    x.grad = None
    (F.apply(x) * 0.5).backward()  # scaled: the engine
    assert calls[-1] == "engine" and torch.equal(x.grad, torch.ones(3))
    x.grad = None
    F.apply(x).backward(retain_graph=True)
    assert calls[-1] == "engine"
    x.grad = None
    h = x.register_post_accumulate_grad_hook(lambda p: calls.append("hook"))
    F.apply(x).backward()  # a leaf with hooks: the engine (the hook runs)
    assert calls[-2:] == ["engine", "hook"]
    h.remove()
    x.grad = None
    loss = F.apply(x)
    loss.register_hook(lambda g: calls.append("loss hook"))
    loss.backward()  # a hook on the loss itself: the engine (the hook runs)
    assert calls[-2:] == ["loss hook", "engine"]
    x.grad = None

    def grad_mode(ctx):  # the direct call runs under no_grad, as the engine's backward does
        calls.append(f"grad enabled {torch.is_grad_enabled()}")
    F2 = type("F2", (F,), {})
    F2.forward = staticmethod(lambda ctx, x: (setattr(ctx, "fast_backward", grad_mode), (2 * x).sum())[1]
                              .as_subclass(model._StepLoss))
    F2.apply(x).backward()
    assert calls[-1] == "grad enabled False"
