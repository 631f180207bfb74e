"""GPU parity: the HIP path (through the C-ABI) vs the CPU oracle and the
reference-generated golden vectors.  Needs an MI355X: ``pytest -m gpu``.

Tolerance (north_star): embeddings / losses within 1e-4 fp32 (rtol 1e-4,
atol 1e-5 on O(1) values, atol 1e-6 on gradients of size ~1e-3).
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np
import pytest
import torch

from oracle import kgat_cpu as K
from tests.conftest import KGAT_CASES, ROOT, golden, load_pkg

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-4, 1e-5
DEV = "cuda"
# Parameters after an Adam step: Adam normalises each element by sqrt(v) + eps
# (eps = 1e-8), so an element whose gradient is ~1e-9 (rows many hops from the
# batch) moves by ~lr * g / (|g| + eps) and a 1e-10 fp32-summation-order
# difference in g moves it by ~1e-5.  Gradients are compared at RTOL/1e-6
# above; params after the step get an absolute slack of 2 % of one lr=1e-3 step.
ADAM_ATOL = 2e-5


@pytest.fixture(scope="module")
def pkg():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_pkg()


def _mods(pkg):
    graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])
    kernels = __import__(pkg.__name__ + ".kernels", fromlist=["kernels"])
    return graph, kernels


def random_graph(graph_mod, n, avg_deg, hubs=0, hub_deg=0, seed=0, mids=0, mid_deg=0):
    rng = np.random.default_rng(seed)
    e = n * avg_deg
    rows = rng.integers(0, n, e)
    cols = rng.integers(0, n, e)
    for k, deg in ((hubs, hub_deg), (mids, mid_deg)):
        if k:
            hr = rng.integers(0, n, k)
            rows = np.concatenate([rows, np.repeat(hr, deg)])
            cols = np.concatenate([cols, rng.integers(0, n, k * deg)])
    vals = rng.standard_normal(rows.size).astype(np.float32)
    rowptr, col, val = graph_mod.csr_from_coo(n, rows, cols, vals)
    lay = graph_mod.GraphLayout(n_nodes=n, rel_order=[], heads=np.zeros(0, np.int64), rels=np.zeros(0, np.int64),
                                tails=np.zeros(0, np.int64), edge_vals=np.zeros(0, np.float32), rowptr=rowptr,
                                col=col, val=val, slot=np.zeros(0, np.int64))
    r = np.repeat(np.arange(n), np.diff(rowptr))
    A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([r, col.astype(np.int64)])), torch.from_numpy(val),
                                (n, n)).coalesce()
    return lay, A


@pytest.mark.parametrize("d", [16, 32, 64, 128, 256])
def test_spmm_parity(pkg, d):
    graph_mod, kernels = _mods(pkg)
    lay, A = random_graph(graph_mod, 3000, 9, hubs=5, hub_deg=2000, seed=d)
    g = graph_mod.DeviceGraph(lay, DEV)
    assert g.A.n_long >= 5 and g.AT.n_long >= 0
    X = torch.randn(3000, d)
    Y = kernels.spmm(g, X.to(DEV)).cpu()
    np.testing.assert_allclose(Y.numpy(), torch.sparse.mm(A, X).numpy(), rtol=RTOL, atol=1e-4)
    # transpose + accumulate
    Z0 = torch.randn(3000, d)
    Z = Z0.to(DEV)
    kernels.spmm(g, X.to(DEV), out=Z, transpose=True, accumulate=True)
    ref = torch.sparse.mm(A.t().coalesce(), X) + Z0
    np.testing.assert_allclose(Z.cpu().numpy(), ref.numpy(), rtol=RTOL, atol=1e-4)
    # strided (ld > d) input/output views
    big = torch.randn(3000, d + 32)
    out = torch.zeros(3000, d + 16, device=DEV)
    kernels.spmm(g, big.to(DEV)[:, 16:16 + d], out=out[:, :d])
    np.testing.assert_allclose(out[:, :d].cpu().numpy(), torch.sparse.mm(A, big[:, 16:16 + d]).numpy(),
                               rtol=RTOL, atol=1e-4)


def test_spmm_symmetric_hubs_transpose_accumulate(pkg):
    """CKG-like pattern (every edge has its inverse) with hub rows: A^T has long rows too,
    exercising the segment + fix-up path with accumulate (the backward's use)."""
    graph_mod, kernels = _mods(pkg)
    rng = np.random.default_rng(11)
    n = 4000
    h = np.concatenate([rng.integers(0, n, 30000), np.repeat(rng.integers(0, n, 4), 1500)])
    t = rng.integers(0, n, h.size)
    rows, cols = np.concatenate([h, t]), np.concatenate([t, h])
    vals = rng.random(rows.size).astype(np.float32)
    rowptr, col, val = graph_mod.csr_from_coo(n, rows, cols, vals)
    lay = graph_mod.GraphLayout(n_nodes=n, rel_order=[], heads=np.zeros(0, np.int64), rels=np.zeros(0, np.int64),
                                tails=np.zeros(0, np.int64), edge_vals=np.zeros(0, np.float32), rowptr=rowptr,
                                col=col, val=val, slot=np.zeros(0, np.int64))
    g = graph_mod.DeviceGraph(lay, DEV)
    assert g.A.n_long >= 4 and g.AT.n_long >= 4
    r = np.repeat(np.arange(n), np.diff(rowptr))
    A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([r, col.astype(np.int64)])), torch.from_numpy(val),
                                (n, n)).coalesce()
    for d in (32, 64):
        X, Z0 = torch.randn(n, d), torch.randn(n, d)
        Z = Z0.to(DEV)
        kernels.spmm(g, X.to(DEV), out=Z, transpose=True, accumulate=True)
        ref = torch.sparse.mm(A.t().coalesce(), X) + Z0
        np.testing.assert_allclose(Z.cpu().numpy(), ref.numpy(), rtol=RTOL, atol=1e-4)


def test_spmm_empty_rows_and_deterministic(pkg):
    graph_mod, kernels = _mods(pkg)
    lay, A = random_graph(graph_mod, 1000, 1, hubs=2, hub_deg=3000, seed=7)
    g = graph_mod.DeviceGraph(lay, DEV)
    X = torch.randn(1000, 64, device=DEV)
    a = kernels.spmm(g, X)
    b = kernels.spmm(g, X)
    assert torch.equal(a, b)
    np.testing.assert_allclose(a.cpu().numpy(), torch.sparse.mm(A, X.cpu()).numpy(), rtol=RTOL, atol=1e-4)


def test_spmm_segment_plans_and_launch_order(pkg):
    """A's hub rows under the column-cut plan (kgat_csr_plan_cols) and the XCD-grouped launch order
    (kgat_csr::seg_order): the order is scheduling only -- identity, the built order and a reversed one give
    the same bits; the column-cut and the fixed-length plans both match the sparse product."""
    from types import SimpleNamespace

    graph_mod, kernels = _mods(pkg)
    n = 80000  # > 8 column blocks of 8192: the column cuts and the launch order apply
    lay, A = random_graph(graph_mod, n, 6, hubs=12, hub_deg=6000, seed=5, mids=40, mid_deg=400)
    g = graph_mod.DeviceGraph(lay, DEV)
    fixed = graph_mod.long_row_plan(lay.rowptr)
    assert g.A.col_cuts and g.A.seg_order is not None and g.A.n_seg > fixed[2].size  # column cuts happened
    X = torch.randn(n, 64, device=DEV)
    Y = kernels.spmm(g, X)
    order = g.A.seg_order
    try:
        g.A.seg_order = None
        Y_id = kernels.spmm(g, X)
        g.A.seg_order = torch.flip(order, [0]).contiguous()
        Y_rev = kernels.spmm(g, X)
    finally:
        g.A.seg_order = order
    assert torch.equal(Y, Y_id) and torch.equal(Y, Y_rev)
    small = graph_mod.DeviceGraph(random_graph(graph_mod, 3000, 9, hubs=5, hub_deg=2000, seed=1)[0], DEV)
    assert not small.A.col_cuts and small.A.seg_order is None  # a table within 8 column blocks: fixed plan
    ref = torch.sparse.mm(A, X.cpu()).numpy()
    atol = 1e-3  # 6,000-term hub sums of magnitude ~100: fp32 summation-order differences reach ~1.5e-4
    np.testing.assert_allclose(Y.cpu().numpy(), ref, rtol=RTOL, atol=atol)
    csr_fixed = graph_mod._DeviceCSR(lay.rowptr, lay.col, g.A.val, DEV, col_cuts=False)
    assert csr_fixed.n_seg == fixed[2].size
    Y_fixed = kernels.spmm(SimpleNamespace(A=csr_fixed, AT=g.AT, n_nodes=n), X)
    np.testing.assert_allclose(Y_fixed.cpu().numpy(), ref, rtol=RTOL, atol=atol)


BI_SHAPES = [(64, 64), (64, 32), (32, 16), (128, 64), (64, 16), (128, 128), (16, 16)]


@pytest.mark.parametrize("din,dout", BI_SHAPES)
def test_biinter_fwd_bwd_parity(pkg, din, dout):
    _, kernels = _mods(pkg)
    torch.manual_seed(din * 7 + dout)
    n = 1000 + 13  # ragged tail sub-tile
    X, S = torch.randn(n, din), torch.randn(n, din)
    W1, W2 = torch.randn(dout, din) * 0.2, torch.randn(dout, din) * 0.2
    b1, b2 = torch.randn(dout) * 0.1, torch.randn(dout) * 0.1
    dH = torch.randn(n, dout)
    leaves = [t.clone().requires_grad_(True) for t in (X, S, W1, b1, W2, b2)]
    x, s, w1, bb1, w2, bb2 = leaves
    pre1 = torch.nn.functional.linear(x + s, w1, bb1)
    pre2 = torch.nn.functional.linear(x * s, w2, bb2)
    h = torch.nn.functional.leaky_relu(pre1, 0.01) + torch.nn.functional.leaky_relu(pre2, 0.01)
    ref = h / h.norm(dim=1, keepdim=True).clamp_min(1e-12)
    ref.backward(dH)
    dv = [t.to(DEV) for t in (X, S, W1, b1, W2, b2)]
    H = kernels.biinter_fwd(*dv)
    np.testing.assert_allclose(H.cpu().numpy(), ref.detach().numpy(), rtol=RTOL, atol=ATOL)
    dXd, dS, dW1, db1, dW2, db2 = kernels.biinter_bwd(dv[0], dv[1], dH.to(DEV), *dv[2:])
    # dX (direct) + dS: the autograd X/S grads see x+s and x*s
    np.testing.assert_allclose(dXd.cpu().numpy(), x.grad.numpy(), rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(dS.cpu().numpy(), s.grad.numpy(), rtol=1e-3, atol=1e-5)
    for got, want in ((dW1, w1.grad), (db1, bb1.grad), (dW2, w2.grad), (db2, bb2.grad)):
        np.testing.assert_allclose(got.cpu().numpy(), want.numpy(), rtol=1e-3, atol=1e-4)
    if kernels.saved_state_supported(din, dout):
        st = kernels.BiState(n, DEV, din, dout)
        H2 = kernels.biinter_fwd(*dv, state=st)
        assert torch.equal(H, H2)
        got = kernels.biinter_bwd(dv[0], dv[1], dH.to(DEV), *dv[2:], H=H2, state=st)
        want = (x.grad, s.grad, w1.grad, bb1.grad, w2.grad, bb2.grad)
        for i, (a, b) in enumerate(zip(got, want)):
            np.testing.assert_allclose(a.cpu().numpy(), b.numpy(), rtol=1e-3, atol=1e-5 if i < 2 else 1e-4)


@pytest.mark.parametrize("din,dout", [(64, 64), (64, 32), (32, 16), (16, 16), (128, 32)])
def test_biinter_saved_state_matches_recompute(pkg, din, dout):
    """The backward from the forward's saved state (norm + sign/keep bits) equals the
    recomputing backward: dense and frontier rows, dropout on/off, clamped (all-zero) rows."""
    _, kernels = _mods(pkg)
    torch.manual_seed(din + dout)
    n = 3000 + 7
    X, S = torch.randn(n, din), torch.randn(n, din)
    X[100:140] = 0.0  # with b = 0 these rows give g = 0: F.normalize's clamp is active
    S[100:140] = 0.0
    W1, W2 = torch.randn(dout, din) * 0.2, torch.randn(dout, din) * 0.2
    b1, b2 = torch.zeros(dout), torch.zeros(dout)
    dv = [t.to(DEV) for t in (X, S, W1, b1, W2, b2)]
    dH = torch.randn(n, dout).to(DEV)
    F = torch.from_numpy(np.random.default_rng(2).choice(n, 300, replace=False))
    F[:5] = torch.arange(100, 105)
    rows = torch.cat([F, torch.full((20,), -1)]).int().to(DEV)
    dHc = torch.zeros(320, dout, device=DEV)
    dHc[:300] = torch.randn(300, dout, device=DEV)
    for p in (0.0, 0.2):
        st = kernels.BiState(n, DEV, din, dout)
        H = kernels.biinter_fwd(*dv, dropout_p=p, seed=5, state=st)
        assert torch.equal(H, kernels.biinter_fwd(*dv, dropout_p=p, seed=5))
        norm = st.norm[:n].cpu()
        assert torch.all(norm[100:140] < 0) and torch.all(norm[:100] > 0)
        for rr, g in ((None, dH), (rows, dHc)):
            a = kernels.biinter_bwd(dv[0], dv[1], g, *dv[2:], dropout_p=p, seed=5, rows=rr)
            b = kernels.biinter_bwd(dv[0], dv[1], g, *dv[2:], dropout_p=p, seed=5, rows=rr, H=H, state=st)
            for i, (x, y) in enumerate(zip(a, b)):
                np.testing.assert_allclose(y.cpu().numpy(), x.cpu().numpy(), rtol=1e-4,
                                           atol=1e-6 if i < 2 else 1e-5, err_msg=f"p={p} rows={rr is not None} {i}")


def test_biinter_dropout_consistent(pkg):
    """fwd/bwd regenerate the same keep mask; masked elements are exactly zero."""
    _, kernels = _mods(pkg)
    torch.manual_seed(3)
    n, din, dout, p = 4096, 64, 64, 0.1
    X, S = torch.randn(n, din), torch.randn(n, din)
    W1, W2 = torch.randn(dout, din) * 0.2, torch.randn(dout, din) * 0.2
    b1, b2 = torch.randn(dout) * 0.1, torch.randn(dout) * 0.1
    dv = [t.to(DEV) for t in (X, S, W1, b1, W2, b2)]
    H = kernels.biinter_fwd(*dv, dropout_p=p, seed=1234).cpu()
    H2 = kernels.biinter_fwd(*dv, dropout_p=p, seed=1234).cpu()
    assert torch.equal(H, H2)
    keep = (H != 0).float()
    frac = 1 - keep.mean().item()
    assert abs(frac - p) < 0.01, frac
    leaves = [t.clone().requires_grad_(True) for t in (X, S, W1, b1, W2, b2)]
    x, s, w1, bb1, w2, bb2 = leaves
    h = (torch.nn.functional.leaky_relu(torch.nn.functional.linear(x + s, w1, bb1), 0.01)
         + torch.nn.functional.leaky_relu(torch.nn.functional.linear(x * s, w2, bb2), 0.01))
    h = h * keep / (1 - p)
    ref = h / h.norm(dim=1, keepdim=True).clamp_min(1e-12)
    np.testing.assert_allclose(H.numpy(), ref.detach().numpy(), rtol=RTOL, atol=ATOL)
    dH = torch.randn(n, dout)
    ref.backward(dH)
    dXd, dS, dW1, db1, dW2, db2 = kernels.biinter_bwd(dv[0], dv[1], dH.to(DEV), *dv[2:], dropout_p=p, seed=1234)
    np.testing.assert_allclose(dXd.cpu().numpy(), x.grad.numpy(), rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(dW1.cpu().numpy(), w1.grad.numpy(), rtol=1e-3, atol=1e-4)


def test_adam_parity(pkg):
    _, kernels = _mods(pkg)
    torch.manual_seed(0)
    p = torch.randn(10007)
    opt = K.AdamOracle(lr=1e-3)
    P = {"p": p.clone()}
    pd, m, v = p.to(DEV), torch.zeros(10007, device=DEV), torch.zeros(10007, device=DEV)
    import math
    for t in range(1, 4):
        g = torch.randn(10007)
        opt.step(P, {"p": g})
        kernels.adam(pd, g.to(DEV), m, v, 1e-3 / (1 - 0.9 ** t), 0.9, 0.999, math.sqrt(1 - 0.999 ** t), 1e-8)
    np.testing.assert_allclose(pd.cpu().numpy(), P["p"].numpy(), rtol=1e-6, atol=1e-7)


def _model_from_golden(pkg, g):
    U, E = int(g["user_num"]), int(g["entity_num"])
    n = U + E
    layers = g["layers"].tolist()
    A = torch.sparse_coo_tensor(torch.from_numpy(g["A_idx"]), torch.from_numpy(g["A_val"]), (n, n))
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(g["adjacency_relations"]),
                              cf_embedding_dim=int(g["dim"]), kg_embedding_dim=int(g["dim"]), attentive_matrix=A,
                              layer_size=layers, message_dropout=[0.1] * len(layers)))
    sd = m.state_dict()
    for k in sd:
        if not sd[k].is_sparse:
            sd[k] = torch.from_numpy(g["init/" + k])
    m.load_state_dict(sd)
    m.to(DEV)
    m.eval()
    return m


@pytest.mark.parametrize("case", KGAT_CASES)
def test_propagation_vs_reference(pkg, case):
    g = golden("kgat_" + case)
    m = _model_from_golden(pkg, g)
    all_emb = m._build_cf_embeddings().cpu().numpy()
    np.testing.assert_allclose(all_emb, g["all_emb"], rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("case", KGAT_CASES)
def test_cf_train_steps_vs_reference(pkg, case):
    """Loss, every gradient and the params after each Adam step match the reference run."""
    g = golden("kgat_" + case)
    m = _model_from_golden(pkg, g)
    m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    named = dict(m.named_parameters())
    s = 0
    while f"cf{s}/loss" in g:
        ids = [torch.from_numpy(g[f"cf{s}/{x}"]).to(DEV) for x in ("users", "pos", "neg")]
        loss = m(*ids, mode=pkg.KGATMode.TRAIN_CF)
        loss.backward()
        np.testing.assert_allclose(loss.item(), g[f"cf{s}/loss"], rtol=1e-5)
        for k, prm in named.items():
            ref = g.get(f"cf{s}/grad/{k}")
            if ref is None:
                assert prm.grad is None, k
            else:
                np.testing.assert_allclose(prm.grad.cpu().numpy(), ref, rtol=RTOL, atol=1e-6, err_msg=k)
        m.update_cf_weights()
        s += 1
    for k, v in g.items():
        if k.startswith("after_cf/"):
            np.testing.assert_allclose(named[k[9:]].detach().cpu().numpy(), v, rtol=RTOL, atol=ADAM_ATOL,
                                       err_msg=k)


def test_cf_step_dropout_train_mode_runs(pkg):
    """Train mode (dropout active, as main.py:292 runs it): finite loss, grads, deterministic per seed."""
    g = golden("kgat_L3_d64")
    m = _model_from_golden(pkg, g)
    m.train()
    m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    ids = [torch.from_numpy(g[f"cf0/{x}"]).to(DEV) for x in ("users", "pos", "neg")]
    torch.manual_seed(5)
    loss = m(*ids, mode=pkg.KGATMode.TRAIN_CF)
    loss.backward()
    assert torch.isfinite(loss).item()
    assert torch.isfinite(m._user_entity_embedding.weight.grad).all().item()
    m.update_cf_weights()


@pytest.mark.parametrize("dim,layers,batch", [(64, [64, 32], 256), (64, [64, 32, 16], 512), (256, [256, 128], 256),
                                              (128, [128, 64, 32], 256), (256, [256, 128, 64], 256)])
def test_cf_step_synthetic_hubs_vs_oracle(pkg, dim, layers, batch):
    """Synthetic CKG with Zipf hub rows (long-row path in A and A^T), duplicate ids in the
    batch (users repeat, items collide with user rows): loss and every gradient vs the oracle."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(6000, 60000, seed=11)
    lay = graph_mod.build_layout(U, E, inter, trip)
    torch.manual_seed(2024)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=layers,
                              cf_embedding_dim=dim, kg_embedding_dim=dim))
    init = {k: v.clone() for k, v in m.state_dict().items() if not v.is_sparse}
    g = m.attach_graph(lay, DEV)
    assert g.A.n_long > 0 and g.AT.n_long > 0
    m.eval()
    rng = np.random.default_rng(0)
    ids = [torch.from_numpy(rng.integers(0, hi, batch)) for hi in (U, int(E * 0.1), int(E * 0.1))]
    loss = m(*[t.to(DEV) for t in ids], mode=pkg.KGATMode.TRAIN_CF)
    loss.backward()
    rows, cols, vals = lay.coo()
    A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, cols])), torch.from_numpy(vals),
                                (U + E, U + E)).coalesce()
    P = {k: v.clone().requires_grad_(True) for k, v in init.items()}
    ref = K.cf_loss(torch.cat(K.propagate(P, A), 1), *ids)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-5)
    for k, prm in m.named_parameters():
        if prm.grad is None:
            assert P[k].grad is None if k in P else True, k
            continue
        np.testing.assert_allclose(prm.grad.cpu().numpy(), P[k].grad.numpy(), rtol=RTOL, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("dim,layers", [(64, [64, 32]), (128, [128, 64, 32]), (256, [256, 128, 64])])
def test_cf_step_large_hub_graph_vs_oracle(pkg, dim, layers):
    """bench-like scale -- 2M nodes, 3M edges, a hub row of ~114k edges (hundreds of
    long-row segments + the ordered fix-up, in A and A^T) -- eval-mode propagation of every layer,
    the CF loss and every gradient vs the oracle; the batch holds the hub item."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(2_000_000, 1_500_000, seed=2024)
    lay = graph_mod.build_layout(U, E, inter, trip)
    deg = np.diff(lay.rowptr)
    assert lay.nnz >= 2_000_000 and deg.max() > 100_000
    torch.manual_seed(2024)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=layers,
                              cf_embedding_dim=dim, kg_embedding_dim=dim))
    init = {k: v.clone() for k, v in m.state_dict().items() if not v.is_sparse and
            (k.startswith("_aggregator") or k == "_user_entity_embedding.weight")}
    m.attach_graph(lay, DEV)
    m.eval()
    rng = np.random.default_rng(3)
    hub_item = int(np.argmax(deg)) - U  # the hub row is an item node (U + item)
    assert 0 <= hub_item < int(E * 0.1)
    ids = [torch.from_numpy(rng.integers(0, hi, 256)) for hi in (U, int(E * 0.1), int(E * 0.1))]
    ids[1][:8] = hub_item
    tabs = [t.cpu() for t in m.propagate()]
    loss = m(*[t.to(DEV) for t in ids], mode=pkg.KGATMode.TRAIN_CF)
    loss.backward()
    rows, cols, vals = lay.coo()
    A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, cols])), torch.from_numpy(vals),
                                (U + E, U + E)).coalesce()
    P = {k: v.clone().requires_grad_(True) for k, v in init.items()}
    outs = K.propagate(P, A)
    # north_star's embedding tolerance (1e-4 fp32): a 114k-term row summed in another order (512-edge
    # segments + ordered fix-up vs the CPU's sequential sum) moves a few normalised entries by ~3e-5
    for l, (a, w) in enumerate(zip(tabs, outs)):
        np.testing.assert_allclose(a.numpy(), w.detach().numpy(), rtol=RTOL, atol=1e-4, err_msg=f"layer {l}")
    ref = K.cf_loss(torch.cat(outs, 1), *ids)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-5)
    for k in P:
        prm = dict(m.named_parameters())[k]
        np.testing.assert_allclose(prm.grad.cpu().numpy(), P[k].grad.numpy(), rtol=RTOL, atol=1e-6, err_msg=k)


def test_frontier_build_and_reset(pkg):
    _, kernels = _mods(pkg)
    rng = np.random.default_rng(5)
    n, B = 500, 256
    u, p, q = (torch.from_numpy(rng.integers(0, 60, B)) for _ in range(3))
    node_map = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    rows, count = kernels.frontier_build(u.to(DEV), p.to(DEV), q.to(DEV), node_map)
    ids = torch.cat([u, p, q]).numpy()
    _, first = np.unique(ids, return_index=True)
    want = ids[np.sort(first)]
    got = rows.cpu().numpy()
    assert int(count.item()) == want.size
    np.testing.assert_array_equal(got[:want.size], want)
    assert np.all(got[want.size:] == -1)
    nm = node_map.cpu().numpy()
    np.testing.assert_array_equal(nm[want], np.arange(want.size))
    kernels.frontier_reset(rows, node_map)
    assert int((node_map != -1).sum().item()) == 0


@pytest.mark.parametrize("d", [32, 64])
def test_spmm_masked_matches_dense(pkg, d):
    graph_mod, kernels = _mods(pkg)
    rng = np.random.default_rng(d)
    n = 4000
    h = np.concatenate([rng.integers(0, n, 30000), np.repeat(rng.integers(0, n, 4), 1500)])
    t = rng.integers(0, n, h.size)
    rowptr, col, val = graph_mod.csr_from_coo(n, np.concatenate([h, t]), np.concatenate([t, h]),
                                              rng.random(2 * h.size).astype(np.float32))
    lay = graph_mod.GraphLayout(n_nodes=n, rel_order=[], heads=np.zeros(0, np.int64), rels=np.zeros(0, np.int64),
                                tails=np.zeros(0, np.int64), edge_vals=np.zeros(0, np.float32), rowptr=rowptr,
                                col=col, val=val, slot=np.zeros(0, np.int64))
    g = graph_mod.DeviceGraph(lay, DEV)
    F = rng.choice(n, 300, replace=False)
    Xc, Yc = torch.randn(310, d), torch.randn(310, d)
    node_map = np.full(n, -1, np.int32)
    node_map[F] = np.arange(300)
    X = torch.zeros(n, d)
    X[F] = Xc[:300]
    Y0 = torch.zeros(n, d)
    Y0[F] = Yc[:300]
    for tr in (False, True):
        out = kernels.spmm_masked(g, torch.from_numpy(node_map).to(DEV), Xc.to(DEV), Yc.to(DEV), transpose=tr)
        ref = kernels.spmm(g, X.to(DEV), transpose=tr).cpu() + Y0
        np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-6)


def test_spmm_masked_row_hit_hop_compact_and_row_blocks(pkg):
    """The hop chain's pieces: row_hit flags exactly the rows that gathered a frontier edge or
    carry a Yc row (long hub rows included), kgat_hop_compact lists them ascending with their
    map, and row-block views with yc_row0 reproduce the whole masked product bit for bit."""
    graph_mod, kernels = _mods(pkg)
    rng = np.random.default_rng(3)
    n, d = 5000, 64
    h = np.concatenate([rng.integers(0, n, 20000), np.repeat(rng.integers(0, n, 5), 1200)])
    t = rng.integers(0, n, h.size)
    rowptr, col, val = graph_mod.csr_from_coo(n, np.concatenate([h, t]), np.concatenate([t, h]),
                                              rng.random(2 * h.size).astype(np.float32))
    lay = graph_mod.GraphLayout(n_nodes=n, rel_order=[], heads=np.zeros(0, np.int64), rels=np.zeros(0, np.int64),
                                tails=np.zeros(0, np.int64), edge_vals=np.zeros(0, np.float32), rowptr=rowptr,
                                col=col, val=val, slot=np.zeros(0, np.int64))
    g = graph_mod.DeviceGraph(lay, DEV)
    assert g.AT.n_long > 0
    F = rng.choice(n, 120, replace=False)
    node_map = np.full(n, -1, np.int32)
    node_map[F] = np.arange(F.size)
    Xc, Yc = torch.randn(F.size, d, device=DEV), torch.randn(F.size, d, device=DEV)
    hit = g.hop_buffers()[0]
    hit.fill_(7)  # stale flags must be cleared by the call
    nm = torch.from_numpy(node_map).to(DEV)
    out = kernels.spmm_masked(g, nm, Xc, Yc_init=Yc, transpose=True, row_hit=hit)
    # expected flags: rows r of A^T with an edge into F, or r in F
    rt = g.AT.rowptr_host
    colt = g.AT.col.cpu().numpy()
    inF = np.zeros(n, bool)
    inF[F] = True
    want = np.zeros(n, bool)
    want[np.repeat(np.arange(n), np.diff(rt))[inF[colt]]] = True
    want |= inF
    np.testing.assert_array_equal(hit.cpu().numpy().astype(bool), want)
    hrows, hmap, _, cnt = kernels.hop_compact(g, sync=True)
    assert cnt == int(want.sum())
    np.testing.assert_array_equal(hrows.cpu().numpy(), np.nonzero(want)[0])
    m = hmap.cpu().numpy()
    np.testing.assert_array_equal(m[want], np.arange(cnt))
    assert np.all(m[~want] == -1)
    # rows outside the hop set are exactly zero
    assert float(out[torch.from_numpy(~want).to(DEV)].abs().max()) == 0.0
    # the bitmap membership test gives the same bits (and flags)
    bits = kernels.map_bits(nm, torch.empty(2 * ((n + 63) // 64), dtype=torch.int32, device=DEV))
    bw = np.unpackbits(bits.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    np.testing.assert_array_equal(bw, inF)
    hit2 = torch.zeros_like(hit)
    out2 = kernels.spmm_masked(g, nm, Xc, Yc_init=Yc, transpose=True, row_hit=hit2, src_bits=bits)
    assert torch.equal(out2, out)
    np.testing.assert_array_equal(hit2.cpu().numpy().astype(bool), want)
    # an ascending-order source set (the hop set): rank words (membership + compact row in one
    # load) give the same bits as the map lookup
    Hc = torch.randn(cnt, d, device=DEV)
    rank = kernels.map_rank(hmap, torch.empty((n + 31) // 32, dtype=torch.int64, device=DEV))
    by_map = kernels.spmm_masked(g, hmap, Hc, transpose=True)
    by_rank = kernels.spmm_masked(g, hmap, Hc, transpose=True, src_rank=rank)
    assert torch.equal(by_map, by_rank)
    # row-block views (yc_row0) give the same bits
    bounds = [(0, 1700), (1700, 3333), (3333, n)]
    blk = torch.empty_like(out)
    for v in g.transpose_row_blocks(bounds):
        kernels.spmm_block_masked(v, nm, Xc, blk[v.r0:v.r0 + v.n_rows], Yc_init=Yc, row0=v.r0)
    assert torch.equal(blk, out)


def test_frontier_hop_and_masked_rows_product(pkg):
    """kgat_frontier_hop marks the batch frontier and its A-neighbours (= the rows the masked A^T
    product over the frontier flags), and kgat_spmm_csr_masked_rows_f32 produces exactly those rows
    of that product, compactly and with the same bits (hub rows included)."""
    graph_mod, kernels = _mods(pkg)
    rng = np.random.default_rng(8)
    n, d = 6000, 64
    h = np.concatenate([rng.integers(0, n, 24000), np.repeat(rng.integers(0, n, 5), 1500)])
    t = rng.integers(0, n, h.size)
    rowptr, col, val = graph_mod.csr_from_coo(n, np.concatenate([h, t]), np.concatenate([t, h]),
                                              rng.random(2 * h.size).astype(np.float32))
    lay = graph_mod.GraphLayout(n_nodes=n, rel_order=[], heads=np.zeros(0, np.int64), rels=np.zeros(0, np.int64),
                                tails=np.zeros(0, np.int64), edge_vals=np.zeros(0, np.float32), rowptr=rowptr,
                                col=col, val=val, slot=np.zeros(0, np.int64))
    g = graph_mod.DeviceGraph(lay, DEV)
    B = 64
    users = torch.from_numpy(rng.integers(0, n, B)).to(DEV)
    pos = torch.from_numpy(np.concatenate([rng.integers(0, n, B - 1), [int(np.argmax(np.diff(rowptr)))]])).to(DEV)
    neg = torch.from_numpy(rng.integers(0, n, B)).to(DEV)
    rows0, cnt0 = kernels.frontier_build(users, pos, neg, g.node_map)
    n0 = int(cnt0.item())
    Xc = torch.randn(3 * B, d, device=DEV)
    Yc = torch.randn(3 * B, d, device=DEV)
    hit = g.hop_buffers()[0]
    fb = torch.zeros_like(g.hop_buffers()[6])
    kernels.map_bits(g.node_map, fb)
    dense = kernels.spmm_masked(g, g.node_map, Xc, Yc_init=Yc, transpose=True, row_hit=hit, src_bits=fb)
    want = hit.cpu().numpy().astype(bool)
    hrows, hmap, hcount, hbits, fbits = kernels.frontier_hop(g, rows0)
    cnt = int(hcount.item())
    assert cnt == int(want.sum())
    np.testing.assert_array_equal(hrows[:cnt].cpu().numpy(), np.nonzero(want)[0])
    m = hmap.cpu().numpy()
    np.testing.assert_array_equal(m[want], np.arange(cnt))
    assert np.all(m[~want] == -1)
    assert torch.equal(fbits[:fb.numel()], fb)
    # the hop set's rank words written alongside (kgat_map_rank's layout; the count half of a word
    # without members is unused, so only member words are compared there)
    words = (n + 31) // 32
    got = g.hop_buffers()[9][:words].cpu().numpy().view(np.uint64)
    ref = kernels.map_rank(hmap, torch.empty(words, dtype=torch.int64, device=DEV)).cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got & 0xFFFFFFFF, ref & 0xFFFFFFFF)
    mem = (ref & 0xFFFFFFFF) != 0
    np.testing.assert_array_equal(got[mem] >> 32, ref[mem] >> 32)
    comp = kernels.spmm_masked_rows(g, g.node_map, fbits, Xc, Yc, hrows, hmap, hcount, hbits)
    assert torch.equal(comp[:cnt], dense[hrows[:cnt].long()])
    kernels.frontier_reset(rows0, g.node_map)
    assert n0 > 0


@pytest.mark.parametrize("layers", [[64, 32], [64, 32, 16]])
def test_cf_hop_chain_matches_dense_backward(pkg, layers):
    """The hop-chain backward (lower layers on their hop sets) against the dense backward of the
    same model and batch: the table gradient bit for bit (same per-row arithmetic and order),
    the aggregator weight gradients within fp32 summation-order tolerance."""
    graph_mod, _ = _mods(pkg)
    model_mod = __import__(pkg.__name__ + ".model", fromlist=["model"])
    U, E, inter, trip = graph_mod.synthetic_ckg(20000, 200000, seed=5)
    lay = graph_mod.build_layout(U, E, inter, trip)
    torch.manual_seed(2024)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=layers,
                              message_dropout=[0.1] * len(layers)))
    m.attach_graph(lay, DEV)
    m.train()
    rng = np.random.default_rng(4)
    ids = [torch.from_numpy(rng.integers(0, hi, 64)).to(DEV) for hi in (U, int(E * 0.1), int(E * 0.1))]
    grads = {}
    old = model_mod.HOP_DENSE_FRACTION
    try:
        for frac in (1.0, 0.0):
            model_mod.HOP_DENSE_FRACTION = frac
            for p in m.parameters():
                p.grad = None
            torch.manual_seed(123)  # same dropout seeds for both runs
            m(*ids, mode=pkg.KGATMode.TRAIN_CF).backward()
            grads[frac] = {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}
    finally:
        model_mod.HOP_DENSE_FRACTION = old
    sp, de = grads[1.0], grads[0.0]
    assert sp.keys() == de.keys()
    assert torch.equal(sp["_user_entity_embedding.weight"], de["_user_entity_embedding.weight"])
    for k in sp:
        np.testing.assert_allclose(sp[k].cpu().numpy(), de[k].cpu().numpy(), rtol=1e-5, atol=1e-7, err_msg=k)


@pytest.mark.parametrize("din,dout", [(64, 64), (64, 32), (32, 16)])
def test_biinter_fwd_row_blocks_bit_identical(pkg, din, dout):
    """kgat_biinter_fwd_rows_f32 (kernels.biinter_fwd_rows) on row blocks of the table -- 16-aligned
    starts, a ragged last block, dropout drawn by global node id -- gives the whole-table launch's H and
    saved state (norms, sign/keep words) bit for bit."""
    graph_mod, kernels = _mods(pkg)
    lay, _ = random_graph(graph_mod, 5003, 10, hubs=5, hub_deg=1500, seed=din)
    g = graph_mod.DeviceGraph(lay, DEV)
    torch.manual_seed(din + dout)
    n = lay.n_nodes
    X = torch.randn(n, din, device=DEV)
    W1, W2 = torch.randn(dout, din, device=DEV) * 0.2, torch.randn(dout, din, device=DEV) * 0.2
    b1, b2 = torch.randn(dout, device=DEV) * 0.1, torch.randn(dout, device=DEV) * 0.1
    st = kernels.make_state(n, din, dout, DEV)
    S, H = kernels.propagate_layer(g, X, W1, b1, W2, b2, 0.1, 1234, state=st)
    st2 = kernels.make_state(n, din, dout, DEV)
    H2 = torch.full_like(H, 7.0)
    bounds = [0, 1008, 1024, 2512, n]
    for r0, r1 in zip(bounds[:-1], bounds[1:]):
        kernels.biinter_fwd_rows(X, S, W1, b1, W2, b2, r0, r1 - r0, H2, 0.1, 1234, state=st2)
    assert torch.equal(H, H2)
    assert torch.equal(st.norm[:n], st2.norm[:n])
    assert torch.equal(st.mask[:(n + 15) // 16 * 64], st2.mask[:(n + 15) // 16 * 64])


def test_row_softmax_short_and_long_rows(pkg):
    """a7: the windowed short-row softmax + the hub rows by their long-row plan segments (model.py:355-366)
    against torch.sparse.softmax on the same CSR; the scan fallback (no long-row list: a block per hub
    row) agrees to fp32 rounding.  A row's bits do not depend on where the entry windows cut: a row view
    starting mid-window (as a shard's rows) reproduces the whole-CSR values bit for bit."""
    graph_mod, kernels = _mods(pkg)
    # short rows (~9), 300 rows of 33..256 entries, 4 hubs of ~3000 (several 512-entry segments each)
    lay, A = random_graph(graph_mod, 4000, 9, hubs=4, hub_deg=3000, seed=17, mids=300, mid_deg=90)
    g = graph_mod.DeviceGraph(lay, DEV)
    deg = np.diff(lay.rowptr)
    assert g.A.n_long > 0 and ((deg > 32) & (deg <= 256)).sum() > 200
    logits = torch.randn(lay.nnz) * 3
    kernels.row_softmax(g, logits.to(DEV))
    got = g.A.val.detach().cpu()
    ref = torch.sparse.softmax(torch.sparse_coo_tensor(A.indices(), logits, A.shape).coalesce(), dim=1)
    np.testing.assert_allclose(got.numpy(), ref.values().numpy(), rtol=1e-5, atol=1e-7)
    lib = __import__(pkg.__name__ + "._lib", fromlist=["_lib"])
    out = torch.empty(lay.nnz, device=DEV)
    lib.call("kgat_row_softmax_f32", g.A.rowptr.data_ptr(), g.n_nodes, logits.to(DEV).data_ptr(), out.data_ptr(),
             torch.cuda.current_stream().cuda_stream)
    np.testing.assert_allclose(out.cpu().numpy(), got.numpy(), rtol=1e-5, atol=1e-8)
    for r0, r1 in ((0, 4000), (7, 3901), (1234, 1300), (2999, 4000)):
        view = graph_mod._CSRRowView(g.A, r0, r1, DEV)
        part = torch.full((lay.nnz,), float("nan"), device=DEV)
        kernels.row_softmax_csr(view, logits.to(DEV), part)
        e0, e1 = int(lay.rowptr[r0]), int(lay.rowptr[r1])
        assert torch.equal(part[e0:e1].cpu(), got[e0:e1]), (r0, r1)
        assert torch.isnan(part[:e0]).all() and torch.isnan(part[e1:]).all()  # nothing written outside


def test_row_softmax_wide_graph_column_cut_plan(pkg):
    """on a graph wide enough for the SpMM's column-cut plan (>= 8 x 8192 columns: A.descriptor()'s
    hub segments end at 8192-column boundaries, variable length) the row softmax runs on the fixed 512-entry
    plan (softmax_descriptor) and matches torch.sparse.softmax -- hub rows crossing many column blocks, the
    whole CSR and row views of it bit for bit -- and kgat_row_softmax_plan_f32 rejects the column-cut
    descriptor (seg_len 0) instead of computing wrong hub-row values."""
    graph_mod, kernels = _mods(pkg)
    lay, A = random_graph(graph_mod, 80000, 6, hubs=6, hub_deg=4000, seed=23, mids=200, mid_deg=120)
    g = graph_mod.DeviceGraph(lay, DEV)
    assert g.A.col_cuts and g.A.n_long >= 6
    desc, sdesc = g.A.descriptor(), g.A.softmax_descriptor()
    assert desc.seg_len == 0 and sdesc.seg_len == graph_mod.SEG_LEN and desc.n_seg > sdesc.n_seg
    logits = (torch.randn(lay.nnz) * 3).to(DEV)
    kernels.row_softmax(g, logits)
    got = g.A.val.detach().cpu()
    ref = torch.sparse.softmax(torch.sparse_coo_tensor(A.indices(), logits.cpu(), A.shape).coalesce(), dim=1)
    np.testing.assert_allclose(got.numpy(), ref.values().numpy(), rtol=1e-5, atol=1e-7)
    for r0, r1 in ((0, 80000), (11, 79001), (40000, 40517)):
        view = graph_mod._CSRRowView(g.A, r0, r1, DEV)
        assert view.descriptor().seg_len == 0
        part = torch.full((lay.nnz,), float("nan"), device=DEV)
        kernels.row_softmax_csr(view, logits, part)
        e0, e1 = int(lay.rowptr[r0]), int(lay.rowptr[r1])
        assert torch.equal(part[e0:e1].cpu(), got[e0:e1]), (r0, r1)
    lib = __import__(pkg.__name__ + "._lib", fromlist=["_lib"])
    work = torch.empty(2 * desc.n_seg + 2, device=DEV)
    out = torch.empty(lay.nnz, device=DEV)
    rc = lib.lib().kgat_row_softmax_plan_f32(ctypes.byref(desc), ctypes.c_void_p(logits.data_ptr()),
                                             ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(work.data_ptr()),
                                             ctypes.c_int64(work.numel()),
                                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 1001  # KGAT_ERR_INVALID: the column-cut plan is not the softmax's


def test_biinter_bwd_rows_matches_dense(pkg):
    _, kernels = _mods(pkg)
    torch.manual_seed(9)
    n, din, dout = 2000, 64, 32
    X, S = torch.randn(n, din), torch.randn(n, din)
    W1, W2 = torch.randn(dout, din) * 0.2, torch.randn(dout, din) * 0.2
    b1, b2 = torch.randn(dout) * 0.1, torch.randn(dout) * 0.1
    F = torch.from_numpy(np.random.default_rng(1).choice(n, 150, replace=False))
    rows = torch.cat([F, torch.full((42,), -1)]).int()
    dHc = torch.zeros(192, dout)
    dHc[:150] = torch.randn(150, dout)
    dH = torch.zeros(n, dout)
    dH[F] = dHc[:150]
    dv = [t.to(DEV) for t in (X, S, W1, b1, W2, b2)]
    for p in (0.0, 0.1):
        dense = kernels.biinter_bwd(dv[0], dv[1], dH.to(DEV), *dv[2:], dropout_p=p, seed=77)
        comp = kernels.biinter_bwd(dv[0], dv[1], dHc.to(DEV), *dv[2:], dropout_p=p, seed=77, rows=rows.to(DEV))
        np.testing.assert_allclose(comp[0][:150].cpu().numpy(), dense[0][F.to(DEV)].cpu().numpy(), rtol=1e-5,
                                   atol=1e-7)
        np.testing.assert_allclose(comp[1][:150].cpu().numpy(), dense[1][F.to(DEV)].cpu().numpy(), rtol=1e-5,
                                   atol=1e-7)
        for a, b in zip(comp[2:], dense[2:]):
            np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4, atol=1e-6)


def _load_params(m, g, prefixes):
    sd = m.state_dict()
    for k in sd:
        if sd[k].is_sparse:
            continue
        for pre in prefixes:
            if pre + k in g:
                sd[k] = torch.from_numpy(g[pre + k])
    m.load_state_dict(sd)


@pytest.mark.parametrize("case", KGAT_CASES)
def test_kg_train_steps_vs_reference(pkg, case):
    """TransR loss, dense table / relation / trans gradients and the KG Adam step (model.py:204-261, 414-419)."""
    g = golden("kgat_" + case)
    m = _model_from_golden(pkg, g)
    _load_params(m, g, ["init/", "after_cf/"])
    m.to(DEV)
    m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    named = dict(m.named_parameters())
    s = 0
    while f"kg{s}/loss" in g:
        ids = [torch.from_numpy(g[f"kg{s}/{x}"]).to(DEV) for x in ("heads", "rels", "pos", "neg")]
        loss = m(*ids, mode=pkg.KGATMode.TRAIN_KG)
        loss.backward()
        np.testing.assert_allclose(loss.item(), g[f"kg{s}/loss"], rtol=1e-5)
        for k, prm in named.items():
            ref = g.get(f"kg{s}/grad/{k}")
            if ref is None:
                assert prm.grad is None, k
            else:
                np.testing.assert_allclose(prm.grad.cpu().numpy(), ref, rtol=RTOL, atol=1e-6, err_msg=k)
        m.update_kg_weights()
        s += 1
    for k, v in g.items():
        if k.startswith("after_kg/"):
            np.testing.assert_allclose(named[k[9:]].detach().cpu().numpy(), v, rtol=RTOL, atol=ADAM_ATOL, err_msg=k)


@pytest.mark.parametrize("dim,batch,n_rel", [(64, 512, 10), (64, 700, 3), (256, 300, 10), (32, 1, 4)])
def test_kg_step_synthetic_vs_oracle(pkg, dim, batch, n_rel):
    """TransR loss and every gradient vs the oracle at batch sizes that cross the weight-gradient
    kernel's 256-sample windows and LDS stages (d = 256 stages 6 samples, d = 64 16), with
    repeated ids and relations holding no sample."""
    n = 3000
    torch.manual_seed(dim + batch)
    m = pkg.KGAT(pkg.KGATArgs(user_num=100, entity_num=n - 100, relation_num=n_rel, cf_embedding_dim=dim,
                              kg_embedding_dim=dim, layer_size=[dim]))
    init = {k: v.clone() for k, v in m.state_dict().items() if not v.is_sparse}
    m.to(DEV)
    rng = np.random.default_rng(batch)
    rel_hi = max(1, n_rel - 1)  # the last relation gets no sample
    ids = [torch.from_numpy(rng.integers(0, hi, batch)) for hi in (200, rel_hi, 200, n)]
    loss = m(*[t.to(DEV) for t in ids], mode=pkg.KGATMode.TRAIN_KG)
    loss.backward()
    P = {k: v.clone().requires_grad_(True) for k, v in init.items()}
    ref = K.transr_loss(P, *ids)
    ref.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-5)
    for k, prm in m.named_parameters():
        if prm.grad is None or P[k].grad is None:
            continue
        np.testing.assert_allclose(prm.grad.cpu().numpy(), P[k].grad.numpy(), rtol=RTOL, atol=1e-6, err_msg=k)
    assert float(m._trans_matrix.grad[n_rel - 1].abs().max()) == 0.0 or n_rel == 1


def _refreshed_model(pkg, g):
    m = _model_from_golden(pkg, g)
    _load_params(m, g, ["init/", "after_cf/", "after_kg/"])
    m.to(DEV)
    m.eval()
    args = [torch.from_numpy(g[x]).to(DEV) for x in ("kg_heads", "kg_rels", "kg_tails", "adjacency_relations")]
    m(*args, mode=pkg.KGATMode.UPDATE_ATTENTION)
    return m


@pytest.mark.parametrize("case", KGAT_CASES)
def test_attention_refresh_vs_reference(pkg, case):
    """Edge scores + per-row softmax stay on the device (model.py:318-366, host round trip removed)."""
    g = golden("kgat_" + case)
    m = _refreshed_model(pkg, g)
    att = m.attentive_matrix.data.coalesce()
    np.testing.assert_array_equal(att.indices().cpu().numpy(), g["att_idx"])
    np.testing.assert_allclose(att.values().cpu().numpy(), g["att_val"], rtol=RTOL, atol=1e-6)
    # A^T values follow the refresh (used by the next backward)
    gr = m.graph()
    np.testing.assert_array_equal(gr.AT.val.cpu().numpy(), gr.A.val.cpu().numpy()[gr.perm_t.cpu().numpy()])


@pytest.mark.parametrize("case", KGAT_CASES)
def test_predict_scores_and_top20_vs_reference(pkg, case):
    g = golden("kgat_" + case)
    m = _refreshed_model(pkg, g)
    users = torch.from_numpy(g["eval_users"]).to(DEV)
    items = torch.arange(int(g["item_num"]), device=DEV)
    with torch.no_grad():
        sc = m(users, items, mode=pkg.KGATMode.PREDICT).cpu()
    np.testing.assert_allclose(sc.numpy(), g["scores"], rtol=RTOL, atol=1e-5)
    masked = sc.clone()
    ref_masked = torch.from_numpy(g["scores"].copy())
    for u, i in g["train_flat"]:
        row = np.nonzero(g["eval_users"] == u)[0]
        if row.size:
            masked[row[0], i] = -np.inf
            ref_masked[row[0], i] = -np.inf
    top = torch.topk(masked, 20, dim=1).indices.numpy()
    ref_top = g["topk20"]
    # bit-exact top-20 except where the reference's own scores are within fp32 noise of a tie
    for r in range(top.shape[0]):
        if not np.array_equal(top[r], ref_top[r]):
            vals = np.sort(ref_masked[r].numpy())[::-1][:21]
            assert np.min(np.abs(np.diff(vals))) < 1e-5, (r, top[r], ref_top[r])


def _nfm_batch(g, users, items):
    U = int(g["user_num"])
    F = U + int(g["entity_num"])
    I = int(g["item_num"])
    feat = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([g["feat_row"], g["feat_col"]])),
                                   torch.from_numpy(g["feat_val"]), (I, int(g["entity_num"]))).to_dense()
    x = torch.zeros(len(users), F)
    x[torch.arange(len(users)), torch.from_numpy(np.asarray(users))] = 1.0
    x[:, U:] = feat[torch.from_numpy(np.asarray(items))]
    return x.to_sparse()


def _nfm_from_golden(pkg, g):
    m = pkg.NFM(pkg.NFMArgs(user_num=int(g["user_num"]), item_num=int(g["item_num"]), entity_num=int(g["entity_num"]),
                            embedding_dim=int(g["dim"]), hidden_dim=g["hidden"].tolist()))
    m.load_state_dict({k[5:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("init/")})
    return m.to(DEV)


def test_nfm_train_steps_vs_reference(pkg):
    """NFM BPR loss, every gradient and the Adam step (NFM/model.py:103-147) vs the reference run."""
    g = golden("nfm_h3_d64")
    m = _nfm_from_golden(pkg, g)
    m.eval()
    m.build_optimizer(lr=1e-4)
    named = dict(m.named_parameters())
    for s in range(2):
        xp = _nfm_batch(g, g[f"tr{s}/users"], g[f"tr{s}/pos"]).to(DEV)
        xn = _nfm_batch(g, g[f"tr{s}/users"], g[f"tr{s}/neg"]).to(DEV)
        loss = m(xp, xn, mode=pkg.NFMMode.TRAIN)
        loss.backward()
        np.testing.assert_allclose(loss.item(), g[f"tr{s}/loss"], rtol=1e-5)
        for k, prm in named.items():
            ref = g.get(f"tr{s}/grad/{k}")
            assert ref is not None, k
            np.testing.assert_allclose(prm.grad.cpu().numpy(), ref, rtol=RTOL, atol=1e-6, err_msg=k)
        m.update_weights()
    for k, v in g.items():
        if k.startswith("after/"):
            name = k[6:]
            # An element whose reference gradient stayed at fp32-cancellation level in every step (e.g. the
            # wide-head bias: it cancels exactly in y_pos - y_neg, so its true gradient is 0) is moved by Adam a
            # full +-lr per step in whichever direction the residue's sign points: allow that, nothing else.
            noise = np.all([np.abs(g[f"tr{s}/grad/{name}"]) < 1e-7 for s in range(2)], axis=0)
            tol = np.where(noise, 2 * 1e-4 + 1e-7, ADAM_ATOL + RTOL * np.abs(v))
            got = named[name].detach().cpu().numpy()
            assert np.all(np.abs(got - v) <= tol), (name, np.max(np.abs(got - v)))
    # PREDICT from the reference's own post-training weights (the wide bias above is noise-driven)
    sd = m.state_dict()
    for k in sd:
        sd[k] = torch.from_numpy(g["after/" + k]) if "after/" + k in g else sd[k]
    m.load_state_dict(sd)
    users = g["pred_users"]
    I = int(g["item_num"])
    x = _nfm_batch(g, np.repeat(users, I), np.tile(np.arange(I), len(users))).to(DEV)
    sc = m(x, mode=pkg.NFMMode.PREDICT).cpu().numpy()
    np.testing.assert_allclose(sc, g["pred_scores"], rtol=RTOL, atol=1e-5)


def _skewed_nfm_batch(rng, rows, U, F):
    """Rows of one user (from 5: runs of ~rows/5 equal feature ids), one item, three of
    eight shared tags and a real-valued rating feature: long runs cross the backward's
    16-entry chunks of the feature-sorted entries."""
    r_idx, c_idx, vals = [], [], []
    for r in range(rows):
        feats = [int(rng.integers(0, 5)), int(U + rng.integers(0, 50))]
        feats += [int(U + 50 + t) for t in rng.choice(8, 3, replace=False)]
        vs = [1.0] * 5
        feats.append(F - 1)
        vs.append(float(rng.uniform(0.2, 1.0)))
        r_idx += [r] * len(feats)
        c_idx += feats
        vals += vs
    return torch.sparse_coo_tensor(torch.tensor([r_idx, c_idx]), torch.tensor(vals, dtype=torch.float32), (rows, F))


@pytest.mark.parametrize("dim,hidden", [(64, [64, 32, 16]), (128, [128, 64]), (200, [96]), (32, [])])
def test_nfm_shapes_and_long_runs_vs_oracle(pkg, dim, hidden):
    """NFM loss, every gradient and PREDICT scores vs the oracle (NFM/model.py:73-129) for the
    LDS-staged (d=64), global-weight (d=128, 200) and no-hidden-layer forwards, with feature
    runs far longer than a backward chunk."""
    rng = np.random.default_rng(dim)
    torch.manual_seed(dim)
    U, E = 40, 120
    m = pkg.NFM(pkg.NFMArgs(user_num=U, item_num=60, entity_num=E, embedding_dim=dim, hidden_dim=hidden,
                            message_dropout=[0.1] * len(hidden))).to(DEV)
    m.eval()
    F = U + E
    xp = _skewed_nfm_batch(rng, 700, U, F)
    xn = _skewed_nfm_batch(rng, 700, U, F)
    params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.named_parameters()}
    ref = K.nfm_loss(params, xp, xn, lam=1e-5)
    ref.backward()
    loss = m(xp.to(DEV), xn.to(DEV), mode=pkg.NFMMode.TRAIN)
    loss.backward()
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-5)
    for k, prm in m.named_parameters():
        want = params[k].grad.numpy()
        np.testing.assert_allclose(prm.grad.cpu().numpy(), want, rtol=1e-3, atol=1e-6 + 1e-4 * np.abs(want).max(),
                                   err_msg=k)
    with torch.no_grad():
        sc = m(xp.to(DEV), mode=pkg.NFMMode.PREDICT).cpu().numpy()
        want = K.nfm_score({k: v.detach() for k, v in params.items()}, xp).numpy()
    np.testing.assert_allclose(sc, want, rtol=RTOL, atol=1e-5)


def test_nfm_batcher_vs_reference_batches(pkg):
    """§8(f)2: NFMBatcher's device-built feature batches equal the reference's scipy construction
    (NFM/preprocess.py:150-193 feature matrix, 284-307 train rows, 309-334 test grid), entry for
    entry after coalescing, and score / train identically to the COO input."""
    rng = np.random.default_rng(5)
    U, I, E = 30, 40, 90
    heads = rng.integers(0, I, 150)
    tails = rng.integers(I, E, 150)  # duplicates included: summed like coo -> csr
    inter = {u: sorted(rng.choice(I, 5, replace=False).tolist()) for u in range(U)}
    b = pkg.NFMBatcher(U, I, E, heads, tails, inter, DEV, train_batch_size=16)
    feat = K.nfm_feature_matrix(I, E, heads, tails)

    def same(got, want):
        want = want.coalesce()
        assert got.shape == tuple(want.shape)
        np.testing.assert_array_equal(torch.stack([got.rows, got.cols]).cpu().numpy(), want.indices().numpy())
        np.testing.assert_array_equal(got.vals.cpu().numpy(), want.values().numpy())
        rp = np.searchsorted(want.indices()[0].numpy(), np.arange(got.shape[0] + 1))
        np.testing.assert_array_equal(got.rowptr.cpu().numpy(), rp)

    users, items = rng.integers(0, U, 50), rng.integers(0, I, 50)
    xb = b.build(torch.from_numpy(users), torch.from_numpy(items))
    same(xb, K.nfm_train_feature_batch(U, feat, users, items))
    grid = b.generate_test_batch([3, 7, 0])
    same(grid, K.nfm_test_feature_batch(U, feat, [3, 7, 0]))
    assert b.build(torch.zeros(0, dtype=torch.int64), torch.zeros(0, dtype=torch.int64)).rows.numel() == 0
    with pytest.raises(IndexError):
        b.build(torch.tensor([U]), torch.tensor([0]))

    pos, neg = b.generate_train_batch()
    for r in range(pos.shape[0]):  # row r: user column, then the item's one-hot at user_num + item
        beg = int(pos.rowptr[r])
        u, it = int(pos.cols[beg]), int(pos.cols[beg + 1]) - U
        assert it in inter[u]
        nb = int(neg.rowptr[r])
        assert int(neg.cols[nb]) == u and int(neg.cols[nb + 1]) - U not in inter[u]
    torch.manual_seed(1)
    m = pkg.NFM(pkg.NFMArgs(user_num=U, item_num=I, entity_num=E)).to(DEV)
    m.eval()
    with torch.no_grad():
        np.testing.assert_array_equal(m(grid, mode=pkg.NFMMode.PREDICT).cpu().numpy(),
                                      m(grid.to_sparse_coo(), mode=pkg.NFMMode.PREDICT).cpu().numpy())
    l1 = m(pos, neg, mode=pkg.NFMMode.TRAIN)
    l2 = m(pos.to_sparse_coo(), neg.to_sparse_coo(), mode=pkg.NFMMode.TRAIN)
    assert l1.item() == l2.item()


def test_nfm_train_mode_dropout_runs(pkg):
    g = golden("nfm_h3_d64")
    m = _nfm_from_golden(pkg, g)
    m.train()
    xp = _nfm_batch(g, g["tr0/users"], g["tr0/pos"]).to(DEV)
    xn = _nfm_batch(g, g["tr0/users"], g["tr0/neg"]).to(DEV)
    loss = m(xp, xn, mode=pkg.NFMMode.TRAIN)
    loss.backward()
    assert torch.isfinite(loss).item()
    assert all(torch.isfinite(p.grad).all().item() for p in m.parameters())


def _dicts_from_golden(g):
    train, test = {}, {}
    for u, i in g["train_flat"]:
        train.setdefault(int(u), []).append(int(i))
    for u, i in g["test_flat"]:
        test.setdefault(int(u), []).append(int(i))
    for u in g["eval_users"]:
        train.setdefault(int(u), [])
    return train, test


def _assert_metrics(got, g, scores_ref, train):
    """Metrics equal the reference's except on rows whose own top-k boundary is a fp32 near-tie."""
    users = g["eval_users"]
    for k in (20, 40):
        for m in ("precision", "recall", "ndcg"):
            a, b = got[k][m], g[f"metrics/{k}/{m}"]
            bad = ~np.isclose(a, b, rtol=1e-5, atol=1e-7, equal_nan=True)
            for r in np.nonzero(bad)[0]:
                row = scores_ref[r].copy()
                row[train[int(users[r])]] = -np.inf
                vals = np.sort(row)[::-1][:k + 1]
                assert np.min(np.abs(np.diff(vals))) < 1e-5, (k, m, r, a[r], b[r])


@pytest.mark.parametrize("case", KGAT_CASES)
def test_rank_metrics_on_reference_scores(pkg, case):
    """The reference's own score matrix through kgat_mask_rows/topk/rank_metrics == its metrics_at_k."""
    ev = pkg.evaluation
    g = golden("kgat_" + case)
    train, test = _dicts_from_golden(g)
    sc = torch.from_numpy(g["scores"].copy()).to(DEV)
    got = ev.metrics_at_k(sc, train, test, g["eval_users"], np.arange(int(g["item_num"])), [20, 40])
    _assert_metrics(got, g, g["scores"], train)
    # in-place masking, as the reference does
    for u, i in g["train_flat"][:50]:
        r = np.nonzero(g["eval_users"] == u)[0]
        if r.size:
            assert sc[r[0], i].item() == float("-inf")


@pytest.mark.parametrize("case", KGAT_CASES)
def test_evaluate_vs_reference(pkg, case):
    """main.py:70-130 driven through evaluation.evaluate (one propagation) == the reference's means."""
    ev = pkg.evaluation
    g = golden("kgat_" + case)
    m = _refreshed_model(pkg, g)
    train, test = _dicts_from_golden(g)
    test = {int(u): test[int(u)] for u in g["eval_users"]}  # the reference iterates eval users in this order
    scores, res, per_user = ev.evaluate(m, train, test, int(g["item_num"]), k_list=[20, 40], batch_size=64,
                                        return_per_user=True)
    np.testing.assert_allclose(scores.numpy(), g["scores"], rtol=RTOL, atol=1e-5)
    # per user: exactly the reference's metric, except users whose reference top-k boundary is a near-tie
    _assert_metrics(per_user, g, g["scores"], train)
    for k in (20, 40):
        for name in ("precision", "recall", "ndcg"):
            assert res[k][name] == pytest.approx(float(np.mean(per_user[k][name])), rel=1e-6)


@pytest.mark.parametrize("rows,cols,k", [(3, 1, 1), (64, 1000, 20), (17, 5000, 100), (8, 100_000, 1024),
                                         (33, 777, 777)])
def test_topk_kernel_ties_and_inf(pkg, rows, cols, k):
    ev = pkg.evaluation
    rng = np.random.default_rng(rows * 7 + k)
    x = rng.integers(-50, 50, size=(rows, cols)).astype(np.float32) / 8  # many exact ties
    x[rng.random((rows, cols)) < 0.05] = -np.inf
    x[rng.random((rows, cols)) < 0.01] = np.inf
    idx, val = ev.topk(torch.from_numpy(x).to(DEV), k, values=True)
    for r in range(rows):
        order = np.lexsort((np.arange(cols), -x[r].astype(np.float64)))[:k]
        np.testing.assert_array_equal(idx[r].cpu().numpy(), order)
        np.testing.assert_array_equal(val[r].cpu().numpy(), x[r][order])


def test_recommend_topk_matches_masked_torch_topk(pkg):
    ev = pkg.evaluation
    g = golden("kgat_L2_d64")
    m = _refreshed_model(pkg, g)
    train, _ = _dicts_from_golden(g)
    users = list(range(int(g["user_num"])))
    I = int(g["item_num"])
    top = ev.recommend_topk(m, users, I, train, k=20, batch_size=32)
    with torch.no_grad():
        sc = m(torch.tensor(users, device=DEV), torch.arange(I, device=DEV), mode=pkg.KGATMode.PREDICT).cpu()
    for u in users:
        sc[u, train.get(u, [])] = -np.inf
    ref = torch.topk(sc, 20, dim=1)
    got_vals = torch.gather(sc, 1, top)
    np.testing.assert_array_equal(got_vals.numpy(), ref.values.numpy())  # same scores at every rank


def test_bpr_bwd_row_map_skips_unowned_rows(pkg):
    """row_map -1 (a row another shard owns) is skipped; mapped rows get the dense gradient."""
    _, kernels = _mods(pkg)
    torch.manual_seed(4)
    n, d, B = 300, 32, 64
    tab = torch.randn(n, d, device=DEV)
    users = torch.randint(0, n, (B,), device=DEV)
    pos = torch.randint(0, n, (B,), device=DEV)
    neg = torch.randint(0, n, (B,), device=DEV)
    loss, coef = kernels.bpr_fwd([tab], users, pos, neg, 1e-5)
    gout = torch.ones(1, device=DEV)
    dense = torch.zeros(n, d, device=DEV)
    kernels.bpr_bwd([tab], 0, users, pos, neg, 1e-5, coef, gout, dense)
    owned = torch.arange(n, device=DEV) % 3 == 0
    row_map = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    row_map[owned] = torch.arange(int(owned.sum()), dtype=torch.int32, device=DEV)
    comp = torch.zeros(int(owned.sum()), d, device=DEV)
    kernels.bpr_bwd([tab], 0, users, pos, neg, 1e-5, coef, gout, comp, row_map=row_map)
    torch.testing.assert_close(comp, dense[owned], rtol=0, atol=0)


@pytest.mark.parametrize("din,dout", [(256, 256), (256, 128), (128, 256), (96, 48)])
def test_biinter_wide_gemm_path(pkg, din, dout):
    """Shapes the fused kernels do not dispatch run rocBLAS GEMMs + HIP epilogues: forward and
    backward vs a torch fp32 autograd reference, with dropout, clamped rows and frontier rows."""
    _, kernels = _mods(pkg)
    assert not kernels.fused_supported(din, dout)
    torch.manual_seed(din + 3 * dout)
    n, p = 2000 + 5, 0.2
    X, S = torch.randn(n, din), torch.randn(n, din)
    X[10:20] = 0.0
    S[10:20] = 0.0
    W1, W2 = torch.randn(dout, din) * 0.1, torch.randn(dout, din) * 0.1
    b1, b2 = torch.zeros(dout), torch.zeros(dout)  # zero rows => g = 0 => F.normalize's clamp
    dv = [t.to(DEV) for t in (X, S, W1, b1, W2, b2)]
    st = kernels.make_state(n, din, dout, DEV)
    H = kernels.biinter_fwd(*dv, dropout_p=p, seed=9, state=st)
    keep = (H.cpu() != 0).float()
    keep[10:20] = 1.0  # zero rows: the mask is not visible there (g = 0 anyway)
    assert abs((1 - keep[20:].mean().item()) - p) < 0.02
    leaves = [t.clone().requires_grad_(True) for t in (X, S, W1, b1, W2, b2)]
    x, s, w1, bb1, w2, bb2 = leaves
    h = (torch.nn.functional.leaky_relu(torch.nn.functional.linear(x + s, w1, bb1), 0.01)
         + torch.nn.functional.leaky_relu(torch.nn.functional.linear(x * s, w2, bb2), 0.01)) * keep / (1 - p)
    ref = h / h.norm(dim=1, keepdim=True).clamp_min(1e-12)
    np.testing.assert_allclose(H.cpu().numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-5)
    dH = torch.randn(n, dout)
    dH[10:20] = 0.0  # keep the 1/eps gradient of clamped rows out of the comparison
    ref.backward(dH)
    got = kernels.biinter_bwd(dv[0], dv[1], dH.to(DEV), *dv[2:], dropout_p=p, seed=9, H=H, state=st)
    want = (x.grad, s.grad, w1.grad, bb1.grad, w2.grad, bb2.grad)
    for i, (a, b) in enumerate(zip(got, want)):
        np.testing.assert_allclose(a.cpu().numpy(), b.numpy(), rtol=1e-3, atol=1e-5 if i < 2 else 1e-4,
                                   err_msg=f"grad {i}")
    # frontier rows (compact dH) == the dense backward restricted to those rows
    F = torch.from_numpy(np.random.default_rng(3).choice(n, 100, replace=False))
    rows = torch.cat([F, torch.full((12,), -1)]).int().to(DEV)
    dHc = torch.zeros(112, dout)
    dHc[:100] = torch.randn(100, dout)
    dHd = torch.zeros(n, dout)
    dHd[F] = dHc[:100]
    st2 = kernels.make_state(n, din, dout, DEV)
    H2 = kernels.biinter_fwd(*dv, dropout_p=p, seed=9, state=st2)
    dense = kernels.biinter_bwd(dv[0], dv[1], dHd.to(DEV), *dv[2:], dropout_p=p, seed=9, H=H2, state=st2)
    st3 = kernels.make_state(n, din, dout, DEV)
    H3 = kernels.biinter_fwd(*dv, dropout_p=p, seed=9, state=st3)
    comp = kernels.biinter_bwd(dv[0], dv[1], dHc.to(DEV), *dv[2:], dropout_p=p, seed=9, rows=rows, H=H3, state=st3)
    Fd = F.to(DEV)
    np.testing.assert_allclose(comp[0][:100].cpu().numpy(), dense[0][Fd].cpu().numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(comp[1][:100].cpu().numpy(), dense[1][Fd].cpu().numpy(), rtol=1e-4, atol=1e-6)
    for a, b in zip(comp[2:], dense[2:]):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("din,dout", [(128, 128), (128, 64)])
def test_biinter_wide_bits_state(pkg, din, dout):
    """C4's wide layers: fused MFMA forward keeping norm + sign/keep bits (ceil(d_out/64) words per
    lane), rocBLAS backward from those bits -- vs a torch fp32 autograd reference (dropout, clamped
    rows), frontier rows vs the dense backward, and vs the pre-activation (gemm) state path."""
    _, kernels = _mods(pkg)
    assert kernels.bits_supported(din, dout)
    torch.manual_seed(din + 5 * dout)
    n, p = 3000 + 9, 0.2
    X, S = torch.randn(n, din), torch.randn(n, din)
    X[10:20] = 0.0
    S[10:20] = 0.0
    W1, W2 = torch.randn(dout, din) * 0.1, torch.randn(dout, din) * 0.1
    b1, b2 = torch.zeros(dout), torch.zeros(dout)
    dv = [t.to(DEV) for t in (X, S, W1, b1, W2, b2)]
    st = kernels.make_state(n, din, dout, DEV)
    assert st.kind == "bits"
    H = kernels.biinter_fwd(*dv, dropout_p=p, seed=9, state=st)
    assert torch.equal(H, kernels.biinter_fwd(*dv, dropout_p=p, seed=9))
    keep = (H.cpu() != 0).float()
    keep[10:20] = 1.0
    leaves = [t.clone().requires_grad_(True) for t in (X, S, W1, b1, W2, b2)]
    x, s, w1, bb1, w2, bb2 = leaves
    h = (torch.nn.functional.leaky_relu(torch.nn.functional.linear(x + s, w1, bb1), 0.01)
         + torch.nn.functional.leaky_relu(torch.nn.functional.linear(x * s, w2, bb2), 0.01)) * keep / (1 - p)
    ref = h / h.norm(dim=1, keepdim=True).clamp_min(1e-12)
    np.testing.assert_allclose(H.cpu().numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-5)
    dH = torch.randn(n, dout)
    dH[10:20] = 0.0
    ref.backward(dH)
    got = kernels.biinter_bwd(dv[0], dv[1], dH.to(DEV), *dv[2:], dropout_p=p, seed=9, H=H, state=st)
    want = (x.grad, s.grad, w1.grad, bb1.grad, w2.grad, bb2.grad)
    for i, (a, b) in enumerate(zip(got, want)):
        np.testing.assert_allclose(a.cpu().numpy(), b.numpy(), rtol=1e-3, atol=1e-5 if i < 2 else 1e-4,
                                   err_msg=f"grad {i}")
    # the pre-activation (gemm) path agrees (its forward is rocBLAS: sums in another order)
    sg = kernels.BiState(n, DEV, din, dout, kind="gemm")
    Hg = kernels.biinter_fwd(*dv, dropout_p=p, seed=9, state=sg)
    np.testing.assert_allclose(Hg.cpu().numpy(), H.cpu().numpy(), rtol=1e-4, atol=1e-6)
    gg = kernels.biinter_bwd(dv[0], dv[1], dH.to(DEV), *dv[2:], dropout_p=p, seed=9, H=Hg, state=sg)
    for i, (a, b) in enumerate(zip(got, gg)):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-3, atol=1e-5, err_msg=f"gemm {i}")
    # frontier rows (compact dH, -1 padding) == the dense backward restricted to those rows
    F = torch.from_numpy(np.random.default_rng(3).choice(n, 150, replace=False))
    F[:3] = torch.tensor([10, 11, n - 1])
    rows = torch.cat([F, torch.full((10,), -1)]).int().to(DEV)
    dHc = torch.zeros(160, dout)
    dHc[:150] = torch.randn(150, dout)
    dHd = torch.zeros(n, dout)
    dHd[F] = dHc[:150]
    dense = kernels.biinter_bwd(dv[0], dv[1], dHd.to(DEV), *dv[2:], dropout_p=p, seed=9, H=H, state=st)
    comp = kernels.biinter_bwd(dv[0], dv[1], dHc.to(DEV), *dv[2:], dropout_p=p, seed=9, rows=rows, H=H, state=st)
    Fd = F.to(DEV)
    np.testing.assert_allclose(comp[0][:150].cpu().numpy(), dense[0][Fd].cpu().numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(comp[1][:150].cpu().numpy(), dense[1][Fd].cpu().numpy(), rtol=1e-4, atol=1e-6)
    assert float(comp[0][150:].abs().max()) == 0.0 and float(comp[1][150:].abs().max()) == 0.0
    for a, b in zip(comp[2:], dense[2:]):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-3, atol=1e-5)


def test_reference_checkpoint_predict_and_round_trip(pkg, tmp_path):
    """§8(f)4: a kgat.pth / nfm.pth written by the reference's save_model loads through its load_model
    recipe (load_state_dict, eval) and PREDICT reproduces the scores the reference computed from that
    state; our own checkpoint round-trips bit-exactly."""
    from tests.conftest import GOLDEN
    g = golden("kgat_L2_d64")
    args = pkg.KGATArgs(user_num=int(g["user_num"]), entity_num=int(g["entity_num"]),
                        relation_num=len(g["adjacency_relations"]), layer_size=[64, 32])
    m = pkg.KGAT(args)
    ck = torch.load(GOLDEN / "kgat_L2_d64_ckpt.pth", map_location="cpu", weights_only=True)
    m.load_state_dict(ck["model_state_dict"])
    m.eval()
    m.to(DEV)
    users = torch.from_numpy(g["eval_users"]).to(DEV)
    items = torch.arange(int(g["item_num"]), device=DEV)
    with torch.no_grad():
        sc = m(users, items, mode=pkg.KGATMode.PREDICT)
    np.testing.assert_allclose(sc.cpu().numpy(), g["scores"], rtol=RTOL, atol=1e-5)
    torch.save({"model_state_dict": m.state_dict()}, tmp_path / "kgat.pth")
    m2 = pkg.KGAT(args)
    m2.load_state_dict(torch.load(tmp_path / "kgat.pth", map_location="cpu", weights_only=True)["model_state_dict"])
    m2.eval()
    m2.to(DEV)
    with torch.no_grad():
        assert torch.equal(m2(users, items, mode=pkg.KGATMode.PREDICT), sc)
    gn = golden("nfm_h3_d64")
    n = pkg.NFM(pkg.NFMArgs(user_num=int(gn["user_num"]), item_num=int(gn["item_num"]),
                            entity_num=int(gn["entity_num"]), embedding_dim=int(gn["dim"]),
                            hidden_dim=gn["hidden"].tolist()))
    ckn = torch.load(GOLDEN / "nfm_h3_d64_ckpt.pth", map_location="cpu", weights_only=True)
    n.load_state_dict(ckn["model_state_dict"])
    n.eval()
    n.to(DEV)
    I = int(gn["item_num"])
    x = _nfm_batch(gn, np.repeat(gn["pred_users"], I), np.tile(np.arange(I), len(gn["pred_users"]))).to(DEV)
    np.testing.assert_allclose(n(x, mode=pkg.NFMMode.PREDICT).cpu().numpy(), gn["pred_scores"], rtol=RTOL, atol=1e-5)


def test_adam_multi_matches_single_bit_exact(pkg):
    _, kernels = _mods(pkg)
    torch.manual_seed(8)
    sizes = [1, 3, 4, 5, 1023, 4096, 4097, 300001] + [17] * 12  # > 16 tensors: two launches
    single, multi = [], []
    for n in sizes:
        p, g = torch.randn(n, device=DEV), torch.randn(n, device=DEV) * 1e-3
        m, v = torch.randn(n, device=DEV) * 1e-3, torch.rand(n, device=DEV) * 1e-6
        single.append([t.clone() for t in (p, g, m, v)])
        multi.append([t.clone() for t in (p, g, m, v)])
    for k, (p, g, m, v) in enumerate(single):
        kernels.adam(p, g, m, v, 1e-3 / (1 - 0.9 ** (k + 1)), 0.9, 0.999, (1 - 0.999 ** (k + 1)) ** 0.5, 1e-8)
    kernels.adam_multi([(p, g, m, v, 1e-3 / (1 - 0.9 ** (k + 1)), (1 - 0.999 ** (k + 1)) ** 0.5)
                        for k, (p, g, m, v) in enumerate(multi)], 0.9, 0.999, 1e-8)
    for a, b in zip(single, multi):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


@pytest.mark.parametrize("dim", [64, 128, 256])
def test_attention_refresh_synthetic_vs_oracle(pkg, dim):
    """UPDATE_ATTENTION on a synthetic CKG vs the oracle: d=64 / 128 run the fused MFMA scorer (tiles paired
    per wave; relation boundaries inside a pair), d=256 (C5) the GEMM scorer (csrc/attention_gemm.hip);
    several chunks and relation runs per chunk."""
    graph_mod, kernels = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(3000, 24000, seed=21)
    lay = graph_mod.build_layout(U, E, inter, trip)
    torch.manual_seed(5)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[dim // 2],
                              cf_embedding_dim=dim, kg_embedding_dim=dim))
    params = {k: v.clone() for k, v in m.state_dict().items() if not v.is_sparse}
    m.attach_graph(lay, DEV)
    m.eval()
    h, r, t = (torch.from_numpy(x).to(DEV) for x in (lay.heads, lay.rels, lay.tails))
    old, kernels.EDGE_GEMM_CHUNK = kernels.EDGE_GEMM_CHUNK, 5000  # chunks end inside relation runs
    try:
        m(h, r, t, torch.tensor(lay.rel_order, device=DEV), mode=pkg.KGATMode.UPDATE_ATTENTION)
    finally:
        kernels.EDGE_GEMM_CHUNK = old
    ref = K.refresh_attention(params, torch.from_numpy(lay.heads), torch.from_numpy(lay.rels),
                              torch.from_numpy(lay.tails), lay.rel_order, U + E)
    att = m.attentive_matrix.data.coalesce()
    np.testing.assert_array_equal(att.indices().cpu().numpy(), ref.indices().numpy())
    np.testing.assert_allclose(att.values().cpu().numpy(), ref.values().numpy(), rtol=1e-4, atol=1e-6)


def test_rows_union_and_merge(pkg):
    """kgat_rows_union / kgat_rows_merge_f32 (the replicas' hop-set exchange): the union of G ascending
    lists (padding after each count ignored) and, per union row, the scaled sum of the lists' rows in
    list order -- bit-exact against numpy summing in the same order."""
    graph_mod, kernels = _mods(pkg)
    rng = np.random.default_rng(21)
    n, G, cap, w = 5000, 3, 900, 128
    h, t = rng.integers(0, n, 2000), rng.integers(0, n, 2000)
    rowptr, col, val = graph_mod.csr_from_coo(n, h, t, rng.random(h.size).astype(np.float32))
    lay = graph_mod.GraphLayout(n_nodes=n, rel_order=[], heads=np.zeros(0, np.int64), rels=np.zeros(0, np.int64),
                                tails=np.zeros(0, np.int64), edge_vals=np.zeros(0, np.float32), rowptr=rowptr,
                                col=col, val=val, slot=np.zeros(0, np.int64))
    g = graph_mod.DeviceGraph(lay, DEV)
    counts = np.array([900, 0, 611], np.int32)
    lists = np.full(G * cap, -7, np.int32)  # padding must be ignored
    for k in range(G):
        lists[k * cap:k * cap + counts[k]] = np.sort(rng.choice(n, counts[k], replace=False))
    vals = rng.standard_normal((G * cap, w)).astype(np.float32)
    ld, cd, vd = (torch.from_numpy(x).to(DEV) for x in (lists, counts, vals))
    rows, node_map, count, rank = kernels.rows_union(g, ld, cd, cap)
    want = np.unique(np.concatenate([lists[k * cap:k * cap + counts[k]] for k in range(G)]))
    u = int(count.item())
    assert u == want.size
    np.testing.assert_array_equal(rows[:u].cpu().numpy(), want)
    m = node_map.cpu().numpy()
    np.testing.assert_array_equal(m[want], np.arange(u))
    assert np.all(np.delete(m, want) == -1)
    words = (n + 31) // 32
    ref = kernels.map_rank(node_map, torch.empty(words, dtype=torch.int64, device=DEV)).cpu().numpy().view(np.uint64)
    got = rank[:words].cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got & 0xFFFFFFFF, ref & 0xFFFFFFFF)
    out = kernels.rows_merge(ld, cd, cap, vd, rows, count, G * cap, 0.5).cpu().numpy()
    exp = np.zeros((u, w), np.float32)
    for k in range(G):
        pos = np.searchsorted(want, lists[k * cap:k * cap + counts[k]])
        exp[pos] = exp[pos] + vals[k * cap:k * cap + counts[k]]
    np.testing.assert_array_equal(out[:u], exp * np.float32(0.5))


def test_driver_train_predict_recommend(pkg, tmp_path):
    """make train / predict / recommend (driver.py, main.py:234-636) end to end on a small
    Codeforces-shaped dataset: losses finite and falling, checkpoint in the reference's format,
    PREDICT metrics of the reloaded model equal the last epoch's evaluation of the trained one,
    recommendations exclude every train / test problem of the user."""
    import argparse
    import importlib
    drv = importlib.import_module(pkg.__name__ + ".driver")
    inter, trip, E = drv.synthetic_codeforces(users=60, problems=400, contests=60, tags=12, ratings=8,
                                              per_user=(10, 80), seed=5)
    tr, va, te = drv.split_interactions(inter, 60, seed=5)
    ds = drv.Dataset(60, E, 400, tr, va, te, trip)
    ds.save(tmp_path / "ds.npz")
    args = argparse.Namespace(sm=True, dataset=str(tmp_path / "ds.npz"), epochs=3, max_batches=None, dim=64,
                              layers=[64, 32], result_dir=str(tmp_path / "result"))
    hist = drv.train(args)
    assert len(hist["cf_loss"]) == 3 and all(np.isfinite(hist["cf_loss"] + hist["kg_loss"]))
    assert hist["cf_loss"][-1] < hist["cf_loss"][0]
    ck = torch.load(tmp_path / "result" / "model" / "kgat.pth", map_location="cpu", weights_only=True)
    assert {"_user_entity_embedding.weight", "attentive_matrix", "_trans_matrix"} <= set(ck["model_state_dict"])
    res = drv.predict(args)
    for k in drv.METRICS_K_LIST:
        assert 0.0 < res[k]["recall"] <= 1.0
        for m in ("precision", "recall", "ndcg"):  # same state, same test split as the last epoch's "training"
            assert abs(res[k][m] - hist["training"][-1][k][m]) <= 1e-6, (k, m)
    top = drv.recommend(args).numpy()
    assert top.shape == (60, 20)
    for u in range(60):
        seen = set(tr[tr[:, 0] == u, 1].tolist()) | set(te[te[:, 0] == u, 1].tolist())
        assert not seen & set(top[u].tolist())
    assert (tmp_path / "result" / "recommendations.txt").exists()


def test_out_of_range_ids_raise_index_error(pkg):
    """ids are range-checked before any kernel indexes a table with them (the reference's
    nn.Embedding gathers raise IndexError).  Host ids: at once.  Device ids: on the device, no host
    sync (kgat_ids_check zeroes them, so nothing reads out of range); IndexError at the next call."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(3000, 20000, seed=4)
    lay = graph_mod.build_layout(U, E, inter, trip)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32]))
    m.attach_graph(lay, DEV)
    n = U + E
    ok = torch.arange(8)
    good = (ok.to(DEV), ok.to(DEV), ok.to(DEV))
    calls = [
        lambda bad: m(ok, bad, ok, mode=pkg.KGATMode.TRAIN_CF),
        lambda bad: m(ok, ok % 10, bad, ok, mode=pkg.KGATMode.TRAIN_KG),
        lambda bad: m(bad, ok, mode=pkg.KGATMode.PREDICT),
    ]
    for bad in (torch.full((8,), n), torch.full((8,), -1)):
        for call in calls:
            with pytest.raises(IndexError):  # host ids: immediately
                call(bad)
    with pytest.raises(IndexError):
        m(ok, torch.full((8,), len(lay.rel_order)), ok, ok, mode=pkg.KGATMode.TRAIN_KG)
    for bad in (torch.full((8,), n, device=DEV), torch.full((8,), -7, device=DEV)):
        for mode_call in (lambda: m(ok.to(DEV), bad, ok.to(DEV), mode=pkg.KGATMode.TRAIN_CF),
                          lambda: m(ok.to(DEV), (ok % 10).to(DEV), bad, ok.to(DEV), mode=pkg.KGATMode.TRAIN_KG),
                          lambda: m(ok.to(DEV), bad, ok.to(DEV), ok.to(DEV), mode=pkg.KGATMode.TRAIN_KG),
                          lambda: m(bad, ok.to(DEV), mode=pkg.KGATMode.PREDICT)):
            out = mode_call()  # device ids: runs on zeroed ids, no host sync
            if out is not None:
                assert torch.isfinite(out).all()
            torch.cuda.synchronize()
            with pytest.raises(IndexError):
                m(*good, mode=pkg.KGATMode.TRAIN_CF)
    loss = m(*good, mode=pkg.KGATMode.TRAIN_CF)  # the flag was cleared by the raise
    m.raise_pending(block=True)
    assert torch.isfinite(loss)


def test_c1_sm_shaped_pipeline_vs_reference(pkg):
    """C1 scale (500 users, 9.5k problems, 1.18M nnz, 1 layer, d=64) through the HIP path:
    two eval-mode CF steps + Adam, UPDATE_ATTENTION on all edges, evaluation.evaluate and
    recommend_topk -- top-20 per user and P/R/nDCG@20 per user exactly the reference's (near-ties
    excused by the reference's own top-21 scores), mean recall@20 equal."""
    from tests.conftest import assert_metrics_with_ties, assert_topk_with_ties, c1_inputs

    graph_mod, _ = _mods(pkg)
    ev = pkg.evaluation
    g = golden("kgat_C1_sm")
    U, E, inter, trip, train, test, eval_users = c1_inputs(g)
    lay = graph_mod.build_layout(U, E, inter, trip)
    assert lay.nnz == int(g["nnz"])
    torch.manual_seed(2024)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64],
                              message_dropout=[0.1]))
    m.attach_graph(lay, DEV)
    m.eval()
    m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    for s in range(2):
        loss = m(*(torch.from_numpy(g[f"cf{s}/{x}"]).to(DEV) for x in ("users", "pos", "neg")),
                 mode=pkg.KGATMode.TRAIN_CF)
        np.testing.assert_allclose(loss.item(), g[f"cf{s}/loss"], rtol=1e-5)
        loss.backward()
        m.update_cf_weights()
    att = [torch.from_numpy(x).to(DEV) for x in (lay.heads, lay.rels, lay.tails)] + [torch.tensor(lay.rel_order)]
    m(*att, mode=pkg.KGATMode.UPDATE_ATTENTION)
    test_eval = {int(u): test[int(u)] for u in eval_users}
    _, res, per_user = ev.evaluate(m, train, test_eval, int(g["item_num"]), k_list=[20], return_scores=False,
                                   return_per_user=True)
    assert_metrics_with_ties(per_user[20], g, 20, g["top21_scores"])
    top = ev.recommend_topk(m, [int(u) for u in eval_users], int(g["item_num"]), train, k=20).numpy()
    excused = assert_topk_with_ties(top, g["topk20"].astype(np.int64), g["top21_scores"])
    assert excused <= len(eval_users) // 20, excused  # near-ties at the boundary only, not a ranking error
    # the mean moves only by the excused (near-tie) users' differences
    moved = int((~np.isclose(per_user[20]["recall"], g["metrics/20/recall"], rtol=1e-5, atol=1e-7)).sum())
    assert abs(res[20]["recall"] - float(g["recall20_mean"])) <= 1e-6 + moved / len(eval_users)


@pytest.mark.parametrize("layers", [[64, 32], [32, 16, 16], [64]])
def test_fused_table_update_bit_identical(pkg, layers):
    """KGAT.fuse_table_update (the layer-0 A^T product fused with the table's Adam step,
    kgat_spmm_csr_masked_adam_f32) against the unfused backward + Adam: parameters and both
    Adam moments bit for bit over three train-mode CF steps with a KG step in between (which
    materialises nothing: the CF step already consumed its gradient); a deferred gradient
    materialised on demand equals the unfused one."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(20000, 200000, seed=5)
    lay = graph_mod.build_layout(U, E, inter, trip)
    models = []
    for fused in (False, True):
        torch.manual_seed(2024)
        m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=layers,
                                  message_dropout=[0.1] * len(layers)))
        m.attach_graph(lay, DEV)
        assert m.graph().AT.n_long > 0  # hub rows take the segment + fix-up path
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        m.fuse_table_update = fused
        # the fused model's plain backward also skips the autograd engine (model._StepLoss): the real
        # _cf_fast_backward against the engine's path, bit for bit
        m.direct_backward = fused
        models.append(m)
    rng = np.random.default_rng(4)
    R = len(lay.rel_order)
    for step in range(3):
        ids = [torch.from_numpy(rng.integers(0, hi, 64)).to(DEV) for hi in (U, int(E * 0.1), int(E * 0.1))]
        kg = [torch.from_numpy(rng.integers(0, hi, 32)).to(DEV) for hi in (U + E, R, U + E, U + E)]
        for m in models:
            torch.manual_seed(100 + step)  # same dropout seeds
            loss = m(*ids, mode=pkg.KGATMode.TRAIN_CF)
            assert (getattr(loss.grad_fn, "fast_backward", None) is not None) == m.direct_backward
            loss.backward()
            deferred = m._table_update.pending is not None
            assert deferred == (m._user_entity_embedding.weight.grad is None)
            if m.fuse_table_update and layers == [64, 32]:
                assert deferred  # a compact layer-0 hop set: the fused kernel runs
            m.update_cf_weights()
            m(kg[0], kg[1], kg[2], kg[3], mode=pkg.KGATMode.TRAIN_KG).backward()
            m.update_kg_weights()
    a, b = models
    for (k, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        if not pa.is_sparse:
            assert torch.equal(pa, pb), k
    ta = a._cf_optimizer.state[id(a._user_entity_embedding.weight)]
    tb = b._cf_optimizer.state[id(b._user_entity_embedding.weight)]
    assert ta["step"] == tb["step"] == 3
    assert torch.equal(ta["exp_avg"], tb["exp_avg"]) and torch.equal(ta["exp_avg_sq"], tb["exp_avg_sq"])
    # on-demand materialisation of a deferred gradient
    ids = [torch.from_numpy(rng.integers(0, hi, 64)).to(DEV) for hi in (U, int(E * 0.1), int(E * 0.1))]
    grads = []
    for m in models:
        torch.manual_seed(7)
        m(*ids, mode=pkg.KGATMode.TRAIN_CF).backward()
        if m.fuse_table_update and layers == [64, 32]:
            assert m._user_entity_embedding.weight.grad is None
        m.materialize_table_grad()
        grads.append(m._user_entity_embedding.weight.grad.detach().clone())
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("layers", [[64, 32, 16], [128, 64, 32]])
def test_dense_layer_returns_to_hop_chain(pkg, layers):
    """a lower layer whose hop set was large at one step runs densely afterwards (its size is
    known from the previous step only) -- and re-measures the set every HOP_REPROBE_STEPS dense steps, so
    once the batches are small again the layer goes back to the hop chain (fused and wide kinds)."""
    graph_mod, _ = _mods(pkg)
    model_mod = sys.modules[pkg.__name__ + ".model"]
    # 60k nodes: an 8-pair batch's second hop is ~15 % of the nodes, a 1,300-pair batch's ~65 %
    U, E, inter, trip = graph_mod.synthetic_ckg(60000, 300000, seed=21)
    lay = graph_mod.build_layout(U, E, inter, trip)
    d0 = layers[0] if layers[0] == 128 else 64
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=layers,
                              cf_embedding_dim=d0, kg_embedding_dim=d0, message_dropout=[0.1] * 3))
    m.attach_graph(lay, DEV)
    m.train()
    m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    g = m.graph()
    n = g.n_nodes
    rng = np.random.default_rng(3)

    def step(B):
        ids = [torch.from_numpy(rng.integers(0, hi, B)).to(DEV) for hi in (U, E, E)]
        m(*ids, mode=pkg.KGATMode.TRAIN_CF).backward()
        m.update_cf_weights()
        torch.cuda.synchronize()
        return model_mod._hop_estimate(g, 0)

    step(8)
    big = step(1300)  # the second hop of a 3,900-row batch: most of the graph
    assert big is not None and big > model_mod.HOP_DENSE_FRACTION * n, big
    # layer 1 (the first hop) may have gone dense too: it re-probes first, then layer 0
    ests = [step(8) for _ in range(2 * model_mod.HOP_REPROBE_STEPS + 2)]
    assert ests[-1] is not None and ests[-1] <= model_mod.HOP_DENSE_FRACTION * n, ests
    assert g._hop_dense_steps.get(0, 0) >= 1


def test_fused_table_update_keeps_extra_table_gradient(pkg):
    """with fuse_table_update the CF backward defers the table's gradient, but
    another term of the loss (here an L2 penalty on the whole table) still writes .grad through
    autograd.  update_cf_weights must sum the two (it materialises the deferred product into .grad)
    instead of launching the fused kernel, which never reads .grad: same parameters and moments as
    the unfused step, bit for bit; FusedAdam refuses a fused launch for a parameter with a .grad."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(20000, 200000, seed=5)
    lay = graph_mod.build_layout(U, E, inter, trip)
    models = []
    for fused in (False, True):
        torch.manual_seed(2024)
        m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32],
                                  message_dropout=[0.1, 0.1]))
        m.attach_graph(lay, DEV)
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        m.fuse_table_update = fused
        models.append(m)
    rng = np.random.default_rng(9)
    for step in range(2):
        ids = [torch.from_numpy(rng.integers(0, hi, 64)).to(DEV) for hi in (U, int(E * 0.1), int(E * 0.1))]
        for m in models:
            torch.manual_seed(200 + step)
            loss = m(*ids, mode=pkg.KGATMode.TRAIN_CF) + 1e-3 * m._user_entity_embedding.weight.pow(2).sum()
            loss.backward()
            assert m._user_entity_embedding.weight.grad is not None
            m.update_cf_weights()
    a, b = models
    for (k, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        if not pa.is_sparse:
            assert torch.equal(pa, pb), k
    ta = a._cf_optimizer.state[id(a._user_entity_embedding.weight)]
    tb = b._cf_optimizer.state[id(b._user_entity_embedding.weight)]
    assert torch.equal(ta["exp_avg"], tb["exp_avg"]) and torch.equal(ta["exp_avg_sq"], tb["exp_avg_sq"])
    # the optimiser's own guard
    p = b._user_entity_embedding.weight
    p.grad = torch.zeros_like(p)
    with pytest.raises(RuntimeError, match="fused launch"):
        b._cf_optimizer.step(fused={id(p): lambda *a: None})
    p.grad = None


@pytest.mark.parametrize("dim,batch", [(64, 512), (256, 300), (64, 2000)])
def test_fused_kg_table_update_bit_identical(pkg, dim, batch):
    """KGAT.fuse_kg_table_update (TransR's table rows written compactly,
    kgat_transr_bwd_ex_f32, and the KG Adam stepping the table from them, kgat_adam_rows_f32)
    against the dense backward + Adam: parameters and both KG Adam moments bit for bit over
    alternating CF / KG steps (batches with repeated ids); a deferred KG gradient materialised on
    demand equals the dense one.  B = 2000 exceeds the compact map's 4096 slots: the dense path
    runs, same bits."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(20000, 200000, seed=5)
    lay = graph_mod.build_layout(U, E, inter, trip)
    R = len(lay.rel_order)
    models = []
    for fused in (False, True):
        torch.manual_seed(2024)
        m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=R, layer_size=[dim, dim // 2],
                                  cf_embedding_dim=dim, kg_embedding_dim=dim, message_dropout=[0.1, 0.1]))
        m.attach_graph(lay, DEV)
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        m.fuse_kg_table_update = fused
        models.append(m)
    rng = np.random.default_rng(6)
    for step in range(3):
        ids = [torch.from_numpy(rng.integers(0, hi, 64)).to(DEV) for hi in (U, int(E * 0.1), int(E * 0.1))]
        kg = [torch.from_numpy(rng.integers(0, hi, batch)).to(DEV) for hi in (U + E, R, U + E, U + E)]
        kg[2][:7] = kg[0][:7]  # repeated ids across heads / tails: summed in slot order
        for m in models:
            torch.manual_seed(300 + step)
            m(*ids, mode=pkg.KGATMode.TRAIN_CF).backward()
            m.update_cf_weights()
            m(*kg, mode=pkg.KGATMode.TRAIN_KG).backward()
            deferred = m._kg_table_update.pending is not None
            assert deferred == (m.fuse_kg_table_update and 3 * batch <= 4096)
            assert deferred == (m._user_entity_embedding.weight.grad is None)
            m.update_kg_weights()
    a, b = models
    for (k, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        if not pa.is_sparse:
            assert torch.equal(pa, pb), k
    ta = a._kg_optimizer.state[id(a._user_entity_embedding.weight)]
    tb = b._kg_optimizer.state[id(b._user_entity_embedding.weight)]
    assert ta["step"] == tb["step"] == 3
    assert torch.equal(ta["exp_avg"], tb["exp_avg"]) and torch.equal(ta["exp_avg_sq"], tb["exp_avg_sq"])
    kg = [torch.from_numpy(rng.integers(0, hi, batch)).to(DEV) for hi in (U + E, R, U + E, U + E)]
    grads = []
    for m in models:
        m(*kg, mode=pkg.KGATMode.TRAIN_KG).backward()
        m.materialize_table_grad()
        grads.append(m._user_entity_embedding.weight.grad.detach().clone())
        m.zero_grad(set_to_none=True)
    assert torch.equal(grads[0], grads[1])
    assert int((b._kg_table_update.node_map() >= 0).sum()) == 0  # the batch-row map is reset


@pytest.mark.parametrize("fused", [False, True])
def test_device_id_error_moves_no_parameter(pkg, fused):
    """a device-side id out of range moves no parameter.  The check runs on the
    device without a host synchronisation (kgat_ids_check_ex); its device flag is the optimiser
    kernels' skip flag, so update_cf_weights / update_kg_weights leave the table, the weights and
    both Adam moments as they were (with and without the fused table updates), and IndexError is
    raised at a later call; after it the flag is clear and training steps normally again."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(6000, 60000, seed=11)
    lay = graph_mod.build_layout(U, E, inter, trip)
    torch.manual_seed(5)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32]))
    m.attach_graph(lay, DEV)
    m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    m.fuse_table_update = m.fuse_kg_table_update = fused
    ok = torch.zeros(16, dtype=torch.int64, device=DEV)
    m(ok, ok + 1, ok + 2, mode=pkg.KGATMode.TRAIN_CF).backward()  # one good step: moments exist
    m.update_cf_weights()
    torch.cuda.synchronize()
    before = {k: v.detach().clone() for k, v in m.named_parameters() if not v.is_sparse}
    st = m._cf_optimizer.state[id(m._user_entity_embedding.weight)]
    mom = (st["exp_avg"].clone(), st["exp_avg_sq"].clone())
    bad = torch.full((16,), U + E + 5, dtype=torch.int64, device=DEV)
    m(ok, bad, ok, mode=pkg.KGATMode.TRAIN_CF).backward()
    raised = False
    try:
        m.update_cf_weights()  # may or may not raise yet (the flag's event may have fired); nothing may move
    except IndexError:
        raised = True
    torch.cuda.synchronize()
    for k, v in m.named_parameters():
        if not v.is_sparse:
            assert torch.equal(v.detach(), before[k]), k
    assert torch.equal(st["exp_avg"], mom[0]) and torch.equal(st["exp_avg_sq"], mom[1])
    if not raised:
        with pytest.raises(IndexError):
            m.raise_pending(block=True)
    kg = [ok, ok.clone(), ok + 3, ok + 4]
    m(*kg, mode=pkg.KGATMode.TRAIN_KG).backward()
    m.update_kg_weights()
    torch.cuda.synchronize()
    assert not torch.equal(m._user_entity_embedding.weight.detach(), before["_user_entity_embedding.weight"])


def test_tagged_cf_check_keeps_a_bad_step_reported(pkg):
    """TRAIN_CF's id check reports completion through a tag in pinned memory (kgat_cf_begin_ex: no event
    record behind the launch).  A bad step followed by a good one launched before the host saw the first
    (the GPU held busy) still raises: the flag word is only ever set by the kernels.  After the raise the
    flag is clear, the tag is the last launch's, and the next steps run."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(3000, 20000, seed=4)
    lay = graph_mod.build_layout(U, E, inter, trip)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32]))
    m.attach_graph(lay, DEV)
    ok = torch.arange(8, device=DEV)
    bad = torch.full((8,), U + E + 3, dtype=torch.int64, device=DEV)
    m(ok, ok + 1, ok + 2, mode=pkg.KGATMode.TRAIN_CF)
    m.raise_pending(block=True)
    busy = torch.empty(1 << 26, device=DEV)
    for _ in range(40):  # ~10 ms of GPU work ahead of the two checks
        busy.fill_(1.0)
    m(ok, bad, ok, mode=pkg.KGATMode.TRAIN_CF)
    raised = False
    try:
        m(ok, ok + 1, ok + 2, mode=pkg.KGATMode.TRAIN_CF)  # its check's tag follows the bad one's
    except IndexError:
        raised = True  # the GPU caught up before this call looked
    if not raised:
        with pytest.raises(IndexError):
            m.raise_pending(block=True)
    assert int(m._ids._host[0]) == 0 and int(m._ids._host[1]) == m._ids._tag
    for _ in range(3):
        loss = m(ok, ok + 1, ok + 2, mode=pkg.KGATMode.TRAIN_CF)
    m.raise_pending(block=True)
    assert torch.isfinite(loss)


def test_cf_prologue_marks_first_hop_in_alternating_pairs(pkg):
    """kgat_cf_begin_ex marks the batch's first hop (F and every column of A's rows F) in the spare bitmap
    pair and zeroes the pair the previous step used, in the id check's launch; the listing that follows
    (kgat_frontier_hop_ex, n0 = 0) yields exactly F + N(F), step after step with the pairs alternating, and
    the spare pair is zero between steps."""
    graph_mod, kernels = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(3000, 20000, seed=6)
    lay = graph_mod.build_layout(U, E, inter, trip)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32]))
    m.attach_graph(lay, DEV)
    g = m.graph()
    rp, col = g.A.rowptr_host, g.A.col_host
    rng = np.random.default_rng(3)
    for step in range(4):
        ids = [rng.integers(0, hi, 64) for hi in (U, U + E, U + E)]
        ids[1][:5] = ids[0][:5]  # repeated ids: marked more than once, listed once
        m(*[torch.from_numpy(i).to(DEV) for i in ids], mode=pkg.KGATMode.TRAIN_CF)
        tok = g._marked
        assert tok.cleared == kernels.PREMARKED
        hrows, _, hcount, bits1, bits0 = kernels.frontier_hop(g, tok.rows, precleared=tok.take_cleared())
        torch.cuda.synchronize()
        F = np.unique(np.concatenate(ids))
        want = np.unique(np.concatenate([F] + [col[rp[i]:rp[i + 1]] for i in F]))
        n = int(hcount.item())
        assert np.array_equal(hrows[:n].cpu().numpy(), want), step
        fb = np.unpackbits(bits0.cpu().numpy().view(np.uint8), bitorder="little")[:g.n_nodes]
        assert np.array_equal(np.flatnonzero(fb), F), step
        for t in g._hop_alt:
            assert int(t.count_nonzero()) == 0, step
        m.raise_pending(block=True)


@pytest.mark.parametrize("din,dout", [(64, 64), (64, 32), (128, 128)])
def test_biinter_row_set_forwards_match_whole_table(pkg, din, dout):
    """kgat_biinter_fwd_list_f32 (4-row quads of a row list: unsorted, a repeated row, two rows of one quad,
    -1 padding, the table's ragged last quad) and kgat_biinter_fwd_tiles_f32 (16-row tiles of a bitmap) against
    the whole-table forward: H, the norms and the state words of every row they cover are the same bits (train
    mode: dropout draws keyed by node), and nothing else is written.  128 -> 128 keeps two state words per lane."""
    _, kernels = _mods(pkg)
    n = 5003  # ragged last quad and tile
    g = torch.Generator().manual_seed(31)
    X, S = (torch.randn(n, din, generator=g).to(DEV) for _ in range(2))
    W1, W2 = (torch.randn(dout, din, generator=g).mul_(0.1).to(DEV) for _ in range(2))
    b1, b2 = (torch.randn(dout, generator=g).mul_(0.1).to(DEV) for _ in range(2))
    full = kernels.make_state(n, din, dout, X.device)
    Href = torch.empty(n, dout, device=DEV)
    kernels._lib.call("kgat_biinter_fwd_f32", X.data_ptr(), din, S.data_ptr(), din, W1.data_ptr(), b1.data_ptr(),
                      W2.data_ptr(), b2.data_ptr(), Href.data_ptr(), dout, n, din, dout, 0.1, ctypes.c_uint64(77),
                      full.norm.data_ptr(), full.mask.data_ptr(), kernels.stream_ptr(X.device))
    words = (dout + 63) // 64
    rows = np.array([4100, 17, 5002, 16, 17, 900, 903, 2, 4999, -1, 3000, -1], np.int32)  # (padding inside)
    listed = rows[rows >= 0]
    cover = np.unique(np.concatenate([(listed >> 2) * 4 + k for k in range(4)]))
    cover = cover[cover < n]

    def fresh():
        st = kernels.make_state(n, din, dout, X.device)
        st.norm.fill_(-7.0)
        st.mask.fill_(0x5A5A)
        return torch.full((n, dout), -9.0, device=DEV), st

    def check(H, st, rows_cov):
        r = torch.from_numpy(rows_cov.astype(np.int64)).to(DEV)
        assert torch.equal(H[r], Href[r]) and torch.equal(st.norm[r], full.norm[r])
        quads = np.unique(rows_cov >> 2)
        idx = []
        for qd in quads:
            for gi in range(words):
                base = ((qd >> 2) * words + gi) * 64 + (qd & 3) * 16
                idx.extend(range(base, base + 16))
        w = torch.tensor(idx, device=DEV)
        assert torch.equal(st.mask[w], full.mask[w])
        untouched = np.setdiff1d(np.arange(n), rows_cov)
        u = torch.from_numpy(untouched).to(DEV)
        assert bool((H[u] == -9.0).all()) and bool((st.norm[u] == -7.0).all())

    H, st = fresh()
    rt = torch.from_numpy(rows).to(DEV)
    kernels.biinter_fwd_list(X, S, W1, b1, W2, b2, 0.1, 77, H, rt, torch.tensor([rows.size], dtype=torch.int32,
                                                                                 device=DEV), state=st)
    check(H, st, cover)
    # a count short of the list: only the first 4 entries' quads
    H, st = fresh()
    kernels.biinter_fwd_list(X, S, W1, b1, W2, b2, 0.1, 77, H, rt, torch.tensor([4], dtype=torch.int32, device=DEV),
                             state=st)
    first = rows[:4]
    check(H, st, np.unique(np.concatenate([(first >> 2) * 4 + k for k in range(4)])).clip(max=n - 1))
    # the chunked tile forward on the same set's bitmap: whole 16-row tiles
    bits = np.zeros((n + 31) // 32, np.uint32)
    np.bitwise_or.at(bits, listed >> 5, np.uint32(1) << (listed & 31).astype(np.uint32))
    H, st = fresh()
    kernels.biinter_fwd_tiles(X, S, W1, b1, W2, b2, 0.1, 77, H, torch.from_numpy(bits.view(np.int32)).to(DEV),
                              state=st)
    tiles = np.unique(listed >> 4)
    tcov = np.concatenate([t * 16 + np.arange(16) for t in tiles])
    check(H, st, tcov[tcov < n])


@pytest.mark.parametrize("dim,layers", [(64, [64]), (64, [64, 32]), (64, [64, 64]), (64, [64, 32, 16]),
                                        (128, [128, 64, 32])])
def test_frontier_forward_bit_identical(pkg, dim, layers, monkeypatch):
    """KGAT.frontier_forward (TRAIN_CF's forward on the rows the loss can reach: layer 0 of 2 on
    the first hop F + N(F), the last layer on the batch rows F -- kgat_spmm_csr_rows_f32 +
    kgat_biinter_fwd_tiles_f32) against the full forward: losses, parameters and both Adam
    moments bit for bit over three train-mode CF steps (dropout on, fused table update on) with a
    KG step in between, on a hub-row graph; with 3 layers layer 0 stays whole and layers 1 / 2 run
    on the first hop / the batch rows (C4's shape 128 -> [128, 64, 32]: wide "bits" layers)."""
    graph_mod, _ = _mods(pkg)
    kmod = sys.modules[pkg.__name__ + ".kernels"]
    calls = {"rows": 0}
    real = kmod.spmm_rows

    def counted(*a, **k):
        calls["rows"] += 1
        return real(*a, **k)
    monkeypatch.setattr(kmod, "spmm_rows", counted)
    U, E, inter, trip = graph_mod.synthetic_ckg(20000, 200000, seed=9)
    lay = graph_mod.build_layout(U, E, inter, trip)
    models = []
    for frontier in (False, True):
        torch.manual_seed(77)
        m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=layers,
                                  cf_embedding_dim=dim, kg_embedding_dim=dim, message_dropout=[0.1] * len(layers)))
        m.attach_graph(lay, DEV)
        assert m.graph().A.n_long > 0  # hub rows take the segment + fix-up path
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        m.fuse_table_update = True
        m.frontier_forward = frontier
        models.append(m)
    rng = np.random.default_rng(11)
    R = len(lay.rel_order)
    for step in range(3):
        ids = [torch.from_numpy(rng.integers(0, hi, 96)).to(DEV) for hi in (U, int(E * 0.1), int(E * 0.1))]
        kg = [torch.from_numpy(rng.integers(0, hi, 32)).to(DEV) for hi in (U + E, R, U + E, U + E)]
        losses = []
        for m in models:
            torch.manual_seed(300 + step)  # same dropout seeds
            loss = m(*ids, mode=pkg.KGATMode.TRAIN_CF)
            loss.backward()
            losses.append(loss.detach().clone())
            m.update_cf_weights()
            m(kg[0], kg[1], kg[2], kg[3], mode=pkg.KGATMode.TRAIN_KG).backward()
            m.update_kg_weights()
        assert torch.equal(losses[0], losses[1]), (step, losses)
    assert calls["rows"] == 3 * min(len(layers), 2)  # the restricted layers of the three frontier steps
    a, b = models
    for (k, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        if not pa.is_sparse:
            assert torch.equal(pa, pb), k
    ta = a._cf_optimizer.state[id(a._user_entity_embedding.weight)]
    tb = b._cf_optimizer.state[id(b._user_entity_embedding.weight)]
    assert torch.equal(ta["exp_avg"], tb["exp_avg"]) and torch.equal(ta["exp_avg_sq"], tb["exp_avg_sq"])
    # a no-grad loss evaluation takes the full forward (no backward releases the batch-row map)
    with torch.no_grad():
        torch.manual_seed(5)
        la = a(*ids, mode=pkg.KGATMode.TRAIN_CF)
        torch.manual_seed(5)
        lb = b(*ids, mode=pkg.KGATMode.TRAIN_CF)
    assert torch.equal(la, lb)


def test_frontier_forward_dropped_and_overlapping_forwards(pkg):
    """The frontier forward leaves its batch-row marks and first hop for its own backward.  A dropped
    loss (forward without backward) is released by the next forward: the following steps equal the
    full-forward model's bit for bit.  Two forwards before a backward: the first one's backward raises
    instead of reading the second one's buffers."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(8000, 60000, seed=4)
    lay = graph_mod.build_layout(U, E, inter, trip)
    models = []
    for frontier in (False, True):
        torch.manual_seed(3)
        m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32],
                                  message_dropout=[0.1, 0.1]))
        m.attach_graph(lay, DEV)
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        m.fuse_table_update = True
        m.frontier_forward = frontier
        models.append(m)
    rng = np.random.default_rng(2)
    batches = [[torch.from_numpy(rng.integers(0, hi, 64)).to(DEV) for hi in (U, int(E * 0.1), int(E * 0.1))]
               for _ in range(3)]
    for m in models:
        torch.manual_seed(9)
        m(*batches[0], mode=pkg.KGATMode.TRAIN_CF)  # dropped: no backward
        for b in batches[1:]:
            m(*b, mode=pkg.KGATMode.TRAIN_CF).backward()
            m.update_cf_weights()
    a, b = models
    for (k, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        if not pa.is_sparse:
            assert torch.equal(pa, pb), k
    m = models[1]
    l1 = m(*batches[0], mode=pkg.KGATMode.TRAIN_CF)
    l2 = m(*batches[1], mode=pkg.KGATMode.TRAIN_CF)
    with pytest.raises(RuntimeError, match="reused the batch-row marks"):
        (l1 + l2).backward()
    # the model recovers: the next forward matches the full-forward model's and its backward runs
    m.zero_grad(set_to_none=True)
    m._table_update.pending = None  # whatever the failed backward left
    torch.manual_seed(1)
    la = models[0](*batches[2], mode=pkg.KGATMode.TRAIN_CF)
    torch.manual_seed(1)
    lb = models[1](*batches[2], mode=pkg.KGATMode.TRAIN_CF)
    assert torch.equal(la, lb)
    lb.backward()


def test_fused_table_update_materialises_on_demand(pkg):
    """A deferred table gradient (KGAT.fuse_table_update) meets the calls that need it: a second CF
    backward before the step (gradient accumulation) and an UPDATE_ATTENTION (which rewrites A's
    values) between backward and step.  Parameters after each sequence equal the unfused model's
    bit for bit."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(20000, 200000, seed=6)
    lay = graph_mod.build_layout(U, E, inter, trip)
    models = []
    for fused in (False, True):
        torch.manual_seed(2024)
        m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32],
                                  message_dropout=[0.1, 0.1]))
        m.attach_graph(lay, DEV)
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        m.fuse_table_update = fused
        models.append(m)
    rng = np.random.default_rng(9)
    att = [torch.from_numpy(np.asarray(x, np.int64)).to(DEV) for x in (lay.heads, lay.rels, lay.tails, lay.rel_order)]
    b1, b2 = ([torch.from_numpy(rng.integers(0, hi, 64)).to(DEV) for hi in (U, int(E * 0.1), int(E * 0.1))]
              for _ in range(2))
    for m in models:
        # accumulation: two backwards, one step
        torch.manual_seed(11)
        m(*b1, mode=pkg.KGATMode.TRAIN_CF).backward()
        m(*b2, mode=pkg.KGATMode.TRAIN_CF).backward()
        m.update_cf_weights()
        # an attention refresh between backward and step
        torch.manual_seed(12)
        m(*b1, mode=pkg.KGATMode.TRAIN_CF).backward()
        m.eval()
        m(*att, mode=pkg.KGATMode.UPDATE_ATTENTION)
        m.train()
        m.update_cf_weights()
    a, b = models
    for (k, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        if not pa.is_sparse:
            assert torch.equal(pa, pb), k
    assert torch.equal(a.attentive_matrix.data.coalesce().values(), b.attentive_matrix.data.coalesce().values())


def test_biinter_gemm_rows_matches_whole_table(pkg):
    """kgat_biinter_fwd_gemm_rows_f32 (the row-sharded frontier forward of a wide layer): the listed
    rows' H, pre-activation state and norm bit for bit the whole-table call's (same dropout draws);
    unlisted rows untouched."""
    _, kernels = _mods(pkg)
    din, dout, n = 256, 128, 4000 + 7
    g = torch.Generator().manual_seed(3)
    dv = [t.to(DEV) for t in (torch.randn(n, din, generator=g), torch.randn(n, din, generator=g),
                              torch.randn(dout, din, generator=g) * 0.1, torch.randn(dout, generator=g) * 0.1,
                              torch.randn(dout, din, generator=g) * 0.1, torch.randn(dout, generator=g) * 0.1)]
    st = kernels.BiState(n, DEV, din, dout, kind="gemm")
    H = kernels.biinter_fwd(*dv, dropout_p=0.1, seed=77, state=st)
    rows = np.sort(np.random.default_rng(4).choice(n, 333, replace=False))
    rws = torch.from_numpy(np.concatenate([rows, [-1, -1]]).astype(np.int32)).to(DEV)
    st2 = kernels.BiState(n, DEV, din, dout, kind="gemm")
    st2.P.fill_(7.0)
    H2 = torch.full((n, dout), 5.0, device=DEV)
    kernels.biinter_fwd_gemm_rows(dv[0], dv[1], rws, rws.numel(), *dv[2:], 0.1, 77, H2, st2)
    r = torch.from_numpy(rows).to(DEV)
    assert torch.equal(H2[r], H[r])
    for a, b in zip(st2.gemm_views(), st.gemm_views()):
        assert torch.equal(a[r], b[r])
    other = torch.ones(n, dtype=torch.bool, device=DEV)
    other[r] = False
    assert bool((H2[other] == 5.0).all()) and bool((st2.gemm_views()[0][other] == 7.0).all())


def test_csr_mark_rows_matches_numpy(pkg):
    """kgat_csr_mark_rows on a hub-row graph (long rows scanned by segments): row r flagged iff it is
    in the set or has an edge into it; with a row offset (a shard's rows)."""
    graph_mod, kernels = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(8000, 120000, seed=21)
    lay = graph_mod.build_layout(U, E, inter, trip)
    n = lay.n_nodes
    rng = np.random.default_rng(5)
    members = rng.choice(n, 40, replace=False)
    bits = np.zeros((n + 31) // 32 + 1, np.uint32)
    np.bitwise_or.at(bits, members >> 5, np.uint32(1) << (members & 31).astype(np.uint32))
    inset = np.zeros(n, bool)
    inset[members] = True
    rp, col = lay.rowptr, lay.col
    lo, hi = 1000, n - 500
    sh_rp = rp[lo:hi + 1] - rp[lo]
    sh_col = col[rp[lo]:rp[hi]]
    csr = graph_mod._DeviceCSR(sh_rp, np.ascontiguousarray(sh_col, np.int32),
                               torch.ones(sh_col.size, device=DEV), DEV)
    assert csr.n_long > 0
    hit = torch.full((hi - lo,), 9, dtype=torch.int32, device=DEV)
    kernels.csr_mark_rows(csr, torch.from_numpy(bits.view(np.int32)).to(DEV), n, lo, hit)
    rows = np.repeat(np.arange(hi - lo), np.diff(sh_rp))
    want = inset[lo:hi].copy()
    want[rows[inset[sh_col]]] = True
    np.testing.assert_array_equal(hit.cpu().numpy(), want.astype(np.int32))


@pytest.mark.parametrize("din,dout,kind", [(256, 256, "gemm"), (256, 128, "gemm"), (128, 128, "bits"),
                                           (128, 64, "bits")])
def test_biinter_bwd_rows_matches_gathered(pkg, din, dout, kind):
    """kgat_biinter_bwd_gemm_rows_f32 (the hop rows' wide backward read through the row list, dH by
    node) vs the gathered compact backward (X, S, H, state and dH gathered first): dXd, dS and every
    weight gradient bit for bit, with -1 padding rows and dropout."""
    _, kernels = _mods(pkg)
    n = 5000 + 11
    g = torch.Generator().manual_seed(din + dout)
    dv = [t.to(DEV) for t in (torch.randn(n, din, generator=g), torch.randn(n, din, generator=g),
                              torch.randn(dout, din, generator=g) * 0.1, torch.randn(dout, generator=g) * 0.1,
                              torch.randn(dout, din, generator=g) * 0.1, torch.randn(dout, generator=g) * 0.1)]
    rows_np = np.sort(np.random.default_rng(2).choice(n, 1500, replace=False))
    rows = torch.from_numpy(np.concatenate([rows_np, [-1] * 7]).astype(np.int32)).to(DEV)
    dHfull = torch.randn(n, dout, generator=g).to(DEV)
    outs = []
    for full in (False, True):
        st = kernels.BiState(n, DEV, din, dout, kind=kind)
        H = kernels.biinter_fwd(*dv, dropout_p=0.15, seed=21, state=st)
        dH = dHfull if full else kernels.gather_rows(dHfull, rows)
        outs.append(kernels.biinter_bwd(dv[0], dv[1], dH, *dv[2:], dropout_p=0.15, seed=21, rows=rows, H=H, state=st,
                                        dh_full=full))
    for i, (a, b) in enumerate(zip(*outs)):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("dim", [64, 128])
def test_lazy_kg_adam_bit_identical(pkg, dim):
    """KGAT.lazy_kg_adam (the KG step's table Adam on the batch rows only, the other rows' zero-gradient
    steps replayed when next read) vs the dense KG step: over KG phases of several steps between CF steps,
    a PREDICT in between, a step whose ids are out of range (skipped on the device) and a state_dict at
    the end, the parameters and both optimisers' moments are equal bit for bit."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(3000, 30000, seed=17)
    lay = graph_mod.build_layout(U, E, inter, trip)
    n = U + E
    R = len(lay.rel_order)
    models = []
    for lazy in (False, True):
        torch.manual_seed(3)
        m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=R, layer_size=[dim, 32],
                                  cf_embedding_dim=dim, kg_embedding_dim=dim))
        m.attach_graph(lay, DEV)
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        m.fuse_table_update = m.fuse_kg_table_update = True
        m.lazy_kg_adam = lazy
        models.append(m)
    rng = np.random.default_rng(4)
    for phase in range(4):
        ids = [torch.from_numpy(rng.integers(0, hi, 64)).to(DEV) for hi in (U, int(E * 0.2), int(E * 0.2))]
        kgs = [[torch.from_numpy(rng.integers(0, hi, 48)).to(DEV) for hi in (n, R, n, n)] for _ in range(6)]
        for m in models:
            torch.manual_seed(50 + phase)
            m(*ids, mode=pkg.KGATMode.TRAIN_CF).backward()
            if phase == 3:  # the device skip flag set while a CF step is in flight
                m._ids.skip_flag().fill_(1)
            m.update_cf_weights()
            m._ids.skip_flag().zero_()
            for j, kg in enumerate(kgs):
                if phase == 1 and j == 2:  # a device-side bad id: the step moves nothing
                    bad = kg[2].clone()
                    bad[0] = n + 7
                    m(kg[0], kg[1], bad, kg[3], mode=pkg.KGATMode.TRAIN_KG).backward()
                    torch.cuda.synchronize()  # the check's event has fired: the update reports it, abandons
                    with pytest.raises(IndexError):
                        m.update_kg_weights()
                    continue
                m(*kg, mode=pkg.KGATMode.TRAIN_KG).backward()
                if phase >= 2 and j in (1, 4):
                    # the skip flag set on the device while the step is in flight (the host has not seen it):
                    # the lazy path's history entry (skip = 1) and the dense step move nothing alike, and
                    # both advance Adam's step counter
                    m._ids.skip_flag().fill_(1)
                m.update_kg_weights()
                m._ids.skip_flag().zero_()
            if phase == 2:
                with torch.no_grad():
                    m(ids[0], ids[1], mode=pkg.KGATMode.PREDICT)
                # a second build_optimizer mid-training: the lazy replays still owed under the old
                # optimiser are applied first, and the new optimiser's steps restart every row at t = 0
                m.build_optimizer(cf_lr=1e-3, kg_lr=2e-4)
    sa, sb = models[0].state_dict(), models[1].state_dict()
    for k in sa:
        if not sa[k].is_sparse:
            assert torch.equal(sa[k], sb[k]), k
    for opt in ("_cf_optimizer", "_kg_optimizer"):
        oa, ob = getattr(models[0], opt), getattr(models[1], opt)
        for pa, pb in zip(oa.params, ob.params):
            sa_, sb_ = oa.state.get(id(pa)), ob.state.get(id(pb))
            assert (sa_ is None) == (sb_ is None), opt
            if sa_ is None:
                continue
            assert sa_["step"] == sb_["step"], opt
            assert torch.equal(sa_["exp_avg"], sb_["exp_avg"]) and torch.equal(sa_["exp_avg_sq"], sb_["exp_avg_sq"]), opt


@pytest.mark.parametrize("dim", [64, 128])
def test_captured_kg_step_bit_identical(pkg, dim):
    """KGAT.capture_kg_step (TRAIN_KG forward, backward and update_kg_weights each one replayed HIP graph,
    the step's scalars on the device) vs the eager lazy KG step: over KG phases between CF steps -- with a
    step whose ids are out of range, the skip flag set while a step is in flight, a dropped loss (forward
    without backward), two backwards before one update, a PREDICT and a second build_optimizer -- the
    losses, parameters and both optimisers' states are equal bit for bit, and the graphs did replay."""
    graph_mod, _ = _mods(pkg)
    U, E, inter, trip = graph_mod.synthetic_ckg(3000, 30000, seed=17)
    lay = graph_mod.build_layout(U, E, inter, trip)
    n = U + E
    R = len(lay.rel_order)
    models = []
    for cap in (False, True):
        torch.manual_seed(3)
        m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=R, layer_size=[dim, 32],
                                  cf_embedding_dim=dim, kg_embedding_dim=dim))
        m.attach_graph(lay, DEV)
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        m.fuse_table_update = m.fuse_kg_table_update = m.lazy_kg_adam = True
        m.direct_backward = True  # plain loss.backward() calls take the direct path (model._StepLoss)
        m.capture_kg_step = cap
        models.append(m)
    rng = np.random.default_rng(4)
    for phase in range(4):
        ids = [torch.from_numpy(rng.integers(0, hi, 64)).to(DEV) for hi in (U, int(E * 0.2), int(E * 0.2))]
        kgs = [[torch.from_numpy(rng.integers(0, hi, 48)).to(DEV) for hi in (n, R, n, n)] for _ in range(8)]
        losses = []
        for m in models:
            torch.manual_seed(50 + phase)
            m(*ids, mode=pkg.KGATMode.TRAIN_CF).backward()
            m.update_cf_weights()
            out = []
            for j, kg in enumerate(kgs):
                if phase == 1 and j == 2:  # a device-side bad id: the step moves nothing, the update raises
                    bad = kg[2].clone()
                    bad[0] = n + 7
                    m(kg[0], kg[1], bad, kg[3], mode=pkg.KGATMode.TRAIN_KG).backward()
                    torch.cuda.synchronize()
                    with pytest.raises(IndexError):
                        m.update_kg_weights()
                    continue
                if phase == 2 and j == 3:  # a dropped loss: its batch-row marks are released by the next forward
                    out.append(m(*kg, mode=pkg.KGATMode.TRAIN_KG).detach().clone())
                    continue
                loss = m(*kg, mode=pkg.KGATMode.TRAIN_KG)
                if j == 4:  # a scaled loss takes the autograd engine (upstream gradient 0.5)
                    (loss * 0.5).backward()
                else:  # the plain call: the captured step's direct backward (model._StepLoss)
                    loss.backward()
                if phase == 0 and j == 0:
                    with pytest.raises(RuntimeError):
                        loss.backward()  # a second backward of one loss raises, as the engine does
                if phase == 3 and j == 5:  # two backwards, one update (gradient accumulation)
                    kg2 = kgs[(j + 1) % len(kgs)]
                    m(*kg2, mode=pkg.KGATMode.TRAIN_KG).backward()
                if phase >= 2 and j in (1, 6):
                    m._ids.skip_flag().fill_(1)  # set on the device while the step is in flight
                m.update_kg_weights()
                m._ids.skip_flag().zero_()
                out.append(loss.detach().clone())
            losses.append(torch.stack(out))
            if phase == 2:
                with torch.no_grad():
                    m(ids[0], ids[1], mode=pkg.KGATMode.PREDICT)
                m.build_optimizer(cf_lr=1e-3, kg_lr=2e-4)
        assert torch.equal(losses[0], losses[1]), phase
    assert models[1]._kg_graph.replays >= 20 and models[0]._kg_graph.replays == 0
    sa, sb = models[0].state_dict(), models[1].state_dict()
    for k in sa:
        if not sa[k].is_sparse:
            assert torch.equal(sa[k], sb[k]), k
    for opt in ("_cf_optimizer", "_kg_optimizer"):
        oa, ob = getattr(models[0], opt), getattr(models[1], opt)
        for pa, pb in zip(oa.params, ob.params):
            sa_, sb_ = oa.state.get(id(pa)), ob.state.get(id(pb))
            assert (sa_ is None) == (sb_ is None), opt
            if sa_ is None:
                continue
            assert sa_["step"] == sb_["step"], opt
            assert torch.equal(sa_["exp_avg"], sb_["exp_avg"]) and torch.equal(sa_["exp_avg_sq"], sb_["exp_avg_sq"]), opt


def test_ids_check_multi_per_array_bounds(pkg):
    """kgat_ids_check_multi (the captured KG step's id check): four arrays, each against its own bound,
    copied concatenated into one int64 buffer; an id outside its array's bound is zeroed and raises both
    flags (pinned host + device skip flag), ids inside are copied exactly."""
    import ctypes
    import importlib
    lib = importlib.import_module(pkg.__name__ + "._lib")
    graph_mod = importlib.import_module(pkg.__name__ + ".graph")
    rng = np.random.default_rng(3)
    sizes, bounds = (100, 37, 1, 64), (50, 7, 1000, 3)
    arrs = [torch.from_numpy(rng.integers(0, b, n)).to(DEV) for n, b in zip(sizes, bounds)]

    def run(ts):
        d = lib.Ids()
        for k, t in enumerate(ts):
            d.ptr[k], d.n[k] = t.data_ptr(), t.numel()
        d.count = len(ts)
        bd = (ctypes.c_int64 * lib.KGAT_IDS_MAX)(*bounds)
        out = torch.full((sum(sizes),), -5, dtype=torch.int64, device=DEV)
        host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        dev_flag = torch.zeros(1, dtype=torch.int32, device=DEV)
        lib.call("kgat_ids_check_multi", ctypes.byref(d), bd, out.data_ptr(), host.data_ptr(), dev_flag.data_ptr(),
                 graph_mod.stream_ptr(torch.device(DEV)))
        torch.cuda.synchronize()
        return out, int(host[0]), int(dev_flag[0])

    out, h, dv = run(arrs)
    assert torch.equal(out, torch.cat(arrs)) and h == 0 and dv == 0
    bad = [a.clone() for a in arrs]
    bad[1][4] = 7   # == its bound
    bad[3][0] = -1
    out, h, dv = run(bad)
    want = torch.cat(bad)
    want[100 + 4] = 0
    want[100 + 37 + 1] = 0
    assert torch.equal(out, want) and h == 1 and dv == 1


def test_sched_adam_matches_eager(pkg):
    """The captured KG step's device-scheduled Adam (kgat_adam_multi_sched_f32: the step
    number on the device, step size and sqrt(1 - beta2^t) read from host-filled tables) against the eager
    kgat_adam_multi_ex_f32 with FusedAdam's scalars: parameters and moments equal bit for bit over six steps,
    one of them with the skip flag set."""
    import importlib
    import math
    lib = importlib.import_module(pkg.__name__ + "._lib")
    kernels = importlib.import_module(pkg.__name__ + ".kernels")
    graph_mod = importlib.import_module(pkg.__name__ + ".graph")
    torch.manual_seed(7)
    lr, b1, b2, eps = 1e-3, 0.9, 0.999, 1e-8
    shapes = [(3000, 64), (17, 64, 64)]
    ps = [torch.randn(s, device=DEV) for s in shapes]
    a_state = [(p.clone(), torch.zeros_like(p), torch.zeros_like(p)) for p in ps]
    b_state = [(p.clone(), torch.zeros_like(p), torch.zeros_like(p)) for p in ps]
    sz = torch.tensor([0.0] + [lr / (1.0 - b1 ** t) for t in range(1, 16)], dtype=torch.float32, device=DEV)
    bc = torch.tensor([0.0] + [math.sqrt(1.0 - b2 ** t) for t in range(1, 16)], dtype=torch.float32, device=DEV)
    t_dev = torch.zeros(1, dtype=torch.int32, device=DEV)
    t_next = torch.zeros(1, dtype=torch.int32, device=DEV)
    skip = torch.zeros(1, dtype=torch.int32, device=DEV)
    st = graph_mod.stream_ptr(torch.device(DEV))
    for t in range(1, 7):
        grads = [torch.randn(s, device=DEV) for s in shapes]
        skip.fill_(1 if t == 4 else 0)
        kernels.adam_multi([(p, g, m, v, lr / (1.0 - b1 ** t), math.sqrt(1.0 - b2 ** t))
                            for (p, m, v), g in zip(a_state, grads)], b1, b2, eps, skip)
        arr = (lib.AdamTensor * len(shapes))()
        for a, (p, m, v), g in zip(arr, b_state, grads):
            a.p, a.g, a.m, a.v = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
            a.n, a.step_size, a.bc2_sqrt = p.numel(), 0.0, 0.0
        if t % 2:  # t advanced beforehand, applied as read (t_add 0, no hand-on)
            t_dev.add_(1)
            lib.call("kgat_adam_multi_sched_f32", arr, len(shapes), b1, b2, eps, skip.data_ptr(), t_dev.data_ptr(),
                     sz.data_ptr(), bc.data_ptr(), 0, None, st)
        else:  # the captured update's form: step *t + 1 applied, its number handed on in a second cell
            # (the kernel reads one cell and writes the other), then copied back for the next step
            lib.call("kgat_adam_multi_sched_f32", arr, len(shapes), b1, b2, eps, skip.data_ptr(), t_dev.data_ptr(),
                     sz.data_ptr(), bc.data_ptr(), 1, t_next.data_ptr(), st)
            t_dev.copy_(t_next)
    torch.cuda.synchronize()
    assert int(t_dev[0]) == 6
    for x, y in zip(a_state, b_state):
        for u, w in zip(x, y):
            assert torch.equal(u, w)
