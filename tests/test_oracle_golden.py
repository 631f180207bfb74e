"""Pin the CPU oracle to the reference: every oracle function vs the golden vectors.

The golden vectors were produced by the reference classes themselves
(tests/golden/make_golden.py).  These tests run on CPU (no GPU marker).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import kgat_cpu as K
from tests.conftest import golden

RTOL, ATOL = 1e-4, 1e-5


def params_from(g: dict, prefix: str = "init/") -> dict[str, torch.Tensor]:
    return {k[len(prefix):]: torch.from_numpy(v.copy()) for k, v in g.items() if k.startswith(prefix)}


def oracle_graph(g):
    U = int(g["user_num"])
    n = U + int(g["entity_num"])
    blocks, rel_ids = K.adjacency_blocks(U, [0, 1, 2, 3], g["interactions"], g["triplets"])
    lap = K.normalized_blocks(n, blocks)
    return n, rel_ids, lap


def test_graph_layout(kgat_case):
    _, g = kgat_case
    n, rel_ids, lap = oracle_graph(g)
    assert rel_ids == g["adjacency_relations"].tolist()
    heads, rels, tails, vals = K.kg_edge_arrays(lap, rel_ids)
    np.testing.assert_array_equal(heads, g["kg_heads"])
    np.testing.assert_array_equal(rels, g["kg_rels"])
    np.testing.assert_array_equal(tails, g["kg_tails"])
    np.testing.assert_allclose(vals, g["kg_vals"], rtol=1e-6)
    A = K.initial_attentive(n, lap)
    np.testing.assert_array_equal(A.indices().numpy(), g["A_idx"])
    np.testing.assert_allclose(A.values().numpy(), g["A_val"], rtol=1e-6)


def _A(g, n):
    return torch.sparse_coo_tensor(torch.from_numpy(g["A_idx"]), torch.from_numpy(g["A_val"]), (n, n)).coalesce()


def test_propagation(kgat_case):
    _, g = kgat_case
    n = int(g["user_num"]) + int(g["entity_num"])
    P = params_from(g)
    outs = K.propagate(P, _A(g, n))
    np.testing.assert_allclose(torch.cat(outs, 1).numpy(), g["all_emb"], rtol=RTOL, atol=ATOL)


def test_cf_steps_and_adam(kgat_case):
    _, g = kgat_case
    n = int(g["user_num"]) + int(g["entity_num"])
    A = _A(g, n)
    P = params_from(g)
    opt = K.AdamOracle(lr=1e-3)
    s = 0
    while f"cf{s}/loss" in g:
        leaves = {k: v.clone().requires_grad_(True) for k, v in P.items()}
        loss = K.cf_loss(torch.cat(K.propagate(leaves, A), 1), torch.from_numpy(g[f"cf{s}/users"]),
                         torch.from_numpy(g[f"cf{s}/pos"]), torch.from_numpy(g[f"cf{s}/neg"]))
        loss.backward()
        np.testing.assert_allclose(loss.item(), g[f"cf{s}/loss"], rtol=1e-5)
        grads = {}
        for k, v in leaves.items():
            ref = g.get(f"cf{s}/grad/{k}")
            if ref is None:
                assert v.grad is None or not v.grad.any(), k
                grads[k] = None
            else:
                np.testing.assert_allclose(v.grad.numpy(), ref, rtol=RTOL, atol=1e-6, err_msg=k)
                grads[k] = v.grad.detach()
        opt.step(P, grads)
        s += 1
    for k, v in g.items():
        if k.startswith("after_cf/"):
            np.testing.assert_allclose(P[k[9:]].numpy(), v, rtol=RTOL, atol=1e-6, err_msg=k)


def test_kg_steps_and_adam(kgat_case):
    _, g = kgat_case
    P = params_from(g)
    P.update(params_from(g, "after_cf/"))
    opt = K.AdamOracle(lr=1e-4)
    s = 0
    while f"kg{s}/loss" in g:
        leaves = {k: v.clone().requires_grad_(True) for k, v in P.items()}
        loss = K.transr_loss(leaves, *(torch.from_numpy(g[f"kg{s}/{x}"]) for x in ("heads", "rels", "pos", "neg")))
        loss.backward()
        np.testing.assert_allclose(loss.item(), g[f"kg{s}/loss"], rtol=1e-5)
        grads = {}
        for k, v in leaves.items():
            ref = g.get(f"kg{s}/grad/{k}")
            grads[k] = None if ref is None else v.grad.detach()
            if ref is not None:
                np.testing.assert_allclose(v.grad.numpy(), ref, rtol=RTOL, atol=1e-6, err_msg=k)
        opt.step(P, grads)
        s += 1
    for k, v in g.items():
        if k.startswith("after_kg/"):
            np.testing.assert_allclose(P[k[9:]].numpy(), v, rtol=RTOL, atol=1e-6, err_msg=k)


def _final_params(g):
    P = params_from(g)
    P.update(params_from(g, "after_cf/"))
    P.update(params_from(g, "after_kg/"))
    return P


def test_attention_refresh(kgat_case):
    _, g = kgat_case
    n = int(g["user_num"]) + int(g["entity_num"])
    P = _final_params(g)
    att = K.refresh_attention(P, *(torch.from_numpy(g[x]) for x in ("kg_heads", "kg_rels", "kg_tails")),
                              g["adjacency_relations"], n)
    np.testing.assert_array_equal(att.indices().numpy(), g["att_idx"])
    np.testing.assert_allclose(att.values().numpy(), g["att_val"], rtol=RTOL, atol=1e-6)


def test_predict_and_metrics(kgat_case):
    _, g = kgat_case
    n = int(g["user_num"]) + int(g["entity_num"])
    P = _final_params(g)
    att = torch.sparse_coo_tensor(torch.from_numpy(g["att_idx"]), torch.from_numpy(g["att_val"]), (n, n))
    all_emb = torch.cat(K.propagate(P, att.coalesce()), 1)
    users = torch.from_numpy(g["eval_users"])
    sc = K.scores(all_emb, users, torch.arange(int(g["item_num"])))
    np.testing.assert_allclose(sc.numpy(), g["scores"], rtol=RTOL, atol=1e-5)
    train, test = {}, {}
    for u, i in g["train_flat"]:
        train.setdefault(int(u), []).append(int(i))
    for u, i in g["test_flat"]:
        test.setdefault(int(u), []).append(int(i))
    ref_scores = torch.from_numpy(g["scores"].copy())
    _, met = K.ranking_metrics(ref_scores, train, test, g["eval_users"], [20, 40])
    for k in (20, 40):
        for m in ("precision", "recall", "ndcg"):
            np.testing.assert_allclose(met[k][m], g[f"metrics/{k}/{m}"], rtol=1e-6)


def test_nfm():
    g = golden("nfm_h3_d64")
    U = int(g["user_num"])
    F = U + int(g["entity_num"])
    I = int(g["item_num"])
    feat = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([g["feat_row"], g["feat_col"]])),
                                   torch.from_numpy(g["feat_val"]), (I, int(g["entity_num"]))).to_dense()

    def batch(users, items):
        x = torch.zeros(len(users), F)
        x[torch.arange(len(users)), torch.from_numpy(users)] = 1.0
        x[:, U:] = feat[torch.from_numpy(items)]
        return x.to_sparse()

    P = params_from(g)
    opt = K.AdamOracle(lr=1e-4)
    for s in range(2):
        leaves = {k: v.clone().requires_grad_(True) for k, v in P.items()}
        xp = batch(g[f"tr{s}/users"], g[f"tr{s}/pos"])
        xn = batch(g[f"tr{s}/users"], g[f"tr{s}/neg"])
        loss = K.nfm_loss(leaves, xp, xn)
        loss.backward()
        np.testing.assert_allclose(loss.item(), g[f"tr{s}/loss"], rtol=1e-5)
        grads = {}
        for k, v in leaves.items():
            ref = g.get(f"tr{s}/grad/{k}")
            grads[k] = None if ref is None else v.grad.detach()
            if ref is not None:
                np.testing.assert_allclose(v.grad.numpy(), ref, rtol=RTOL, atol=1e-6, err_msg=k)
        opt.step(P, grads)
    for k, v in g.items():
        if k.startswith("after/"):
            np.testing.assert_allclose(P[k[6:]].numpy(), v, rtol=RTOL, atol=1e-6, err_msg=k)
    users = g["pred_users"]
    x = batch(np.repeat(users, I), np.tile(np.arange(I), len(users)))
    np.testing.assert_allclose(K.nfm_score(P, x).detach().numpy(), g["pred_scores"], rtol=RTOL, atol=1e-5)


def test_c1_sm_shaped_pipeline():
    """C1 scale (BASELINE configs[0] shape: 500 users, 9.5k problems, 1.18M nnz, 1 layer, d=64): two CF
    steps + Adam, the attention refresh on all 1.18M edges, PREDICT and the top-20 / P/R/nDCG@20 of
    every eval user -- against the reference's own run (tests/golden/make_golden.py --c1)."""
    from tests.conftest import assert_metrics_with_ties, assert_topk_with_ties, c1_inputs, load_pkg

    g = golden("kgat_C1_sm")
    U, E, inter, trip, train, test, eval_users = c1_inputs(g)
    n = U + E
    blocks, rel_ids = K.adjacency_blocks(U, [0, 1, 2, 3], inter, trip)
    lap = K.normalized_blocks(n, blocks)
    A = K.initial_attentive(n, lap)
    assert A._nnz() == int(g["nnz"])
    heads, rels, tails, _ = K.kg_edge_arrays(lap, rel_ids)
    pkg = load_pkg()  # the drop-in module creates its parameters in the reference's RNG order (CPU only)
    torch.manual_seed(2024)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(rel_ids), layer_size=[64],
                              message_dropout=[0.1]))
    P = {k: v.detach().clone() for k, v in m.state_dict().items() if not v.is_sparse}
    opt = K.AdamOracle(lr=1e-3)
    for s in range(2):
        cf = {k: v.clone().requires_grad_(True) for k, v in P.items()
              if k == K.EMB or k.startswith("_aggregator")}
        loss = K.cf_loss(torch.cat(K.propagate(cf, A), 1),
                         *(torch.from_numpy(g[f"cf{s}/{x}"]) for x in ("users", "pos", "neg")))
        loss.backward()
        np.testing.assert_allclose(loss.item(), g[f"cf{s}/loss"], rtol=1e-5)
        opt.step(P, {k: v.grad.detach() for k, v in cf.items()})
    att = K.refresh_attention(P, torch.from_numpy(heads), torch.from_numpy(rels), torch.from_numpy(tails),
                              rel_ids, n)
    emb = torch.cat(K.propagate(P, att), 1)
    sc = K.scores(emb, torch.from_numpy(eval_users), torch.arange(int(g["item_num"])))
    masked = sc.clone()
    for r, u in enumerate(eval_users):
        masked[r, train[int(u)]] = -np.inf
    top = torch.topk(masked, k=20, dim=1).indices.numpy()
    assert_topk_with_ties(top, g["topk20"], g["top21_scores"])
    _, met = K.ranking_metrics(sc, train, test, eval_users, [20])
    assert_metrics_with_ties(met[20], g, 20, g["top21_scores"])
    assert float(np.mean(met[20]["recall"])) == pytest.approx(float(g["recall20_mean"]), abs=1e-9)
