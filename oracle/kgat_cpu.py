"""CPU restatement of the reference KGAT + NFM hot path (PyTorch-CPU, fp32).

TEST INFRASTRUCTURE ONLY -- this is the checker, never the product.  It is
imported by ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg and by nothing else.  The product path lives in
``problem-recommender-system-using-kgat-in-codeforces_amd/`` and fails loudly
when its HIP library is missing.

Parity pin: ``tests/test_oracle_golden.py`` checks every function here against
golden vectors produced by the reference classes themselves
(``tests/golden/make_golden.py``), so the restatement is pinned, not trusted.

The restatement is written as free functions over a flat parameter dict whose
keys are the reference ``state_dict`` keys.  Each function cites the reference
lines whose arithmetic it restates (paths relative to the reference root).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn.functional as F

LEAKY_SLOPE = 0.01  # nn.LeakyReLU() default, src/model/KGAT/aggregator.py:23
NORM_EPS = 1e-12  # F.normalize default, src/model/KGAT/aggregator.py:65
LN_EPS = 1e-5  # nn.LayerNorm default, src/model/KGAT/multi_head_attention.py:17

EMB = "_user_entity_embedding.weight"
REL = "_relation_embedding.weight"
TRANS = "_trans_matrix"


# --------------------------------------------------------------------------
# a12: input layout producer (src/model/KGAT/preprocess.py:157-246, 268-326, 628-634)
# --------------------------------------------------------------------------
def adjacency_blocks(user_num: int, kg_relation_ids: list[int], interactions: np.ndarray,
                     triplets: np.ndarray) -> tuple[list[tuple[np.ndarray, np.ndarray]], list[int]]:
    """Directed (head, tail) lists per adjacency relation, in reference order.

    Follows preprocess.py:177-222: the interaction block (user -> U+problem),
    its inverse, then for every KG relation r (in RelationType order) the
    block (U+h -> U+t) with id r+1 and its inverse with id r+2+R.
    ``triplets`` is an int array [T, 3] of (head, relation, tail) entity ids.
    """
    R = len(kg_relation_ids)
    blocks, rel_ids = [], []
    h = interactions[:, 0].astype(np.int64)
    t = interactions[:, 1].astype(np.int64) + user_num
    blocks += [(h, t), (t, h)]
    rel_ids += [0, R + 1]
    for r in kg_relation_ids:
        sel = triplets[:, 1] == r
        hh = triplets[sel, 0].astype(np.int64) + user_num
        tt = triplets[sel, 2].astype(np.int64) + user_num
        blocks += [(hh, tt), (tt, hh)]
        rel_ids += [r + 1, r + 2 + R]
    return blocks, rel_ids


def normalized_blocks(n_nodes: int, blocks) -> list[sp.coo_matrix]:
    """``(D^-1/2 A)^T D^-1/2`` per block, i.e. entry (t, h) = count(h,t)/outdeg(h).

    preprocess.py:224-246.  Built here directly as the transposed random-walk
    matrix (same fp64 values; duplicates summed as scipy does).
    """
    out = []
    for h, t in blocks:
        a = sp.coo_matrix((np.ones(len(h)), (h, t)), shape=(n_nodes, n_nodes)).tocsr()
        a.sum_duplicates()
        deg = np.asarray(a.sum(axis=1)).ravel()
        inv = np.zeros_like(deg)
        nz = deg > 0
        inv[nz] = 1.0 / deg[nz]
        out.append((sp.diags(inv) @ a).T.tocoo())
    return out


def kg_edge_arrays(lap_blocks: list[sp.coo_matrix], rel_ids: list[int]):
    """Flattened edge arrays sorted by head, then tail (preprocess.py:268-326).

    Returns heads, relation ids, tails (int64) and fp32 values.  Ties (the
    same (head, tail) in two relations) keep block order (stable sort).
    """
    heads = np.concatenate([b.row.astype(np.int64) for b in lap_blocks])
    tails = np.concatenate([b.col.astype(np.int64) for b in lap_blocks])
    rels = np.concatenate([np.full(b.nnz, r, np.int64) for b, r in zip(lap_blocks, rel_ids)])
    vals = np.concatenate([b.data for b in lap_blocks]).astype(np.float32)
    order = np.lexsort((tails, heads))  # primary head, secondary tail; stable
    return heads[order], rels[order], tails[order], vals[order]


def initial_attentive(n_nodes: int, lap_blocks: list[sp.coo_matrix]) -> torch.Tensor:
    """Sum of the normalized blocks as a coalesced fp32 COO (preprocess.py:628-634)."""
    total = lap_blocks[0].tocsr()
    for b in lap_blocks[1:]:
        total = total + b.tocsr()
    total = total.tocoo()
    idx = torch.from_numpy(np.vstack((total.row, total.col)).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(total.data.astype(np.float32)),
                                   (n_nodes, n_nodes)).coalesce()


# --------------------------------------------------------------------------
# a1/a2: attentive propagation (aggregator.py:37-65, model.py:124-140)
# --------------------------------------------------------------------------
def bi_interaction_layer(ego: torch.Tensor, A: torch.Tensor, w1, b1, w2, b2,
                         dropout_p: float = 0.0, generator: torch.Generator | None = None) -> torch.Tensor:
    side = torch.sparse.mm(A, ego)                       # aggregator.py:54
    pre_sum = F.linear(ego + side, w1, b1)               # aggregator.py:57
    pre_mul = F.linear(ego * side, w2, b2)               # aggregator.py:58
    h = F.leaky_relu(pre_sum, LEAKY_SLOPE) + F.leaky_relu(pre_mul, LEAKY_SLOPE)
    if dropout_p > 0.0:                                  # aggregator.py:62 (train mode)
        keep = (torch.rand(h.shape, generator=generator) >= dropout_p).to(h.dtype)
        h = h * keep / (1.0 - dropout_p)
    return h / h.norm(dim=1, keepdim=True).clamp_min(NORM_EPS)   # aggregator.py:65


def layer_count(params: dict) -> int:
    return len([k for k in params if k.startswith("_aggregator_layers.") and k.endswith("linear1.weight")])


def propagate(params: dict, A: torch.Tensor, dropout: list[float] | None = None,
              generator: torch.Generator | None = None) -> list[torch.Tensor]:
    """[X0, H1, ..., HL]; the reference concatenates them along dim 1 (model.py:140)."""
    outs = [params[EMB]]
    for l in range(layer_count(params)):
        p = f"_aggregator_layers.{l}."
        outs.append(bi_interaction_layer(
            outs[-1], A, params[p + "linear1.weight"], params[p + "linear1.bias"],
            params[p + "linear2.weight"], params[p + "linear2.bias"],
            0.0 if dropout is None else dropout[l], generator))
    return outs


# --------------------------------------------------------------------------
# a3/a4: CF BPR loss (model.py:142-202)
# --------------------------------------------------------------------------
def half_sq_mean(x: torch.Tensor) -> torch.Tensor:
    """mean over rows of sum(x^2)/2 (model.py:142-163)."""
    return (x * x).sum(dim=1).div(2.0).mean()


def cf_loss(all_emb: torch.Tensor, users, pos, neg, reg: float = 1e-5) -> torch.Tensor:
    # item ids index the user+entity table raw, NOT offset by user_num (model.py:189-191)
    u, p, n = all_emb[users.long()], all_emb[pos.long()], all_emb[neg.long()]
    margin = (u * p).sum(1) - (u * n).sum(1)
    return -F.logsigmoid(margin).mean() + reg * (half_sq_mean(u) + half_sq_mean(p) + half_sq_mean(n))


# --------------------------------------------------------------------------
# a5: TransR KG loss (model.py:204-261)
# --------------------------------------------------------------------------
def transr_loss(params: dict, heads, rels, pos_tails, neg_tails, reg: float = 1e-5) -> torch.Tensor:
    rels = rels.long()
    W = params[TRANS][rels]                                   # [B, d, k]
    e_r = params[REL][rels]                                   # [B, k]
    proj = lambda ids: torch.bmm(params[EMB][ids.long()].unsqueeze(1), W).squeeze(1)  # noqa: E731
    h, tp, tn = proj(heads), proj(pos_tails), proj(neg_tails)
    s_pos = (h + e_r - tp).pow(2).sum(1)
    s_neg = (h + e_r - tn).pow(2).sum(1)
    base = -F.logsigmoid(s_neg - s_pos).mean()
    return base + reg * (half_sq_mean(h) + half_sq_mean(e_r) + half_sq_mean(tp) + half_sq_mean(tn))


# --------------------------------------------------------------------------
# a6/a7: knowledge-aware attention refresh (model.py:263-366, multi_head_attention.py:35-58)
# --------------------------------------------------------------------------
def value_path(params: dict, t_proj: torch.Tensor) -> torch.Tensor:
    """The MHA output for a length-1 sequence.

    softmax over the size-1 key axis is exactly 1.0 (multi_head_attention.py:51-52),
    so query/key are dead and the output is LN(W_o(W_v t + b_v) + b_o).  The
    golden fixtures check this against the reference's full MHA.
    """
    m = "_multi_head_attention."
    v = F.linear(t_proj, params[m + "_value_weight.weight"], params[m + "_value_weight.bias"])
    o = F.linear(v, params[m + "_output.weight"], params[m + "_output.bias"])
    return F.layer_norm(o, (o.shape[-1],), params[m + "_layer_norm.weight"],
                        params[m + "_layer_norm.bias"], LN_EPS)


def edge_logits(params: dict, heads, tails, rel: int, n_nodes: int) -> torch.Tensor:
    """Un-normalised attention for the edges of ONE adjacency relation (model.py:263-316)."""
    t_proj = params[EMB][tails.long()] @ params[TRANS][rel]
    score = torch.tanh(value_path(params, t_proj)).sum(dim=1)
    # degrees are counted within this relation only (model.py:309-314)
    dh = torch.bincount(heads.long(), minlength=n_nodes)
    dt = torch.bincount(tails.long(), minlength=n_nodes)
    w = 1.0 / (torch.log1p(dh[heads.long()]) + torch.log1p(dt[tails.long()]))
    return score * w


def refresh_attention(params: dict, heads, rels, tails, rel_order, n_nodes: int) -> torch.Tensor:
    """New attentive matrix = row softmax over stored entries (model.py:318-366)."""
    rows, cols, vals = [], [], []
    for r in [int(x) for x in rel_order]:
        sel = rels == r
        h, t = heads[sel], tails[sel]
        rows.append(h.long())
        cols.append(t.long())
        vals.append(edge_logits(params, h, t, r, n_nodes))
    coo = torch.sparse_coo_tensor(torch.stack([torch.cat(rows), torch.cat(cols)]),
                                  torch.cat(vals), (n_nodes, n_nodes))
    return torch.sparse.softmax(coo.coalesce(), dim=1).coalesce()


# --------------------------------------------------------------------------
# a8: scoring + ranking metrics (model.py:368-391, metrics_calculator.py:84-131)
# --------------------------------------------------------------------------
def scores(all_emb: torch.Tensor, users, items) -> torch.Tensor:
    return all_emb[users.long()] @ all_emb[items.long()].T


def ranking_metrics(score: torch.Tensor, train: dict, test: dict, users: np.ndarray, ks: list[int]):
    """Precision/recall/nDCG@k after masking train items to -inf (metrics_calculator.py:84-131)."""
    score = score.clone()
    truth = np.zeros(score.shape, dtype=np.float32)
    for i, u in enumerate(users):
        score[i, list(train[int(u)])] = -math.inf
        truth[i, list(test[int(u)])] = 1.0
    order = torch.sort(score, dim=1, descending=True).indices.numpy()
    hits = np.take_along_axis(truth, order, axis=1)
    out = {}
    for k in ks:
        disc = 1.0 / np.log2(np.arange(2, k + 2))
        dcg = ((2.0 ** hits[:, :k] - 1) * disc).sum(1)
        ideal = np.flip(np.sort(hits, axis=1), axis=1)[:, :k]
        idcg = ((2.0 ** ideal - 1) * disc).sum(1)
        idcg[idcg == 0] = np.inf
        out[k] = {"precision": hits[:, :k].mean(1), "recall": hits[:, :k].sum(1) / hits.sum(1),
                  "ndcg": dcg / idcg}
    return order, out


# --------------------------------------------------------------------------
# a9: Adam, two independent instances (model.py:393-419)
# --------------------------------------------------------------------------
@dataclass
class AdamOracle:
    """torch.optim.Adam(lr, betas=(0.9, 0.999), eps=1e-8) restated per tensor."""

    lr: float
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    state: dict = field(default_factory=dict)

    def step(self, params: dict, grads: dict) -> None:
        for name, g in grads.items():
            if g is None:        # zero_grad(set_to_none) => param skipped
                continue
            m, v, t = self.state.get(name, (torch.zeros_like(g), torch.zeros_like(g), 0))
            t += 1
            m = m + (1.0 - self.beta1) * (g - m)
            v = v * self.beta2 + (1.0 - self.beta2) * g * g
            c1 = 1.0 - self.beta1 ** t
            c2s = math.sqrt(1.0 - self.beta2 ** t)
            params[name] = params[name] - (self.lr / c1) * m / (v.sqrt() / c2s + self.eps)
            self.state[name] = (m, v, t)


# --------------------------------------------------------------------------
# a10/a11: NFM (src/model/NFM/model.py:73-129, hidden_layer.py:31-35)
# --------------------------------------------------------------------------
def nfm_feature_matrix(item_num: int, entity_num: int, feature_heads, feature_tails) -> sp.csr_matrix:
    """Item one-hots plus the tails of problem-headed triplets, duplicates summed
    (src/model/NFM/preprocess.py:166-183: coo_matrix(...).tocsr())."""
    rows = list(range(item_num)) + [int(h) for h in feature_heads]
    cols = list(range(item_num)) + [int(t) for t in feature_tails]
    return sp.coo_matrix(([1] * len(rows), (rows, cols)), shape=(item_num, entity_num)).tocsr()


def nfm_train_feature_batch(user_num: int, feature: sp.csr_matrix, users, items) -> torch.Tensor:
    """sp.hstack([user one-hots, feature rows]) as a torch COO (NFM/preprocess.py:284-307, 336-356)."""
    user_matrix = sp.identity(user_num).tocsr()
    coo = sp.hstack([user_matrix[np.asarray(users)], feature[np.asarray(items)]]).tocoo()
    return torch.sparse_coo_tensor(torch.LongTensor(np.vstack((coo.row, coo.col))), torch.FloatTensor(coo.data),
                                   torch.Size(coo.shape))


def nfm_test_feature_batch(user_num: int, feature: sp.csr_matrix, batch_user_ids) -> torch.Tensor:
    """Users x all items (NFM/preprocess.py:309-334)."""
    item_num = feature.shape[0]
    row_num = len(batch_user_ids) * item_num
    user_cols = np.repeat(np.asarray(batch_user_ids), item_num)
    um = sp.coo_matrix(([1] * row_num, (list(range(row_num)), user_cols)), shape=(row_num, user_num)).tocsr()
    coo = sp.hstack([um, sp.vstack([feature] * len(batch_user_ids))]).tocoo()
    return torch.sparse_coo_tensor(torch.LongTensor(np.vstack((coo.row, coo.col))), torch.FloatTensor(coo.data),
                                   torch.Size(coo.shape))


def nfm_score(params: dict, x: torch.Tensor) -> torch.Tensor:
    V = params["_feature_embedding"]
    xv = torch.sparse.mm(x, V)
    x2v2 = torch.sparse.mm(x * x, V * V)
    z = 0.5 * (xv * xv - x2v2)
    l = 0
    while f"_hidden_layers.{l}._linear.weight" in params:
        p = f"_hidden_layers.{l}._linear."
        z = F.relu(F.linear(z, params[p + "weight"], params[p + "bias"]))
        l += 1
    y = z @ params["_output_layer.weight"].T
    wide = torch.sparse.mm(x, params["_linear.weight"].T) + params["_linear.bias"]
    return (wide + y).squeeze()


def nfm_loss(params: dict, x_pos, x_neg, lam: float = 1e-5) -> torch.Tensor:
    diff = nfm_score(params, x_pos) - nfm_score(params, x_neg)
    w = params["_output_layer.weight"]
    return -torch.log(1e-10 + torch.sigmoid(diff)).mean() + lam * w.norm(2).pow(2) / 2
