"""Host samplers (csrc/sampler.cpp via sampler.BatchSampler) against the reference's sampling rules
(src/model/KGAT/preprocess.py:328-525).  The reference's rng is unseeded, so the checks are the
rules themselves plus the distributions, not draw-by-draw equality."""
from __future__ import annotations

import numpy as np
import pytest

from tests.conftest import golden, load_pkg

pkg = load_pkg()
sampler = __import__(pkg.__name__ + ".sampler", fromlist=["sampler"])
graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])


def _case():
    g = golden("kgat_L2_d64")
    U, E = int(g["user_num"]), int(g["entity_num"])
    lay = graph.build_layout(U, E, g["interactions"], g["triplets"])
    inter = {}
    for u, i in g["interactions"]:
        inter.setdefault(int(u), []).append(int(i))
    return g, U, E, lay, inter


def test_cf_batch_rules_and_determinism():
    g, U, E, lay, inter = _case()
    I = int(g["item_num"])
    s = sampler.BatchSampler(inter, I, lay.heads, lay.rels, lay.tails, lay.n_nodes, cf_batch_size=64, seed=7)
    for _ in range(20):
        u, p, n = (t.numpy() for t in s.generate_cf_batch())
        assert len(set(u.tolist())) == u.size  # without replacement (64 <= users)
        for a, b, c in zip(u, p, n):
            assert b in inter[int(a)] and c not in inter[int(a)] and 0 <= c < I
    a = sampler.BatchSampler(inter, I, lay.heads, lay.rels, lay.tails, lay.n_nodes, cf_batch_size=64, seed=7)
    b = sampler.BatchSampler(inter, I, lay.heads, lay.rels, lay.tails, lay.n_nodes, cf_batch_size=64, seed=7)
    for _ in range(3):
        for x, y in zip(a.generate_cf_batch(), b.generate_cf_batch()):
            assert np.array_equal(x.numpy(), y.numpy())
    # batch larger than the user population: with replacement (preprocess.py:399-402)
    big = sampler.BatchSampler(inter, I, lay.heads, lay.rels, lay.tails, lay.n_nodes, cf_batch_size=5 * len(inter))
    u, _, _ = big.generate_cf_batch()
    assert u.numel() == 5 * len(inter) and len(set(u.tolist())) < u.numel()


def test_cf_distributions_uniform():
    items = list(range(0, 40, 2))  # one user, 20 positives among 40 items
    s = sampler.BatchSampler({3: items}, 40, np.array([0]), np.array([0]), np.array([1]), 50, cf_batch_size=1,
                             seed=1)
    pos, neg = [], []
    for _ in range(8000):
        _, p, n = s.generate_cf_batch()
        pos.append(int(p))
        neg.append(int(n))
    cp = np.bincount(pos, minlength=40)[items]
    cn = np.bincount(neg, minlength=40)[[i for i in range(40) if i not in items]]
    for c in (cp, cn):  # 400 expected per bin; chi-square with 19 dof, far tail
        chi2 = ((c - c.mean()) ** 2 / c.mean()).sum()
        assert chi2 < 50, chi2


def test_kg_batch_rules():
    g, U, E, lay, inter = _case()
    edges = {}
    for h, r, t in zip(lay.heads, lay.rels, lay.tails):
        edges.setdefault(int(h), set()).add((int(r), int(t)))
    s = sampler.BatchSampler(inter, int(g["item_num"]), lay.heads, lay.rels, lay.tails, lay.n_nodes, kg_batch_size=128,
                             seed=3)
    for _ in range(20):
        h, r, p, n = (t.numpy() for t in s.generate_kg_batch())
        assert len(set(h.tolist())) == h.size
        for a, b, c, d in zip(h, r, p, n):
            assert (int(b), int(c)) in edges[int(a)]
            assert (int(b), int(d)) not in edges[int(a)] and 0 <= d < lay.n_nodes


def test_sampler_refuses_impossible_rows():
    with pytest.raises(RuntimeError):
        sampler.BatchSampler({0: [0, 1]}, 2, np.array([0]), np.array([0]), np.array([1]), 3,
                             cf_batch_size=1).generate_cf_batch()  # every item is a positive
