"""graph.HashedCKG (csrc/synth.cpp): the row-sharded synthetic CKG builder of the C4/C5 configs.

Pinned to graph.layout_from_blocks -- itself checked bit for bit against the reference's own
Preprocess (tests/test_host_cpu.py) -- on the generator's raw triples: every shard's coalesced CSR
rows must equal the layout's rows exactly (structure, column order, fp32 values), for several
shard cuts, and a RowShard built from the local rows must equal one sliced from the whole graph."""
from __future__ import annotations

import numpy as np
import pytest

from tests.conftest import load_pkg


@pytest.fixture(scope="module")
def mods():
    pkg = load_pkg()
    graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])
    sh = __import__(pkg.__name__ + ".sharded", fromlist=["sharded"])
    return graph, sh


def _transpose(lay):
    """CSR of A^T (rows ascending columns) of a layout, the order graph.DeviceGraph keeps."""
    rows = np.repeat(np.arange(lay.n_nodes, dtype=np.int64), np.diff(lay.rowptr))
    perm = np.lexsort((rows, lay.col.astype(np.int64)))
    rp = np.zeros(lay.n_nodes + 1, np.int64)
    np.cumsum(np.bincount(lay.col, minlength=lay.n_nodes), out=rp[1:])
    return rp, rows[perm].astype(np.int32), lay.val[perm]


@pytest.mark.parametrize("n,t,seed", [(5000, 40000, 3), (20000, 200000, 2024), (60, 500, 1)])
def test_shards_equal_reference_layout(mods, n, t, seed):
    """Rows of A and of A^T, for several shard cuts, equal the layout producer's on the raw triples."""
    graph, sh = mods
    h = graph.HashedCKG(n, t, seed=seed, threads=4)
    U, E, inter, trip = h.raw()
    assert (h.user_num, h.entity_num) == (U, E) and len(inter) + len(trip) == h.n_triples
    if n >= 5000:
        assert h.n_triples == t  # enough distinct triples: exactly t kept
    else:
        assert h.n_triples < t and h.n_interactions == U * h.item_num  # 6 users x 5 items: saturated
    assert inter[:, 1].max() < h.item_num and (trip[:, 1] < 4).all() and trip[:, 2].max() < E
    lay = graph.build_layout(U, E, inter, trip)
    tr = _transpose(lay)
    off = h.row_offsets()
    assert off[-1] == 2 * h.n_triples  # every triple gives an entry and its inverse before coalescing
    for world in (1, 3, 8):
        b = sh.shard_bounds(off, world)
        for k in range(world):
            for (rp, col, val), (Rp, Col, Val) in ((h.shard(int(b[k]), int(b[k + 1])), (lay.rowptr, lay.col, lay.val)),
                                                   (h.shard(int(b[k]), int(b[k + 1]), transpose=True), tr)):
                e0, e1 = Rp[b[k]], Rp[b[k + 1]]
                np.testing.assert_array_equal(rp, Rp[b[k]:b[k + 1] + 1] - e0)
                np.testing.assert_array_equal(col, Col[e0:e1])
                np.testing.assert_array_equal(val, Val[e0:e1])


@pytest.mark.parametrize("n,t", [(20000, 200000), (100000, 1000000)])
def test_triples_distinct_and_entries_twice_triples(mods, n, t):
    """VERDICT r2 #7 / SURVEY §8(d): repeated triples are dropped and redrawn -- every kept
    interaction (user, item) and KG (head, rel, tail) is distinct, the counts are the targets
    (80 % / 20 %), and the attentive matrix holds E within 1 % of 2 T (only (row, col) pairs that
    two blocks share coalesce)."""
    graph, _ = mods
    h = graph.HashedCKG(n, t, seed=2024, threads=8)
    U, E, inter, trip = h.raw()
    assert len(inter) == int(t * 0.8) and len(trip) == t - int(t * 0.8)
    assert np.unique(inter[:, 0] * h.item_num + inter[:, 1]).size == len(inter)
    assert np.unique((trip[:, 0] * 4 + trip[:, 1]) * E + trip[:, 2]).size == len(trip)
    assert h.draws > t  # Zipf item popularity repeats (user, item) pairs: some draws were redrawn
    rp, col, val = h.shard(0, h.n_nodes)
    assert abs(col.size - 2 * t) <= 0.01 * 2 * t, (col.size, 2 * t)


def test_threads_do_not_change_the_graph(mods):
    graph, _ = mods
    a = graph.HashedCKG(30000, 300000, seed=7, threads=1).shard(0, 30000)
    b = graph.HashedCKG(30000, 300000, seed=7, threads=8).shard(0, 30000)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_zipf_hubs_and_relation_mix(mods):
    graph, _ = mods
    h = graph.HashedCKG(200000, 1000000, seed=2024, threads=8)
    assert h.n_interactions == 800000 and h.n_kg == 200000
    _, r, b = h.triples(np.arange(h.n_triples))
    items = np.bincount(b[r < 0], minlength=h.item_num)
    assert items.max() > 50 * items.mean()  # Zipf(1.1) popularity: hub items
    assert np.allclose(np.bincount(r[r >= 0], minlength=4) / h.n_kg, 0.25, atol=0.01)


def test_rowshard_from_local_rows_matches_global(mods):
    """A RowShard built from the generator's own rows (A and A^T, as bench.py's c5 builds it) equals
    one cut from the whole graph: both CSRs, the refresh keys and the value-exchange plan."""
    graph, sh = mods
    h = graph.HashedCKG(3000, 20000, seed=5, threads=2)
    lay = graph.build_layout(*h.raw())
    b = sh.shard_bounds(h.row_offsets(), 3)
    for k in range(3):
        g = sh.RowShard(lay.rowptr, lay.col, lay.val, b, k, "cpu")
        lo, hi = int(b[k]), int(b[k + 1])
        loc = sh.RowShard(*h.shard(lo, hi), b, k, "cpu", local=True, transpose=h.shard(lo, hi, transpose=True))
        np.testing.assert_array_equal(g.local_keys, loc.local_keys)
        for x, y in ((g.A, loc.A), (g.AT, loc.AT)):
            np.testing.assert_array_equal(x.rowptr_host, y.rowptr_host)
            assert np.array_equal(x.col.numpy(), y.col.numpy()) and np.array_equal(x.val.numpy(), y.val.numpy())
        for x, y in zip(g.value_plan(), loc.value_plan()):
            assert np.array_equal(np.asarray(x), np.asarray(y))
