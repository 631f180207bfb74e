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


@pytest.mark.parametrize("n,t,seed", [(5000, 40000, 3), (20000, 200000, 2024), (60, 500, 1)])
def test_shards_equal_reference_layout(mods, n, t, seed):
    graph, sh = mods
    h = graph.HashedCKG(n, t, seed=seed, threads=4)
    U, E, inter, trip = h.raw()
    assert (h.user_num, h.entity_num) == (U, E) and len(inter) + len(trip) == t
    assert inter[:, 1].max() < h.item_num and (trip[:, 1] < 4).all() and trip[:, 2].max() < E
    lay = graph.build_layout(U, E, inter, trip)
    off = h.row_offsets()
    assert off[-1] == 2 * t  # every triple gives an entry and its inverse before coalescing
    for world in (1, 3, 8):
        b = sh.shard_bounds(off, world)
        for k in range(world):
            rp, col, val = h.shard(int(b[k]), int(b[k + 1]))
            e0, e1 = lay.rowptr[b[k]], lay.rowptr[b[k + 1]]
            np.testing.assert_array_equal(rp, lay.rowptr[b[k]:b[k + 1] + 1] - e0)
            np.testing.assert_array_equal(col, lay.col[e0:e1])
            np.testing.assert_array_equal(val, lay.val[e0:e1])


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
    graph, sh = mods
    h = graph.HashedCKG(3000, 20000, seed=5, threads=2)
    lay = graph.build_layout(*h.raw())
    b = sh.shard_bounds(h.row_offsets(), 3)
    for k in range(3):
        g = sh.RowShard(lay.rowptr, lay.col, lay.val, b, k, "cpu")
        loc = sh.RowShard(*h.shard(int(b[k]), int(b[k + 1])), b, k, "cpu", local=True)
        np.testing.assert_array_equal(g.local_keys, loc.local_keys)
        for j in range(3):
            for x, y in ((g.blocks[j], loc.blocks[j]), (g.blocks_t[j], loc.blocks_t[j])):
                np.testing.assert_array_equal(x.rowptr_host, y.rowptr_host)
                assert np.array_equal(x.col.numpy(), y.col.numpy()) and np.array_equal(x.val.numpy(), y.val.numpy())
            assert np.array_equal(g.block_t_pos[j].numpy(), loc.block_t_pos[j].numpy())
