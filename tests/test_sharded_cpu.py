"""CPU checks of the row-sharded mode (sharded.py): the shard plan and the ring / collective
transport over gloo with world_size 2 and 3.  No GPU compute here."""
from __future__ import annotations

import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import load_pkg

pkg = load_pkg()
sharded = __import__(pkg.__name__ + ".sharded", fromlist=["sharded"])
graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])


def _random_csr(n, nnz, seed):
    rng = np.random.default_rng(seed)
    r = rng.integers(0, n, nnz)
    c = (rng.zipf(1.3, nnz) - 1) % n
    key = np.unique(r * n + c)
    r, c = key // n, key % n
    v = rng.random(r.size).astype(np.float32)
    return graph.csr_from_coo(n, r, c, v)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_bounds_cover_and_balance(world):
    rowptr, _, _ = _random_csr(5000, 60000, world)
    b = sharded.shard_bounds(rowptr, world)
    assert b[0] == 0 and b[-1] == 5000 and b.size == world + 1 and np.all(np.diff(b) > 0)
    mean = rowptr[-1] / 5000
    load = [(rowptr[b[k + 1]] - rowptr[b[k]]) + mean * (b[k + 1] - b[k]) for k in range(world)]
    assert max(load) <= 1.25 * (sum(load) / world) + 2000  # hubs make exact balance impossible


def test_shard_bounds_cost_model():
    """The round-6 cost model: rows weigh SHARD_ROW_WEIGHT entries, entries of the ``edge_scale`` ranges their
    factor -- every rank's modelled cost within one heavy row of the mean, an empty scale list = none."""
    rowptr, _, _ = _random_csr(20000, 200000, 5)
    for world in (2, 8):
        plain = sharded.shard_bounds(rowptr, world)
        assert np.array_equal(plain, sharded.shard_bounds(rowptr, world, edge_scale=[]))
        lo, hi, f = 3000, 9000, 2.2
        b = sharded.shard_bounds(rowptr, world, edge_scale=[(lo, hi, f)])
        assert b[0] == 0 and b[-1] == 20000 and np.all(np.diff(b) > 0)
        w = sharded.SHARD_ROW_WEIGHT
        deg = np.diff(rowptr).astype(np.float64)
        cost_row = deg * np.where((np.arange(20000) >= lo) & (np.arange(20000) < hi), f, 1.0) + w
        cost = [cost_row[b[k]:b[k + 1]].sum() for k in range(world)]
        assert max(cost) - min(cost) <= 2 * cost_row.max() + 1e-6
        assert not np.array_equal(b, plain)  # the item-like range moved the cuts


@pytest.mark.parametrize("world", [2, 3])
def test_row_shard_reassembles_A_and_AT(world):
    """Every rank's A rows (global columns) and A^T rows reassemble A and A^T, columns ascending."""
    n = 700
    rowptr, col, val = _random_csr(n, 9000, 7)
    dense = np.zeros((n, n), np.float32)
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    dense[rows, col] = val
    b = sharded.shard_bounds(rowptr, world)
    for k in range(world):
        sh = sharded.RowShard(rowptr, col, val, b, k, "cpu")
        assert sh.nnz == rowptr[b[k + 1]] - rowptr[b[k]]
        for csr, want in ((sh.A, dense[b[k]:b[k + 1]]), (sh.AT, dense.T[b[k]:b[k + 1]])):
            rp, cc, vv = csr.rowptr.numpy(), csr.col.numpy(), csr.val.numpy()
            rr = np.repeat(np.arange(csr.n_rows), np.diff(rp))
            m = np.zeros((sh.n, n), np.float32)
            m[rr, cc] = vv
            np.testing.assert_array_equal(m, want)
            assert np.all(np.diff(rr) >= 0)
            assert all(np.all(np.diff(cc[rp[r]:rp[r + 1]]) > 0) for r in range(csr.n_rows))


def _rendezvous() -> str:
    """A file rendezvous: no TCP port to race for between concurrently started tests."""
    fd, path = tempfile.mkstemp(prefix="kgat_gloo_")
    os.close(fd)
    os.unlink(path)
    return "file://" + path


def _comm_worker(rank: int, world: int, port: int, q) -> None:
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        comm = sharded.Comm()
        assert comm.host and comm.next == (rank + 1) % world and comm.prev == (rank - 1) % world
        # ring exchange (kept for the library transport's tests)
        buf = torch.full((3 + rank, 2), float(rank))
        nxt = torch.empty(3 + (rank - 1) % world, 2)
        comm.exchange(buf, nxt).wait()
        ring_ok = bool((nxt == float((rank - 1) % world)).all())
        # all-peer gather of uneven shards (one rank owns no rows when world = 3)
        sizes = [3, 0, 5][:world] if world == 3 else [4, 2]
        bounds = np.concatenate([[0], np.cumsum(sizes)])
        out = torch.full((int(bounds[-1]), 3), -1.0)
        mine = torch.arange(sizes[rank] * 3, dtype=torch.float32).reshape(-1, 3) + 100 * rank
        comm.gather_v(mine, out, bounds).wait()
        want = torch.cat([torch.arange(sizes[r] * 3, dtype=torch.float32).reshape(-1, 3) + 100 * r for r in range(world)])
        gather_ok = torch.equal(out, want)
        # all-to-all with per-peer sizes: rank r sends (r + 1) * (p + 1) values to rank p
        send_cnt = [(rank + 1) * (p + 1) for p in range(world)]
        send_off = np.concatenate([[0], np.cumsum(send_cnt)])
        send = torch.cat([torch.full((c,), float(10 * rank + p)) for p, c in enumerate(send_cnt)])
        recv_cnt = [(p + 1) * (rank + 1) for p in range(world)]
        recv_off = np.concatenate([[0], np.cumsum(recv_cnt)])
        recv = torch.empty(int(recv_off[-1]))
        comm.all_to_all_v(send, send_off, recv, recv_off)
        a2a_ok = torch.equal(recv, torch.cat([torch.full((c,), float(10 * p + rank)) for p, c in enumerate(recv_cnt)]))
        red = comm.all_reduce_(torch.full((4,), float(rank + 1)))
        gat = comm.all_gather(torch.tensor([rank, 10 * rank]))
        # comm.WireLog: the bytes this rank sent, by the counting rule of each collective
        want_wire = ((3 + rank) * 2 * 4 + sizes[rank] * 3 * 4 * (world - 1)
                     + 4 * (int(send_off[-1]) - send_cnt[rank]) + 2 * (world - 1) * 16 // world + (world - 1) * 2 * 8)
        wire_ok = sharded.wire(comm).bytes == {"other": want_wire}
        q.put((rank, ring_ok, gather_ok, a2a_ok and wire_ok, red.tolist(), gat.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_comm_collectives_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = float(sum(range(1, world + 1)))
    for rank, ring_ok, gather_ok, a2a_ok, red, gat in res:
        assert ring_ok and gather_ok and a2a_ok, (rank, ring_ok, gather_ok, a2a_ok)
        assert red == [total] * 4
        assert gat == [[r, 10 * r] for r in range(world)]


def _csr_dense(blk, n_cols):
    rp, cc, vv = blk.rowptr.numpy(), blk.col.numpy(), blk.val.numpy()
    m = torch.zeros(blk.n_rows, n_cols)
    rr = np.repeat(np.arange(blk.n_rows), np.diff(rp))
    m[torch.from_numpy(rr), torch.from_numpy(cc.astype(np.int64))] = torch.from_numpy(vv)
    return m


def _pull_worker(rank: int, world: int, port: str, q) -> None:
    """The gathered SpMM of sharded.py (column-chunked all-peer gather + local-row product) forward
    with A's rows and backward with A^T's rows, and the refresh's value exchange, with TEST-ONLY dense
    stand-ins for the HIP kernels (the product path calls the HIP library; here only the gather's
    chunking, offsets and ordering are under test)."""
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        n = 500
        rowptr, col, val = _random_csr(n, 6000, 11)
        b = sharded.shard_bounds(rowptr, world)
        sh = sharded.RowShard(rowptr, col, val, b, rank, "cpu")
        comm = sharded.Comm()

        class FakeKernels:
            @staticmethod
            def spmm_block(blk, X, out, accumulate=False, transpose=False):
                y = _csr_dense(blk, X.shape[0]) @ X
                out.copy_(out + y if accumulate else y)
                return out

            @staticmethod
            def gather_rows(src, rows, out=None):
                out.copy_(src[rows.long()])
                return out

        real = sharded.kernels
        sharded.kernels = FakeKernels
        old_chunk = sharded.GATHER_CHUNK
        sharded.GATHER_CHUNK = 3  # 8 columns in chunks of 3, 3, 2
        try:
            g = torch.Generator().manual_seed(5)
            X = torch.randn(n, 8, generator=g)
            G = torch.randn(n, 8, generator=g)
            rows = np.repeat(np.arange(n), np.diff(rowptr))
            A = torch.zeros(n, n)
            A[torch.from_numpy(rows), torch.from_numpy(col.astype(np.int64))] = torch.from_numpy(val)
            lo, hi = sh.lo, sh.hi
            S = torch.empty(hi - lo, 8)
            sharded.gathered_spmm(sh, comm, sh.A, X[lo:hi].contiguous(), S)
            fwd_ok = torch.allclose(S, (A @ X)[lo:hi], atol=1e-4)
            T = torch.ones(hi - lo, 8)
            sharded.gathered_spmm(sh, comm, sh.AT, G[lo:hi].contiguous(), T, accumulate=True, transpose=True)
            bwd_ok = torch.allclose(T, 1.0 + (A.T @ G)[lo:hi], atol=1e-4)
            # the refresh's value exchange: new values on A's rows reach A^T's rows of the owners
            newA = A * 2.0 + 1.0 * (A != 0)
            sh.A.val = newA[torch.from_numpy(np.repeat(np.arange(lo, hi), np.diff(sh._lrp))),
                            torch.from_numpy(sh._lcol.astype(np.int64))].contiguous()
            send_pos, send_off, recv_inv, recv_off = sh.value_plan()
            send = sh.A.val[send_pos.long()]
            recv = torch.empty(int(recv_off[-1]))
            comm.all_to_all_v(send, send_off, recv, recv_off)
            at_val = recv[recv_inv.long()]
            at_rows = torch.from_numpy(np.repeat(np.arange(lo, hi), np.diff(sh._trp)))
            want = newA.T[at_rows, torch.from_numpy(sh._tcol.astype(np.int64))]
            val_ok = torch.equal(at_val, want)
        finally:
            sharded.kernels = real
            sharded.GATHER_CHUNK = old_chunk
        q.put((rank, bool(fwd_ok), bool(bwd_ok), bool(val_ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gathered_spmm_and_value_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous()
    procs = [ctx.Process(target=_pull_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, f, b_, v in res:
        assert f, f"rank {rank}: gathered forward SpMM wrong"
        assert b_, f"rank {rank}: gathered transposed SpMM wrong"
        assert v, f"rank {rank}: refresh value exchange wrong"
