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


@pytest.mark.parametrize("world", [2, 3])
def test_row_shard_blocks_reassemble_A(world):
    n = 700
    rowptr, col, val = _random_csr(n, 9000, 7)
    dense = np.zeros((n, n), np.float32)
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    dense[rows, col] = val
    b = sharded.shard_bounds(rowptr, world)
    for k in range(world):
        sh = sharded.RowShard(rowptr, col, val, b, k, "cpu")
        assert sum(sh.nnz) == rowptr[b[k + 1]] - rowptr[b[k]]
        for j in range(world):
            for blk, t in ((sh.blocks[j], False), (sh.blocks_t[j], True)):
                rp, cc, vv = blk.rowptr.numpy(), blk.col.numpy(), blk.val.numpy()
                rr = np.repeat(np.arange(blk.n_rows), np.diff(rp))
                m = np.zeros((sh.n, b[j + 1] - b[j]) if not t else (b[j + 1] - b[j], sh.n), np.float32)
                m[rr, cc] = vv
                want = dense[b[k]:b[k + 1], b[j]:b[j + 1]]
                np.testing.assert_array_equal(m.T if t else m, want)
                # rows sorted, columns sorted within a row (the reference's coalesced order)
                assert np.all(np.diff(rr) >= 0)


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
        # ring: after world-1 hops every rank has seen every shard once, in ring order
        buf = torch.full((3 + rank, 2), float(rank))
        seen = [rank]
        for s in range(world - 1):
            src = (rank - s - 1) % world
            nxt = torch.empty(3 + src, 2)
            comm.exchange(buf, nxt).wait()
            buf = nxt
            seen.append(int(buf[0, 0].item()))
            assert buf.shape[0] == 3 + src
        red = comm.all_reduce_(torch.full((4,), float(rank + 1)))
        gat = comm.all_gather(torch.tensor([rank, 10 * rank]))
        q.put((rank, seen, red.tolist(), gat.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_comm_ring_and_collectives_gloo(world):
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
    for rank, seen, red, gat in res:
        assert seen == [(rank - s) % world for s in range(world)]
        assert red == [total] * 4
        assert gat == [[r, 10 * r] for r in range(world)]


def _csr_dense(blk, n_cols):
    rp, cc, vv = blk.rowptr.numpy(), blk.col.numpy(), blk.val.numpy()
    m = torch.zeros(blk.n_rows, n_cols)
    rr = np.repeat(np.arange(blk.n_rows), np.diff(rp))
    m[torch.from_numpy(rr), torch.from_numpy(cc.astype(np.int64))] = torch.from_numpy(vv)
    return m


def _ring_worker(rank: int, world: int, port: str, q) -> None:
    """Ring all-gather SpMM and ring reduce-scatter of sharded.py with TEST-ONLY dense stand-ins for
    the three block kernels (the product path calls the HIP library; here only the ring's indexing
    and ordering are under test)."""
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        n = 500
        rowptr, col, val = _random_csr(n, 6000, 11)
        b = sharded.shard_bounds(rowptr, world)
        sh = sharded.RowShard(rowptr, col, val, b, rank, "cpu")
        comm = sharded.Comm()

        class FakeKernels:
            @staticmethod
            def spmm_block(blk, X, out, accumulate=False):
                y = _csr_dense(blk, X.shape[0]) @ X
                out.copy_(out + y if accumulate else y)
                return out

            @staticmethod
            def spmm_block_masked(blk, src_map, Xc, out):
                X = torch.zeros(src_map.numel(), Xc.shape[1])
                m = src_map >= 0
                X[m] = Xc[src_map[m].long()]
                out.copy_(_csr_dense(blk, X.shape[0]) @ X)
                return out

            @staticmethod
            def add_(y, x):
                y += x
                return y

        real = sharded.kernels
        sharded.kernels = FakeKernels
        try:
            g = torch.Generator().manual_seed(5)
            X = torch.randn(n, 8, generator=g)
            G = torch.randn(n, 8, generator=g)
            rows = np.repeat(np.arange(n), np.diff(rowptr))
            A = torch.zeros(n, n)
            A[torch.from_numpy(rows), torch.from_numpy(col.astype(np.int64))] = torch.from_numpy(val)
            lo, hi = sh.lo, sh.hi
            S = sharded.ring_spmm(sh, comm, X[lo:hi].contiguous())
            fwd_ok = torch.allclose(S, (A @ X)[lo:hi], atol=1e-4)
            # every rank holds its rows of G (= dS); the reduce-scatter returns (A^T G)[own rows]
            T = sharded.ring_spmm_t(sh, comm, 8, "cpu",
                                    lambda blk, out: FakeKernels.spmm_block(blk, G[lo:hi].contiguous(), out))
            bwd_ok = torch.allclose(T, (A.T @ G)[lo:hi], atol=1e-4)
            # frontier variant: only some local rows of G are nonzero (compact + src_map)
            F = torch.arange(0, hi - lo, 3)
            src_map = torch.full((hi - lo,), -1, dtype=torch.int32)
            src_map[F] = torch.arange(F.numel(), dtype=torch.int32)
            Gc = G[lo:hi][F].contiguous()
            Tm = sharded.ring_spmm_t(sh, comm, 8, "cpu",
                                     lambda blk, out: FakeKernels.spmm_block_masked(blk, src_map, Gc, out))
            Gm = torch.zeros_like(G)
            Gm[lo + F] = G[lo + F]
            gathered = comm.all_gather(Gm)  # every rank's frontier rows
            Gfull = gathered.sum(0)
            mask_ok = torch.allclose(Tm, (A.T @ Gfull)[lo:hi], atol=1e-4)
        finally:
            sharded.kernels = real
        q.put((rank, bool(fwd_ok), bool(bwd_ok), bool(mask_ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ring_spmm_and_reduce_scatter_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous()
    procs = [ctx.Process(target=_ring_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, f, b_, m in res:
        assert f, f"rank {rank}: ring all-gather SpMM wrong"
        assert b_, f"rank {rank}: ring reduce-scatter wrong"
        assert m, f"rank {rank}: masked ring reduce-scatter wrong"
