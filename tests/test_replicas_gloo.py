"""Multi-process (world_size 2, gloo, CPU) checks of the data-parallel replica logic."""
from __future__ import annotations

import os
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import load_pkg


def _rendezvous() -> str:
    """A file rendezvous: no TCP port to race for between concurrently started tests."""
    fd, path = tempfile.mkstemp(prefix="kgat_gloo_")
    os.close(fd)
    os.unlink(path)
    return "file://" + path


def _worker(rank: int, world: int, port: int, q) -> None:
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        pkg = load_pkg()
        rep = __import__(pkg.__name__ + ".replicas", fromlist=["replicas"])
        torch.manual_seed(100 + rank)  # different init per rank ...
        m = pkg.KGAT(pkg.KGATArgs(user_num=10, entity_num=30, relation_num=10, layer_size=[64, 32]))
        rep.broadcast_parameters(m)    # ... until rank 0's weights are broadcast
        emb = m._user_entity_embedding.weight
        # rank-dependent fake gradients; a big one (the table) and small ones
        rep.SMALL_BUCKET_BYTES = 4096
        for p in m.parameters():
            if not p.is_sparse:
                p.grad = torch.full_like(p, float(rank + 1))
        m._relation_embedding.weight.grad = None  # skipped on every rank
        rep.allreduce_gradients(list(m.parameters()))
        ok_avg = all(torch.allclose(p.grad, torch.full_like(p, 1.5)) for p in m.parameters()
                     if not p.is_sparse and p.grad is not None)
        # plain numpy through the queue: a shared-memory tensor handle can outlive its exiting sender
        q.put((rank, ok_avg, emb.detach().clone().numpy(), m._relation_embedding.weight.grad is None))
    finally:
        dist.destroy_process_group()


def test_allreduce_and_broadcast_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), "gradients not averaged"
    assert (res[0][2] == res[1][2]).all(), "replicas did not start from the same weights"
    assert all(r[3] for r in res)


def _sharded_worker(rank: int, world: int, port: str, q) -> None:
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        pkg = load_pkg()
        rep = __import__(pkg.__name__ + ".replicas", fromlist=["replicas"])
        table = torch.nn.Parameter(torch.zeros(11, 4))   # 11 rows over 2 ranks: blocks of 5 + 1 tail row
        small = torch.nn.Parameter(torch.zeros(3))
        g = torch.arange(44, dtype=torch.float32).view(11, 4) * (rank + 1)
        table.grad, small.grad = g.clone(), torch.full((3,), float(rank + 1))
        sync = rep.ShardedGradSync([table, small], big_bytes=64)
        ranges = sync.reduce()
        r0, r1 = 5 * rank, 5 * rank + 5
        mean = torch.arange(44, dtype=torch.float32).view(11, 4) * 1.5
        ok = ranges == {id(table): [(r0, r1), (10, 11)]}
        ok &= torch.equal(table.grad[r0:r1], mean[r0:r1]) and torch.equal(table.grad[10:], mean[10:])
        ok &= torch.equal(small.grad, torch.full((3,), 1.5))
        # the optimizer touches only the owned rows (+ the replicated tail) ...
        with torch.no_grad():
            table.data[r0:r1] = rank + 7.0
            table.data[10:] = 3.0
        sync.gather()  # ... and the gather makes every replica whole again
        want = torch.cat([torch.full((5, 4), 7.0), torch.full((5, 4), 8.0), torch.full((1, 4), 3.0)])
        q.put((rank, bool(ok), torch.equal(table.data, want)))
    finally:
        dist.destroy_process_group()


def test_sharded_grad_sync_world2():
    """replicas.ShardedGradSync: row-block reduce-scatter (gloo: all-reduce) of the big gradient,
    tail rows and small gradients all-reduced, the row ranges the optimizer steps, the all-gather."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), res
    assert all(r[2] for r in res), res


def _discard_worker(rank: int, world: int, port: str, q) -> None:
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        pkg = load_pkg()
        rep = __import__(pkg.__name__ + ".replicas", fromlist=["replicas"])
        sync = rep.ShardedGradSync([], replicate_table=True)
        out = []
        for discarded in ((0, 0), (1, 1), (1, 2)):
            sync.discarded = discarded[rank]
            both = sync._gather_info(True, torch.tensor([10 + rank], dtype=torch.int32), "cpu")
            try:
                dev, host = sync._split_info(both, both.reshape(-1).tolist())
                out.append((dev.tolist(), host))
            except RuntimeError as e:
                out.append(str(e)[:80])
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_announce_discards_compared_across_ranks():
    """the replicated exchange's (hop count, discarded announcements) all-gather -- equal
    discard counts pass the counts through in rank order; unequal ones (ranks whose control flow
    diverged) raise instead of pairing up different steps' collectives."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _rendezvous()
    procs = [ctx.Process(target=_discard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, out in res:
        assert out[0] == ([10, 11], [10, 11]) and out[1] == ([10, 11], [10, 11]), out
        assert isinstance(out[2], str) and "discarded different" in out[2], out
