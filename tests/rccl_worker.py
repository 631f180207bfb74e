"""RCCL (backend "nccl") at world 1 on the one GPU of a test box (tests/test_gpu_sharded.py launches it
through ``python -m torch.distributed.run --nproc-per-node 1``).

A pool box has one GPU, so the multi-rank collectives of replicas.py / sharded.py otherwise run over
RCCL only in the driver's 8-GPU bench.  Here every collective those modules issue runs through the
real RCCL library (forced at world 1) and its results are compared with the gloo / no-collective paths:

(1) the raw calls: all_gather_into_tensor (in place), reduce_scatter_tensor (in place), all_reduce,
    reduce, and the ring's batch_isend_irecv (a send to self);
(2) data-parallel replicas over 2 CF steps (train mode, same dropout draws): ShardedGradSync in the
    row-block mode (reduce per transposed row block during the backward, owned-row Adam, in-place
    all-gather) and in the replicated-table mode (hop-set all-gathers, kgat_rows_union / merge) against
    a model without any exchange -- bit-identical parameters;
(3) RowShardedKGAT: one CF step with its collectives on RCCL against the same step on a gloo group
    (host-staged transport) -- loss and every gradient bit-identical;
(4) the library's own RCCL communicator (kgat_comm_*, comm.RcclComm): every call (gather_at on the
    torch.distributed transports too), and the same RowShardedKGAT step with RcclComm as its transport --
    bit-identical to (3).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.conftest import load_pkg  # noqa: E402


def main() -> None:
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    failures = []
    if dist.get_backend() != "nccl" or dist.get_world_size() != 1:
        failures.append(f"backend {dist.get_backend()} world {dist.get_world_size()}")
    gloo = dist.new_group(backend="gloo")
    pkg = load_pkg()
    graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])
    rep = __import__(pkg.__name__ + ".replicas", fromlist=["replicas"])
    sh = __import__(pkg.__name__ + ".sharded", fromlist=["sharded"])

    # (1) raw collectives
    x = torch.arange(4096, dtype=torch.float32, device=dev) * 0.5
    out = torch.empty_like(x)
    dist.all_gather_into_tensor(out, x)
    y = x.clone()
    dist.all_gather_into_tensor(y, y)  # in place (send = recv + rank * count)
    z = x.clone()
    dist.reduce_scatter_tensor(z, z)
    w = x.clone()
    dist.all_reduce(w)
    dist.reduce(w, dst=0)
    comm = sh.Comm(force=True)
    recv = torch.empty_like(x)
    comm.exchange(x, recv).wait()
    for name, t in (("all_gather", out), ("all_gather_inplace", y), ("reduce_scatter", z), ("all_reduce", w),
                    ("ring_exchange", recv)):
        if not torch.equal(t, x):
            failures.append(f"(1) {name} changed the data")

    # (2) data-parallel exchange modes vs no exchange
    U, E, inter, trip = graph.synthetic_ckg(12001, 90000, seed=9)
    lay = graph.build_layout(U, E, inter, trip)
    args = pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32],
                        message_dropout=[0.1, 0.1])
    models, syncs = [], []
    for k in range(3):
        torch.manual_seed(3)
        m = pkg.KGAT(args)
        m.attach_graph(lay, dev)
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        params = [p for p in m.parameters() if not p.is_sparse and p.requires_grad]
        syncs.append(None if k == 0 else rep.ShardedGradSync(params, replicate_table=k == 2, force=True).attach(m))
        models.append(m)
    rng = np.random.default_rng(4)
    for step in range(2):
        b = [torch.from_numpy(v).to(dev) for v in (rng.integers(0, U, 64), rng.integers(0, E // 10, 64),
                                                  rng.integers(0, E // 10, 64))]
        for m, sync in zip(models, syncs):
            torch.manual_seed(100 + step)
            loss = m(*b, mode=pkg.KGATMode.TRAIN_CF)
            loss.backward()
            if sync is None:
                m.update_cf_weights()
            else:
                m.update_cf_weights(row_ranges=sync.reduce())
                sync.gather()
    if syncs[2].stats.get("hop", 0) != 2:
        failures.append(f"(2) replicated mode took {syncs[2].stats}, expected 2 hop-set exchanges")
    for named in zip(*(m.named_parameters() for m in models)):
        na, pa = named[0]
        if pa.is_sparse:
            continue
        for tag, (_, po) in zip(("sharded", "replicated"), named[1:]):
            if not torch.equal(pa.data, po.data):
                failures.append(f"(2) {tag} {na}: max |diff| {(pa.data - po.data).abs().max().item():.3e}")

    # (3) row-sharded CF step: RCCL vs gloo transport
    args3 = pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32, 16],
                         message_dropout=[0.0, 0.0, 0.0])
    res = []
    comm_mod = __import__(pkg.__name__ + ".comm", fromlist=["comm"])
    rc = comm_mod.RcclComm.from_process_group(dev, force=True)
    for transport in (sh.Comm(None, force=True), sh.Comm(gloo, force=True), rc):
        torch.manual_seed(5)
        m = sh.RowShardedKGAT(args3, lay, transport, dev)
        b = [torch.from_numpy(v).to(dev) for v in (np.arange(0, 128), np.arange(5, 133), np.arange(9, 137))]
        loss = m(*b, mode=pkg.KGATMode.TRAIN_CF)
        loss.backward()
        res.append([loss.detach().clone()] + [p.grad.detach().clone() for p in m.parameters()
                                              if p.grad is not None])
    for tag, other in (("(3) gloo", res[1]), ("(4) kgat_comm", res[2])):
        if len(res[0]) != len(other):
            failures.append(f"{tag}: gradient sets differ")
        for i, (a, g) in enumerate(zip(res[0], other)):
            if not torch.equal(a, g):
                failures.append(f"{tag} tensor {i}: max |diff| {(a - g).abs().max().item():.3e}")

    # (4) kgat_comm_* calls at world 1: each collective returns its input (ring: a send to self)
    x = torch.arange(4096, dtype=torch.float32, device=dev) * 0.25
    got = {"all_reduce_": rc.all_reduce_(x.clone()), "all_gather": rc.all_gather(x)[0],
           "all_gather_rows_": rc.all_gather_rows_(x.clone()), "reduce_scatter_rows": rc.reduce_scatter_rows(x.clone())}
    recv = torch.empty_like(x)
    rc.exchange(x, recv).wait()
    got["ring_exchange"] = recv
    # the pipelined row-sharded forward's block post (kgat_comm_gather_at): rows [5, 21) of a 4096 x 1
    # view land at rows [7, 23) of the output, the rest of it untouched
    for tag, tp in (("kgat_comm gather_at", rc), ("torch gather_at", sh.Comm(None, force=True)),
                    ("gloo gather_at", sh.Comm(gloo, force=True))):
        src = x.view(-1, 16)[5:21].contiguous()
        dst = torch.full((40, 16), -1.0, device=dev)
        tp.gather_at(src, dst, [7], [16]).wait()
        want = torch.full((40, 16), -1.0, device=dev)
        want[7:23] = src
        if not torch.equal(dst, want):
            failures.append(f"(4) {tag} placed the rows wrong")
    for name, t in got.items():
        if not torch.equal(t, x):
            failures.append(f"(4) {name} changed the data")
    rc.close()

    print(f"rccl world1: {'OK' if not failures else failures}", flush=True)
    dist.destroy_process_group()
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
