"""One rank of the DistributedDataParallel check (launched by tests/test_gpu_sharded.py through
``python -m torch.distributed.run --nproc-per-node 2``; every rank on cuda:0, gloo).

KGAT wrapped in ``torch.nn.parallel.DistributedDataParallel`` as a user's own data-parallel loop would
(src/model/KGAT/main.py:312's ``loss.backward()`` unchanged): DDP's reducer hooks the leaves' gradient
accumulators from C++, which the model's direct backward (``KGAT.direct_backward``, model._StepLoss) cannot
see -- so it is off by default, the engine runs, and after ``loss.backward()`` every table and aggregator
weight gradient is the mean of the ranks' local gradients.  Each rank also computes its local gradient with
an unwrapped replica of the same weights on its own batch; the local gradients are all-gathered and their
mean compared with what DDP left in ``.grad``.
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
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    pkg = load_pkg()
    graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])
    U, E, inter, trip = graph.synthetic_ckg(6000, 60000, seed=13)
    lay = graph.build_layout(U, E, inter, trip)
    args = pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32],
                        message_dropout=[0.0, 0.0])
    models = []
    for _ in range(2):
        torch.manual_seed(21)
        m = pkg.KGAT(args)
        m.attach_graph(lay, "cuda")
        m.train()
        models.append(m)
    local, wrapped = models
    assert not wrapped.direct_backward  # the default: the autograd engine, DDP's hooks run
    # the sparse attentive matrix is graph data, not a trained weight (it never gets a gradient)
    torch.nn.parallel.DistributedDataParallel._set_params_and_buffers_to_ignore_for_model(
        wrapped, ["attentive_matrix"])
    ddp = torch.nn.parallel.DistributedDataParallel(wrapped, find_unused_parameters=True)
    rng = np.random.default_rng(70 + rank)  # each rank its own batch
    failures = []
    for step in range(2):
        b = [torch.from_numpy(x).cuda() for x in (rng.integers(0, U, 128), rng.integers(0, E // 10, 128),
                                                  rng.integers(0, E // 10, 128))]
        for m in models:
            m.zero_grad(set_to_none=True)
        local(*b, mode=pkg.KGATMode.TRAIN_CF).backward()
        ddp(*b, mode=pkg.KGATMode.TRAIN_CF).backward()
        names = [n for n, p in local.named_parameters() if p.grad is not None]
        if "_user_entity_embedding.weight" not in names or len(names) != 9:
            failures.append(f"step {step}: local gradients on {names}")
        wp = dict(wrapped.named_parameters())
        for n, p in local.named_parameters():
            if p.grad is None:
                continue
            g = p.grad.detach().clone()
            dist.all_reduce(g)
            g /= world
            got = wp[n].grad
            if got is None or not torch.allclose(got, g, rtol=1e-5, atol=1e-9):
                diff = None if got is None else (got - g).abs().max().item()
                failures.append(f"step {step} {n}: DDP gradient is not the mean over ranks (max |diff| {diff})")
            elif world > 1 and torch.equal(got, p.grad) and p.grad.abs().max() > 0:
                failures.append(f"step {step} {n}: DDP gradient equals the rank's local one (no all-reduce ran)")
        # the replicas stay identical after a plain SGD step on the all-reduced gradients
        with torch.no_grad():
            for p in wrapped.parameters():
                if p.grad is not None:
                    p.add_(p.grad, alpha=-1e-2)
            for (n, p), (_, q) in zip(wrapped.named_parameters(), local.named_parameters()):
                if not p.is_sparse:
                    q.copy_(p)  # the local replica follows the wrapped weights
                    other = p.detach().clone()
                    dist.broadcast(other, 0)
                    if not torch.equal(other, p):
                        failures.append(f"step {step} {n}: replicas diverged")
    print(f"rank {rank}: {'DDP OK' if not failures else failures}", flush=True)
    dist.destroy_process_group()
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
