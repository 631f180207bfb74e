"""Data-parallel KGAT replicas: one process per GPU, gradients all-reduced over RCCL.

SURVEY §8(e)(1): every CF step already propagates the whole graph for its own
256-pair batch (model.py:188), so G GPUs run G independent steps on replicas
of the model and graph (global batch 256*G) and average their gradients once
per step.  There is no other data-path collective.  Bucketing follows xGMI's
shape: the [N, d] table gradient is one large all-reduce on its own; the many
small aggregator / relation / trans gradients are coalesced into one flat
bucket so they cost a single ring instead of one launch each.

Works with any torch.distributed backend: ``nccl`` (= RCCL on ROCm) on the
GPU box, ``gloo`` for the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

SMALL_BUCKET_BYTES = 32 << 20


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def broadcast_parameters(module: torch.nn.Module, src: int = 0) -> None:
    """Make every replica start from rank ``src``'s dense parameters."""
    if world() == 1:
        return
    for p in module.parameters():
        if not p.is_sparse:
            dist.broadcast(p.data, src)


def allreduce_gradients(params, average: bool = True) -> None:
    """Average ``p.grad`` over all ranks (params whose grad is None are skipped on every rank:
    the set must agree across ranks, which it does -- it depends only on the mode)."""
    n = world()
    if n == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    big = [g for g in grads if g.numel() * g.element_size() > SMALL_BUCKET_BYTES]
    small = [g for g in grads if g.numel() * g.element_size() <= SMALL_BUCKET_BYTES]
    for g in big:
        dist.all_reduce(g)
        if average:
            g.div_(n)
    if small:
        flat = torch.cat([g.reshape(-1) for g in small])
        dist.all_reduce(flat)
        if average:
            flat.div_(n)
        off = 0
        for g in small:
            k = g.numel()
            g.copy_(flat[off:off + k].view_as(g))
            off += k
