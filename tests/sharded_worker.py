"""One rank of the row-sharded parity check (launched by tests/test_gpu_sharded.py through
``python -m torch.distributed.run --nproc-per-node 2``; every rank on cuda:0, gloo, host-staged).

Every rank also runs the single-GPU KGAT on the GLOBAL batch (all ranks' pairs, rank order)
and checks that the sharded model's loss, its shard of every gradient, the replicated
gradients, the parameters after one Adam step of each optimiser and PREDICT scores agree.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.conftest import load_pkg  # noqa: E402

# Gradients agree to fp32 summation order.  After an Adam step they are compared at 1e-4: the ring
# sums A^T.dS in another order than one GPU, and Adam's eps turns that rounding on ~1e-9 gradients
# into differences up to ~1e-5 of a step (a wrong update is ~lr = 1e-3 off).
ATOL_GRAD, ATOL_PARAM = 1e-6, 1e-4
FAILURES: list[str] = []


def close(name, a, b, atol, rtol=1e-4):
    """Record (never raise): every rank must reach every collective whatever the numbers say."""
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    if a.shape != b.shape or not torch.allclose(a, b, atol=atol, rtol=rtol):
        diff = (a - b).abs().max().item() if a.shape == b.shape else float("nan")
        FAILURES.append(f"{name}: shape {tuple(a.shape)} vs {tuple(b.shape)}, max |diff| {diff:.3e}")


def main() -> None:
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    pkg = load_pkg()
    graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])
    sh = __import__(pkg.__name__ + ".sharded", fromlist=["sharded"])
    U, E, inter, trip = graph.synthetic_ckg(30000, 240000, seed=5)
    lay = graph.build_layout(U, E, inter, trip)
    # SHARDED_WORKER_DIMS "d:l1,l2,...": embedding dim and layer sizes (default the C2 shape; the C5
    # shape is "256:256,128,64", configs[4])
    dim_s, layers_s = os.environ.get("SHARDED_WORKER_DIMS", "64:64,32").split(":")
    dim, layers = int(dim_s), [int(x) for x in layers_s.split(",")]
    args = pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=layers,
                        cf_embedding_dim=dim, kg_embedding_dim=dim, message_dropout=[0.0] * len(layers))
    torch.manual_seed(11)
    ref = pkg.KGAT(args)
    ref.attach_graph(lay, "cuda")
    comm = sh.Comm()
    m = sh.RowShardedKGAT(args, lay, comm, "cuda")
    m.load_full_state(ref.state_dict())
    lo, hi = m.lo, m.hi
    assert hi - lo > 0

    # ---- CF step: each rank its own 64 pairs; the reference sees all of them
    rng = np.random.default_rng(100)
    n_items = int(inter[:, 1].max()) + 1
    glob = [(rng.integers(0, U, 64), rng.integers(0, n_items, 64), rng.integers(0, n_items, 64))
            for _ in range(world)]
    mine = [torch.from_numpy(a).cuda() for a in glob[rank]]
    allb = [torch.from_numpy(np.concatenate([g[i] for g in glob])).cuda() for i in range(3)]
    ref.build_optimizer(1e-3, 1e-4)
    m.build_optimizer(1e-3, 1e-4)
    ref.train()
    m.train()
    lr = ref(*allb, mode=pkg.KGATMode.TRAIN_CF)
    lr.backward()
    ls = m(*mine, mode=pkg.KGATMode.TRAIN_CF)
    ls.backward()
    close("cf loss", ls, lr, 1e-6)
    close("cf d table shard", m._user_entity_embedding_shard.grad, ref._user_entity_embedding.weight.grad[lo:hi],
          ATOL_GRAD)
    # the pull backward sums every table-gradient row over the single GPU's edges in its order
    exact = {"cf_table_grad": torch.equal(m._user_entity_embedding_shard.grad,
                                          ref._user_entity_embedding.weight.grad[lo:hi])}
    for a, b in zip(m._cf_weights(), ref._cf_weights()):
        close("cf d aggregator", a.grad, b.grad, 1e-5)
    ref.update_cf_weights()
    m.update_cf_weights()
    close("table after cf adam", m._user_entity_embedding_shard, ref._user_entity_embedding.weight[lo:hi],
          ATOL_PARAM)
    for a, b in zip(m._cf_weights(), ref._cf_weights()):
        close("aggregator after cf adam", a, b, ATOL_PARAM)

    if rank == 0:
        print(f"sharded_worker world {world}: CF step done", flush=True)
    # ---- KG step (from identical parameters again)
    m.load_full_state(ref.state_dict())
    heads_all = [rng.integers(0, U + E, 32) for _ in range(world)]
    rels_all = [rng.integers(0, len(lay.rel_order), 32) for _ in range(world)]
    pos_all = [rng.integers(0, U + E, 32) for _ in range(world)]
    neg_all = [rng.integers(0, U + E, 32) for _ in range(world)]
    kg_mine = [torch.from_numpy(x[rank]).cuda() for x in (heads_all, rels_all, pos_all, neg_all)]
    kg_all = [torch.from_numpy(np.concatenate(x)).cuda() for x in (heads_all, rels_all, pos_all, neg_all)]
    lr = ref(*kg_all, mode=pkg.KGATMode.TRAIN_KG)
    lr.backward()
    ls = m(*kg_mine, mode=pkg.KGATMode.TRAIN_KG)
    ls.backward()
    close("kg loss", ls, lr, 1e-6)
    close("kg d table shard", m._user_entity_embedding_shard.grad, ref._user_entity_embedding.weight.grad[lo:hi],
          ATOL_GRAD)
    close("kg d relation", m._relation_embedding.weight.grad, ref._relation_embedding.weight.grad, ATOL_GRAD)
    close("kg d trans", m._trans_matrix.grad, ref._trans_matrix.grad, ATOL_GRAD)
    ref.update_kg_weights()
    m.update_kg_weights()
    close("table after kg adam", m._user_entity_embedding_shard, ref._user_entity_embedding.weight[lo:hi],
          ATOL_PARAM)

    if rank == 0:
        print(f"sharded_worker world {world}: KG step done", flush=True)
    # ---- UPDATE_ATTENTION (eval: MHA dropout off), then PREDICT on the refreshed graph
    m.load_full_state(ref.state_dict())
    ref.eval()
    m.eval()
    att = [torch.from_numpy(x).cuda() for x in (lay.heads, lay.rels, lay.tails)] + [torch.tensor(lay.rel_order)]
    ref(*att, mode=pkg.KGATMode.UPDATE_ATTENTION)
    m(*att, mode=pkg.KGATMode.UPDATE_ATTENTION)
    A = ref.graph().A
    close("refreshed A rows", m.shard.local_val, A.val[int(lay.rowptr[lo]):int(lay.rowptr[hi])], 1e-6)
    exact["refreshed_A"] = torch.equal(m.shard.local_val, A.val[int(lay.rowptr[lo]):int(lay.rowptr[hi])])
    with torch.no_grad():
        tabs_s, tabs_r = m.propagate(), ref.propagate()
    for l, (a, b) in enumerate(zip(tabs_s, tabs_r)):
        close(f"propagated table {l}", a, b[lo:hi], 1e-5)
    exact["tables"] = all(torch.equal(a, b[lo:hi]) for a, b in zip(tabs_s, tabs_r))
    # a CF backward on the refreshed graph: A^T's local rows got their values by the all-to-all
    m.load_full_state(ref.state_dict())
    for mm in (ref, m):
        mm.zero_grad(set_to_none=True)
    ref(*allb, mode=pkg.KGATMode.TRAIN_CF).backward()
    m(*mine, mode=pkg.KGATMode.TRAIN_CF).backward()
    close("cf d table shard after refresh", m._user_entity_embedding_shard.grad,
          ref._user_entity_embedding.weight.grad[lo:hi], ATOL_GRAD)
    exact["cf_table_grad_after_refresh"] = torch.equal(m._user_entity_embedding_shard.grad,
                                                       ref._user_entity_embedding.weight.grad[lo:hi])
    # the same step with the frontier forward (last layer on the batch rows, layer L-2 on the first hop)
    full_grads = [p.grad.detach().clone() for p in m.parameters() if not p.is_sparse and p.grad is not None]
    m.zero_grad(set_to_none=True)
    m.frontier_forward = True
    m(*mine, mode=pkg.KGATMode.TRAIN_CF).backward()
    m.frontier_forward = False
    close("cf d table shard (frontier forward)", m._user_entity_embedding_shard.grad,
          ref._user_entity_embedding.weight.grad[lo:hi], ATOL_GRAD)
    fr_grads = [p.grad.detach().clone() for p in m.parameters() if not p.is_sparse and p.grad is not None]
    exact["frontier_vs_full"] = len(fr_grads) == len(full_grads) and all(
        torch.equal(a, b) for a, b in zip(fr_grads, full_grads))
    # the same with every layer's hop set taken (HOP_DENSE_FRACTION raised) and every layer input gathered as a
    # row set (COMPACT_FRACTION 1): the whole frontier chain down to X0's gather on h_L -- full and frontier
    # steps both under the raised fractions (the backward then runs every layer on its hop set either way)
    model_mod = __import__(pkg.__name__ + ".model", fromlist=["model"])
    saved_fr = (model_mod.HOP_DENSE_FRACTION, sh.COMPACT_FRACTION)
    model_mod.HOP_DENSE_FRACTION, sh.COMPACT_FRACTION = 0.95, 1.0
    try:
        outs = []
        for frontier in (False, True):
            m.zero_grad(set_to_none=True)
            m.frontier_forward = frontier
            m(*mine, mode=pkg.KGATMode.TRAIN_CF).backward()
            outs.append([p.grad.detach().clone() for p in m.parameters() if not p.is_sparse and p.grad is not None])
        m.frontier_forward = False
        chain = dict(sh.ROW_SET_STATS)
    finally:
        model_mod.HOP_DENSE_FRACTION, sh.COMPACT_FRACTION = saved_fr
    exact["frontier_vs_full_all_hops"] = len(outs[0]) == len(outs[1]) and all(
        torch.equal(a, b) for a, b in zip(*outs))
    close("cf d table shard (all hops, frontier)", outs[1][0], ref._user_entity_embedding.weight.grad[lo:hi], ATOL_GRAD)
    if world > 1 and rank == 0:
        print(f"sharded_worker world {world}: frontier chain {chain}", flush=True)
    # the table's Adam step fused into its last product (fuse_table_update) vs the unfused step
    snap = {k: v.detach().clone() for k, v in m.state_dict().items()}
    s0, res = m._step, []
    for fuse in (False, True):
        m.load_state_dict(snap)
        m.zero_grad(set_to_none=True)
        m.build_optimizer(1e-3, 1e-4)
        m.fuse_table_update = fuse
        m._step = s0
        m.train()
        m(*mine, mode=pkg.KGATMode.TRAIN_CF).backward()
        m.update_cf_weights()
        st = m._cf_optimizer.state[id(m._user_entity_embedding_shard)]
        res.append([p.detach().clone() for p in m.parameters()] + [st["exp_avg"].clone(), st["exp_avg_sq"].clone()])
    m.fuse_table_update = False
    m.eval()
    exact["fused_table_update"] = all(torch.equal(a, b) for a, b in zip(*res))
    m.load_state_dict(snap)
    users = torch.arange(0, 50, device="cuda")
    items = torch.arange(0, 300, device="cuda")
    with torch.no_grad():
        close("scores", m(users, items, mode=pkg.KGATMode.PREDICT), ref(users, items, mode=pkg.KGATMode.PREDICT),
              1e-5)
    dist.barrier()
    if FAILURES:
        print(f"rank {rank}: " + "; ".join(FAILURES), flush=True)
    else:
        print(f"sharded parity ok: rank {rank}/{world} rows [{lo}, {hi}) d={dim} layers={layers} "
              f"bit-identical {exact}", flush=True)
    dist.destroy_process_group()
    sys.exit(1 if FAILURES else 0)


if __name__ == "__main__":
    main()
