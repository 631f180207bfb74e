"""One rank of the data-parallel replica check (launched by tests/test_gpu_sharded.py through
``python -m torch.distributed.run --nproc-per-node 2`` (or 4); every rank on cuda:0, gloo).

Three replica sets train side by side on the same rank-dependent batches with rank-dependent dropout:
(A) replicas.allreduce_gradients + every rank's full Adam, (B) replicas.ShardedGradSync -- row-block
gradient exchange, Adam on the owned rows, all-gather -- and (C) the same sync attached to the model,
so the table gradient's blocks are exchanged while the backward computes the next block.  With two
ranks every sum has two operands, so all three must agree bit for bit, and each path's replicas must
stay identical.

Two more sets use ``ShardedGradSync(replicate_table=True)`` (the replicas all-gather their compact
layer-0 hop-set terms and each computes the mean table gradient itself): (D) as bench.py runs it, and
(E) with rank 1's backward forced dense (HOP_DENSE_FRACTION = 0 on that rank only), so the ranks
disagree on the hop mode and must fall back to the dense all-reduce together.  Their sums are
associated differently (A^T . mean(dS) instead of mean(A^T . dS)), so they are compared with the
Adam tolerance of DESIGN.md §2, and each path's replicas must stay bit-identical.  (F) is (D) with
``fuse_table_update``: the merged hop-set terms are handed to update_cf_weights, which runs the union
product fused with the table's Adam step -- bit-identical to (D).  (G) is (F) with ``frontier_forward``
(each layer's forward on the rows the loss reaches; it marks the same first hop the exchange
announces early) -- bit-identical to (F): the data-parallel training step bench.py times at N > 1.
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
    rank = dist.get_rank()
    pkg = load_pkg()
    graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])
    rep = __import__(pkg.__name__ + ".replicas", fromlist=["replicas"])
    U, E, inter, trip = graph.synthetic_ckg(20001, 160000, seed=9)  # odd row count: a tail row
    lay = graph.build_layout(U, E, inter, trip)
    # DP_WORKER_DIMS="128:128,64": a 128-wide layer 0 (no fused saved-state backward: its hop set is
    # listed with hop_compact(sync=True), so the compact buffers hold exactly each rank's own count)
    dims = os.environ.get("DP_WORKER_DIMS", "64:64,32")
    d0, layer_size = int(dims.split(":")[0]), [int(x) for x in dims.split(":")[1].split(",")]
    args = pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=layer_size,
                        cf_embedding_dim=d0, kg_embedding_dim=d0, message_dropout=[0.1] * len(layer_size))
    models = []
    model_mod = __import__(pkg.__name__ + ".model", fromlist=["model"])
    for k in range(9):
        torch.manual_seed(3)
        m = pkg.KGAT(args)
        m.attach_graph(lay, "cuda")
        rep.broadcast_parameters(m)
        m.train()
        m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
        m.fuse_table_update = k >= 5
        m.frontier_forward = k in (6, 7)
        models.append(m)
    rng = np.random.default_rng(40 + rank)
    failures = []
    syncs = [None] * 9
    for step in range(3):
        if rank == 0:
            print(f"dp_worker world {dist.get_world_size()} dims {dims}: step {step}", flush=True)
        b = [torch.from_numpy(x).cuda() for x in (rng.integers(0, U, 64), rng.integers(0, E // 10, 64),
                                                  rng.integers(0, E // 10, 64))]
        for k, m in enumerate(models):
            torch.manual_seed(1000 * step + rank)  # same dropout for every path, per rank
            if k and syncs[k] is None:
                params = [p for p in m.parameters() if not p.is_sparse and p.requires_grad]
                syncs[k] = rep.ShardedGradSync(params, replicate_table=3 <= k <= 6, pipeline=k == 8)
                if k >= 2:
                    syncs[k].attach(m)
            frac = model_mod.HOP_DENSE_FRACTION
            if k == 4 and rank == 1:  # rank 1 chooses the dense backward (before its forward, as a rank does)
                model_mod.HOP_DENSE_FRACTION = 0.0
            try:
                loss = m(*b, mode=pkg.KGATMode.TRAIN_CF)
                loss.backward()
            finally:
                model_mod.HOP_DENSE_FRACTION = frac
            params = [p for p in m.parameters() if not p.is_sparse and p.requires_grad]
            if k == 0:
                rep.allreduce_gradients(params)
                m.update_cf_weights()
            else:
                m.update_cf_weights(row_ranges=syncs[k].reduce())
                syncs[k].gather()
            if step == 0:
                with torch.no_grad():  # a loss evaluation without backward opens no exchange
                    m(*b, mode=pkg.KGATMode.TRAIN_CF)
    # a step abandoned at its update (an out-of-range id, reported by update_cf_weights) takes no
    # optimiser step on any path -- the pipelined owner step (I) already ran its block's Adam inside the
    # backward under the device skip flag and takes its step counter back -- and the next good step keeps
    # every path's bits (I still equal to C below)
    for bad in (True, False):
        b = [torch.from_numpy(x).cuda() for x in (rng.integers(0, U, 64), rng.integers(0, E // 10, 64),
                                                  rng.integers(0, E // 10, 64))]
        if bad:
            b[0][5] = U + E + 7
        for k, m in enumerate(models):
            torch.manual_seed(5000 + int(bad) + rank)
            frac = model_mod.HOP_DENSE_FRACTION
            if k == 4 and rank == 1:
                model_mod.HOP_DENSE_FRACTION = 0.0
            try:
                m(*b, mode=pkg.KGATMode.TRAIN_CF).backward()
            finally:
                model_mod.HOP_DENSE_FRACTION = frac
            torch.cuda.synchronize()  # the id check's flag is in: update_cf_weights reports it
            params = [p for p in m.parameters() if not p.is_sparse and p.requires_grad]
            try:
                if k == 0:
                    rep.allreduce_gradients(params)
                    m.update_cf_weights()
                else:
                    m.update_cf_weights(row_ranges=syncs[k].reduce())
                raised = False
            except IndexError:
                raised = True
            if k:
                syncs[k].gather()
            if raised != bad:
                failures.append(f"{'ABCDEFGHI'[k]}: bad-id step raised={raised}")
    for tag, want in (("D", "hop"), ("E", "dense"), ("F", "hop"), ("G", "hop")):
        got = syncs["ABCDEFGHI".index(tag)].stats
        # 2 layers: the layer-0 hop set is the first hop (small); 3 layers: the second hop, which may
        # cross HOP_DENSE_FRACTION -- then every rank agrees on the dense exchange
        if (got.get(want, 0) != 5) if len(layer_size) == 2 else (sum(got.values()) != 5):
            failures.append(f"{tag}: table exchange paths {got}, expected 5 x {want}")
    for named in zip(*(m.named_parameters() for m in models)):
        na, pa = named[0]
        if pa.is_sparse:
            continue
        if not torch.equal(named[3][1].data, named[5][1].data):
            failures.append(f"F {na}: differs from D by {(named[3][1].data - named[5][1].data).abs().max().item():.3e}")
        if not torch.equal(named[5][1].data, named[6][1].data):
            failures.append(f"G {na}: differs from F by {(named[5][1].data - named[6][1].data).abs().max().item():.3e}")
        if not torch.equal(named[2][1].data, named[7][1].data):
            failures.append(f"H {na}: differs from C by {(named[2][1].data - named[7][1].data).abs().max().item():.3e}")
        if not torch.equal(named[2][1].data, named[8][1].data):
            failures.append(f"I {na}: differs from C by {(named[2][1].data - named[8][1].data).abs().max().item():.3e}")
        for tag, (_, po) in zip("BCDE", named[1:5]):
            # two ranks: every sum has two operands, so B / C equal A bit for bit.  More ranks: gloo's ring
            # all-reduce associates an element's G-term sum by the chunk of the buffer it lands in, and C
            # reduces the table gradient block by block (buffers of another size than A's whole-table call),
            # so its sums round differently; Adam then amplifies that rounding on ~eps-sized gradients by up
            # to the Adam tolerance per step (2e-5) -- over the 4 applied steps here, 8e-5.
            # (C, H and I are compared with each other bit for bit above.)
            if tag in "BC" and (not torch.equal(pa.data, po.data) if dist.get_world_size() == 2
                                else not torch.allclose(pa.data, po.data, rtol=0, atol=4 * 2e-5)):
                failures.append(f"{tag} {na}: max |diff| {(pa.data - po.data).abs().max().item():.3e}")
            # D / E associate the table gradient's sums differently at every world size: the same per-step
            # Adam bound over the 4 applied steps
            if tag in "DE" and not torch.allclose(pa.data, po.data, rtol=0, atol=4 * 2e-5):
                failures.append(f"{tag} {na}: max |diff| {(pa.data - po.data).abs().max().item():.3e}")
        for tag, (_, po) in zip("ABCDEFGHI", named):
            other = po.data.clone()
            dist.broadcast(other, 0)
            if not torch.equal(other, po.data):
                failures.append(f"{tag} {na}: replicas diverged")
    print(f"rank {rank}: {'OK' if not failures else failures}", flush=True)
    dist.destroy_process_group()
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
