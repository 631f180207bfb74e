"""KGAT CF training-step benchmark on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]

One step = the reference's hot loop body (src/model/KGAT/main.py:299-316):
full-graph attentive propagation over all L layers, BPR loss on a 256-pair
batch, backward through every layer, dense Adam on the whole model -- in
train mode (dropout on), inputs resident in HBM before timing starts.

value = CKG layer-edges per second of the whole job = n_gpus * E * L / t_step
(weak scaling: every rank runs full propagation for its own batch; for N > 1,
data-parallel replicas, replicas.ShardedGradSync: by default for 2-layer
configs the replicas all-gather their compact layer-0 hop-set gradient terms
over RCCL and each computes the mean table gradient and the full Adam itself
(--dp replicated); otherwise the table gradient is reduce-scattered by row
blocks, each rank runs Adam on its own rows and the rows are all-gathered back
(--dp sharded); small gradients in one flat all-reduce).
Also reported: BPR pairs/s = 256 * n_gpus / t_step, forward-propagation
edges/s, the roofline of the dominant kernel (the SpMM gather, timed live
with HIP events on its launch stream) and the CPU baseline (the oracle's
PyTorch-CPU restatement on the same graph, rank 0 only).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
PKG = "problem-recommender-system-using-kgat-in-codeforces_amd"

# BASELINE.json configs: C2 is the single-GPU headline (configs[1]).
CONFIGS = {
    "c2": dict(nodes=1_000_000, triples=10_000_000, dim=64, layers=[64, 32], batch=256,
               workload="synthetic CKG 1M entities / 10M triples, embed_dim=64, 2 KGAT layers (BASELINE configs[1])"),
    "c4": dict(nodes=10_000_000, triples=100_000_000, dim=128, layers=[128, 64, 32], batch=256,
               workload="synthetic CKG 10M entities / 100M triples, embed_dim=128, 3 KGAT layers (configs[3])"),
    "small": dict(nodes=100_000, triples=1_000_000, dim=64, layers=[64, 32], batch=256,
                  workload="synthetic CKG 100k / 1M (debug)"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def spmm_bytes(n: int, nnz: int, d: int, accumulate: bool) -> int:
    """Algorithmic bytes of one SpMM launch: rowptr (int64), col+val per edge, gathered
    source rows, written output rows (+ read of the accumulated output)."""
    return 8 * (n + 1) + nnz * (8 + 4 * d) + 4 * n * d * (2 if accumulate else 1)


def cpu_baseline(layout, cfg, steps: int = 2) -> dict:
    """The oracle's PyTorch-CPU restatement of one CF step (fwd + bwd + Adam) on the same graph."""
    from oracle import kgat_cpu as K

    torch.set_num_threads(os.cpu_count() or 1)
    threads = torch.get_num_threads()
    n = layout.n_nodes
    rows, cols, vals = layout.coo()
    A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, cols])), torch.from_numpy(vals), (n, n))
    A = A.coalesce()
    g = torch.Generator().manual_seed(0)
    dims = [cfg["dim"], *cfg["layers"]]
    P = {"_user_entity_embedding.weight": torch.randn(n, cfg["dim"], generator=g) * 0.01}
    for l in range(len(cfg["layers"])):
        for w in ("linear1", "linear2"):
            P[f"_aggregator_layers.{l}.{w}.weight"] = torch.randn(dims[l + 1], dims[l], generator=g) * 0.1
            P[f"_aggregator_layers.{l}.{w}.bias"] = torch.zeros(dims[l + 1])
    opt = K.AdamOracle(lr=1e-3)
    times = []
    for _ in range(steps):
        u = torch.randint(0, n // 10, (cfg["batch"],), generator=g)
        p = torch.randint(0, n // 10, (cfg["batch"],), generator=g)
        q = torch.randint(0, n // 10, (cfg["batch"],), generator=g)
        t0 = time.perf_counter()
        leaves = {k: v.requires_grad_(True) for k, v in P.items()}
        loss = K.cf_loss(torch.cat(K.propagate(leaves, A, dropout=[0.1] * len(cfg["layers"]), generator=g), 1),
                         u, p, q)
        loss.backward()
        grads = {k: v.grad for k, v in leaves.items()}
        P = {k: v.detach() for k, v in leaves.items()}
        opt.step(P, grads)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    L = len(cfg["layers"])
    return {"value": layout.nnz * L / t, "unit": "layer-edges/s", "cores": threads, "kind": "port",
            "sample": f"oracle/kgat_cpu.py CF step (fwd+bwd+Adam, dropout on) on the full {cfg['workload']} graph, "
                      f"median of {steps} steps ({t:.2f} s/step), torch CPU threads={threads}",
            "ms_per_step": t * 1e3}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=1)
    ap.add_argument("--dp", choices=("auto", "replicated", "sharded"), default="auto",
                    help="N>1 table-gradient exchange: replicated = all-gather of the compact layer-0 hop-set "
                         "terms, every rank computes the mean gradient and full Adam; sharded = row-block "
                         "reduce-scatter, owned-row Adam, all-gather; auto = replicated for 2-layer configs")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    pkg = importlib.import_module(PKG)
    graph_mod = importlib.import_module(PKG + ".graph")
    kernels = importlib.import_module(PKG + ".kernels")
    replicas = importlib.import_module(PKG + ".replicas")

    t0 = time.perf_counter()
    log(f"generating the synthetic CKG ({cfg['workload']}) ...")
    U, E, inter, trip = graph_mod.synthetic_ckg(cfg["nodes"], cfg["triples"], seed=2024)
    log(f"  {time.perf_counter() - t0:.1f}s; building the layout ...")
    layout = graph_mod.build_layout(U, E, inter, trip)
    log(f"graph: N={layout.n_nodes} interactions={len(inter)} kg={len(trip)} nnz={layout.nnz} "
        f"({time.perf_counter() - t0:.1f}s host build)")
    torch.manual_seed(2024 + rank)
    model = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(layout.rel_order),
                                  cf_embedding_dim=cfg["dim"], kg_embedding_dim=cfg["dim"], layer_size=cfg["layers"],
                                  message_dropout=[0.1] * len(cfg["layers"])))
    log("attaching the graph (device CSR, transpose, refresh plan) ...")
    model.attach_graph(layout, dev)
    log(f"  attached ({time.perf_counter() - t0:.1f}s)")
    replicas.broadcast_parameters(model)  # identical replicas (no-op at N=1)
    model.train()
    model.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    L = len(cfg["layers"])
    B = cfg["batch"]

    # batches (host sampling is outside the hot path, main.py:300-305): uniform users,
    # a positive from the user's interactions, a uniform negative item
    rng = np.random.default_rng(7 + rank)
    order = np.argsort(inter[:, 0], kind="stable")
    su = inter[order]
    ustart = np.searchsorted(su[:, 0], np.arange(U + 1))
    have = np.nonzero(np.diff(ustart) > 0)[0]
    n_items = max(1, int(E * 0.1))
    batches = []
    for _ in range(args.warmup + args.steps):
        u = rng.choice(have, B, replace=len(have) < B)
        k = ustart[u] + (rng.random(B) * (ustart[u + 1] - ustart[u])).astype(np.int64)
        batches.append([torch.from_numpy(x.astype(np.int64)).to(dev)
                        for x in (u, su[k, 1], rng.integers(0, n_items, B))])
    params = [p for p in model.parameters() if not p.is_sparse and p.requires_grad]
    dp_mode = args.dp if args.dp != "auto" else ("replicated" if L <= 2 else "sharded")
    sync = replicas.ShardedGradSync(params, replicate_table=dp_mode == "replicated").attach(model)

    def step(b):
        loss = model(*b, mode=pkg.KGATMode.TRAIN_CF)
        loss.backward()
        # RCCL over xGMI (no-op at N=1): table gradient reduce-scattered by row blocks, Adam on the
        # owned rows, updated rows all-gathered; small gradients in one flat all-reduce
        model.update_cf_weights(row_ranges=sync.reduce())
        sync.gather()
        return loss

    for i in range(args.warmup):
        step(batches[i])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    kernels.SPMM_EVENTS = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(batches[args.warmup + i])
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    events, kernels.SPMM_EVENTS = kernels.SPMM_EVENTS, None
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([elapsed], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    final_loss = float(loss.item())
    ms = elapsed / args.steps * 1e3

    # dominant kernel: the forward SpMM gather A . X (d = embed dim), timed over the timed region; the
    # pipelined forward (kernels.propagate_layer) launches it per row block: bytes and time summed
    n, nnz = layout.n_nodes, layout.nnz
    d0 = cfg["dim"]
    fwd = []  # (ms, d, algorithmic bytes) per forward launch
    for e0, e1, d, tr, acc in events:
        if tr or acc is True or acc in ("masked",):
            continue
        if isinstance(acc, tuple):  # ("block", rows, nnz)
            fwd.append((e0.elapsed_time(e1), d, spmm_bytes(acc[1], acc[2], d, False)))
        elif acc is False:
            fwd.append((e0.elapsed_time(e1), d, spmm_bytes(n, nnz, d, False)))
    bwd = [(e0.elapsed_time(e1), d) for e0, e1, d, tr, acc in events if tr and acc != "masked"]
    masked = [e0.elapsed_time(e1) for e0, e1, d, tr, acc in events if acc == "masked"]
    fwd_d0 = [(t, b) for t, d, b in fwd if d == d0]
    avg_ms = float(np.mean([t for t, _ in fwd_d0]))
    algo = float(np.mean([b for _, b in fwd_d0]))
    achieved = sum(b for _, b in fwd_d0) / (sum(t for t, _ in fwd_d0) * 1e-3) / 1e9
    t_prop = sum(t for t, _, _ in fwd) / args.steps  # ms of SpMM per step, forward
    traffic = None
    pmc = ROOT / "profiles" / f"pmc_{args.config}.json"
    if pmc.exists():
        try:
            traffic = json.loads(pmc.read_text()).get("spmm_fwd_hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None

    result = {
        "metric": "CKG edges/sec (KGAT propagation step) + BPR pairs/sec at 1/2/4/8 MI355X",
        "value": world * nnz * L / (ms * 1e-3),
        "unit": "layer-edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded CKG per SURVEY §8d; random-init weights; no dataset download)",
        "config": {"workload": cfg["workload"], "nodes": n, "nnz": nnz, "interactions": int(len(inter)),
                   "kg_triples": int(len(trip)), "embed_dim": d0, "layer_size": cfg["layers"], "global_batch": B * world,
                   "parallelism": f"dp{world}" if world > 1 else "single",
                   "dp_exchange": dp_mode if world > 1 else None, "mode": "train (dropout 0.1)"},
        "bpr_pairs_per_s": B * world / (ms * 1e-3),
        "final_loss": final_loss,
        "spmm": {"fwd_launches": len(fwd), "bwd_launches": len(bwd), "fwd_avg_ms": avg_ms,
                 "bwd_avg_ms": float(np.mean([t for t, _ in bwd])) if bwd else None,
                 "bwd_masked_launches": len(masked), "bwd_masked_ms_per_step": sum(masked) / args.steps,
                 "fwd_spmm_ms_per_step": t_prop,
                 "fwd_spmm_layer_edges_per_s": nnz * L / (t_prop * 1e-3)},
        "roofline": {"bound": "hbm", "kernel": f"spmm_main_kernel<{d0}, 0> (+fixup), forward A.X"
                     + (" (per row-block launch)" if kernels.FWD_PIPELINE_BLOCKS > 1 else ""),
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "algorithmic_bytes_per_launch": algo},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing the CPU baseline (oracle restatement) ...")
        result["cpu_baseline"] = cpu_baseline(layout, cfg, steps=args.cpu_steps)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
