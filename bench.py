"""KGAT CF training-step benchmark on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4|c5|small] [--scale F]

One step = the reference's hot loop body (src/model/KGAT/main.py:299-316):
full-graph attentive propagation over all L layers, BPR loss on a 256-pair
batch per rank, backward through every layer, dense Adam on the whole model --
in train mode (dropout on), inputs resident in HBM before timing starts.

``--gpus N`` with no WORLD_SIZE in the environment relaunches this script as N
ranks (torch.distributed.run, one process per GPU, 127.0.0.1 rendezvous) before
anything touches the GPU; under the driver's own torchrun launch it checks that
WORLD_SIZE == N.

Configs (BASELINE.json ``configs``):
  c2  (default, configs[1]) 1M nodes / 10M triples, d=64, [64, 32]: the single-GPU
      headline.  N > 1: data-parallel replicas (replicas.ShardedGradSync) -- the
      replicas all-gather their compact layer-0 hop-set gradient terms over RCCL and
      each computes the mean table gradient and the full Adam (--dp replicated), or
      the table gradient is reduce-scattered by row blocks, Adam on owned rows,
      rows all-gathered (--dp sharded).  value = N * E * L / t_step (weak scaling).
  c4  (configs[3]) 10M / 100M, d=128, [128, 64, 32]: DP replicas as c2.
  c5  (configs[4]) 50M / 500M, d=256, [256, 128, 64]: the table row-sharded over the
      ranks (sharded.RowShardedKGAT), each rank builds only its own rows of the graph
      (graph.HashedCKG); needs >= 4 GPUs (memory estimate below; refused otherwise).
      value = E * L / t_step (the whole graph once per step: strong scaling).
  ``--scale F`` shrinks nodes and triples by F (rehearsals; recorded in the config).

Also reported: BPR pairs/s, forward-propagation edges/s, the roofline of the
dominant kernel (the forward SpMM gather: HIP events on its launch stream over the
timed region; counter-measured bytes from profiles/pmc_<config>.json), on rank 0
at N = 1 the CPU baseline (the oracle's PyTorch-CPU restatement of the same step
on the same graph: thread count swept, 1 warm-up, median of --cpu-steps) and, for
c2, a bench-scale parity check of the timed model against the oracle (eval-mode
propagation, CF loss and table gradient on the full graph).
"""
from __future__ import annotations

import argparse
import gc
import importlib
import json
import os
import socket
import subprocess
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
    "c2": dict(nodes=1_000_000, triples=10_000_000, dim=64, layers=[64, 32], batch=256, mode="dp",
               workload="synthetic CKG 1M entities / 10M triples, embed_dim=64, 2 KGAT layers (BASELINE configs[1])"),
    "c3": dict(users=5000, dim=128, layers=[128, 64, 32], batch=256, mode="dp", codeforces=True,
               nfm=dict(embedding_dim=128, hidden_dim=[128, 64, 32], batch=1024, predict_users=64),
               workload="synthetic full-shaped Codeforces (5,000 users, 9,500 problems, 1,913 contests, 37 tags, 28 "
                        "ratings; driver.synthetic_codeforces, train split), embed_dim=128, 3 KGAT layers + NFM head "
                        "(configs[2])"),
    "c4": dict(nodes=10_000_000, triples=100_000_000, dim=128, layers=[128, 64, 32], batch=256, mode="dp",
               workload="synthetic CKG 10M entities / 100M triples, embed_dim=128, 3 KGAT layers (configs[3])"),
    "c5": dict(nodes=50_000_000, triples=500_000_000, dim=256, layers=[256, 128, 64], batch=256, mode="sharded",
               workload="synthetic CKG 50M entities / 500M triples, embed_dim=256, 3 KGAT layers, table row-sharded "
                        "(configs[4])"),
    "small": dict(nodes=100_000, triples=1_000_000, dim=64, layers=[64, 32], batch=256, mode="dp",
                  workload="synthetic CKG 100k / 1M (debug)"),
}
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
GPU_BYTES = 288e9              # HBM3E per MI355X
GPU_BUDGET = 0.85 * GPU_BYTES  # what a config may plan to use (allocator slack, workspaces)
PARITY_TOL = {"emb": 1e-4, "loss_rel": 1e-4, "grad": 1e-6}  # north_star: 1e-4 fp32 (gradients as in tests/)
EVENT_EVERY = 1  # --event-every


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def spmm_bytes(n: int, nnz: int, d: int, accumulate: bool) -> int:
    """Algorithmic bytes of one SpMM launch: rowptr (int64), col+val per edge, one gathered
    source row per edge, written output rows (+ read of the accumulated output)."""
    return 8 * (n + 1) + nnz * (8 + 4 * d) + 4 * n * d * (2 if accumulate else 1)


CACHE_RESIDENT_BYTES = 64 << 20  # tables up to this size are served from L2 / the Infinity Cache (256 MiB)
L2_GATHER_PEAK_GBS = 18800.0      # MI355X_MICROARCH.md: gathered rows served from the XCDs' L2, chip-wide


def compulsory_bytes(n: int, nnz: int, d: int) -> int:
    """Bytes one SpMM launch cannot avoid: rowptr, col+val, every source row read once, output written."""
    return 8 * (n + 1) + 8 * nnz + 8 * n * d


def sharded_bytes_per_gpu(cfg: dict, world: int) -> float:
    """Planned HBM per rank of the row-sharded mode (sharded.RowShardedKGAT) -- the buffers its step allocates,
    largest shard ~1.15x the mean.  Per local node row (fp32): X0, its gradient and the CF Adam m / v (4d),
    the layer outputs H_l and sides S_l, the wide (GEMM) layers' pre-activation state (2 d_out + 1 per
    layer), three backward temporaries of the widest layer.  Per local edge: the rows of A and of A^T (col
    + val each) and the refresh's two position maps (24 B).  Per node of the whole graph: the gathered
    layer inputs -- the pipelined forward keeps layer l's gathered input and layer l+1's, being posted
    block by block, alive together (sharded._layer_pipelined): max_l (d_l + d_(l+1)) floats -- and the
    batch-row map."""
    import importlib as _il
    kern = _il.import_module(PKG + ".kernels")
    d, layers = cfg["dim"], cfg["layers"]
    dims = [d, *layers]
    gemm_state = sum(2 * b + 1 for a, b in zip(dims[:-1], dims[1:]) if not kern.fused_supported(a, b))
    per_row = 4 * (4 * d + sum(layers) + sum(dims[:-1]) + gemm_state + 3 * max(dims))
    nnz = 2 * cfg["triples"]
    per_rank_rows = 1.15 * cfg["nodes"] / world
    per_rank_edges = 1.15 * nnz / world
    pairs = [dims[l] + dims[l + 1] for l in range(len(layers) - 1)] or [d]
    gathered = 4 * max(pairs) if world > 1 else 0
    return per_row * per_rank_rows + 24 * per_rank_edges + (gathered + 4) * cfg["nodes"]


def min_gpus(cfg: dict) -> int:
    for g in (1, 2, 4, 8, 16, 32):
        if sharded_bytes_per_gpu(cfg, g) <= GPU_BUDGET:
            return g
    return 64


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n: int) -> int:
    """Relaunch this script as n ranks (one process per GPU) and return the launcher's exit code.
    Runs before anything initialises HIP in this process (a GPU-initialised process must not exec)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(Path(__file__).resolve()),
           *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


# --------------------------------------------------------------------------- CPU leg (oracle)
def _oracle_params(layout, cfg, state: dict | None):
    """Flat reference-keyed parameters on the CPU: the GPU model's (state) or seeded random ones."""
    if state is not None:
        return {k: v.detach().float().cpu().clone() for k, v in state.items()}
    g = torch.Generator().manual_seed(0)
    dims = [cfg["dim"], *cfg["layers"]]
    P = {"_user_entity_embedding.weight": torch.randn(layout.n_nodes, cfg["dim"], generator=g) * 0.01}
    for l in range(len(cfg["layers"])):
        for w in ("linear1", "linear2"):
            P[f"_aggregator_layers.{l}.{w}.weight"] = torch.randn(dims[l + 1], dims[l], generator=g) * 0.1
            P[f"_aggregator_layers.{l}.{w}.bias"] = torch.zeros(dims[l + 1])
    return P


def _sweep_threads(A, n: int, d: int) -> tuple[int, dict]:
    """Fastest torch CPU thread count for the step's dominant op (A . X, d wide) on this host."""
    cands = sorted({t for t in (8, 16, 32, 64, 128) if t <= (os.cpu_count() or 1)} | {min(8, os.cpu_count() or 1)})
    X = torch.randn(n, d)
    res = {}
    for t in cands:
        torch.set_num_threads(t)
        best = float("inf")
        for _ in range(2):
            t0 = time.perf_counter()
            torch.sparse.mm(A, X)
            best = min(best, time.perf_counter() - t0)
        res[t] = best
    return min(res, key=res.get), res


def cpu_leg(layout, cfg, steps: int, parity_state: dict | None = None, parity_batch=None,
            parity_gpu: dict | None = None) -> tuple[dict, dict | None]:
    """The oracle's PyTorch-CPU CF step (fwd + bwd + Adam) on the same graph: threads swept, then
    one warm-up step -- the parity step when the GPU's weights are given (eval mode, compared with
    the GPU's propagation / loss / table gradient) -- then the median of `steps` train-mode steps."""
    from oracle import kgat_cpu as K

    n = layout.n_nodes
    rows, cols, vals = layout.coo()
    A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, cols])), torch.from_numpy(vals), (n, n)).coalesce()
    threads, sweep = _sweep_threads(A, n, cfg["dim"])
    torch.set_num_threads(threads)
    L = len(cfg["layers"])
    B = cfg["batch"]
    opt = K.AdamOracle(lr=1e-3)
    parity = None

    def one_step(P, u, p, q, dropout):
        leaves = {k: v.requires_grad_(True) for k, v in P.items()}
        outs = K.propagate(leaves, A, dropout=dropout, generator=g)
        loss = K.cf_loss(torch.cat(outs, 1), u, p, q)
        loss.backward()
        grads = {k: v.grad for k, v in leaves.items()}
        newP = {k: v.detach() for k, v in leaves.items()}
        opt.step(newP, grads)
        return newP, outs, loss, grads

    g = torch.Generator().manual_seed(1)
    P = _oracle_params(layout, cfg, parity_state)
    t0 = time.perf_counter()
    if parity_state is not None:  # warm-up = the parity step
        u, p, q = (t.cpu() for t in parity_batch)
        P, outs, loss, grads = one_step(P, u, p, q, None)
        emb = max(float((o.detach() - gpu).abs().max()) for o, gpu in zip(outs, parity_gpu["tables"]))
        gref = grads["_user_entity_embedding.weight"]
        gerr = float((gref - parity_gpu["table_grad"]).abs().max())
        lrel = abs(float(loss) - parity_gpu["loss"]) / max(abs(float(loss)), 1e-30)
        parity = {"max_abs_emb": emb, "max_abs_grad": gerr, "max_abs_grad_ref": float(gref.abs().max()),
                  "loss_rel": lrel, "loss": parity_gpu["loss"], "loss_oracle": float(loss),
                  "tolerance": PARITY_TOL,
                  "pass": bool(emb <= PARITY_TOL["emb"] and gerr <= PARITY_TOL["grad"] and lrel <= PARITY_TOL["loss_rel"]),
                  "what": "eval-mode propagation of every layer, CF loss and table gradient of the timed model "
                          "(after the timed steps) vs oracle/kgat_cpu.py on the full graph, one 256-pair batch"}
        del outs, grads
    else:
        u = torch.randint(0, n // 10, (B,), generator=g)
        P, *_ = one_step(P, u, u, u, [0.1] * L)
    warm = time.perf_counter() - t0
    times = []
    for _ in range(steps):
        u, p, q = (torch.randint(0, n // 10, (B,), generator=g) for _ in range(3))
        t0 = time.perf_counter()
        P, *_ = one_step(P, u, p, q, [0.1] * L)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    base = {"value": layout.nnz * L / t, "unit": "layer-edges/s", "cores": threads, "kind": "port",
            "sample": f"oracle/kgat_cpu.py CF step (fwd+bwd+Adam, dropout 0.1) on the full {cfg['workload']} graph, "
                      f"median of {steps} after 1 warm-up ({warm:.1f} s), threads={threads} (best of sweep "
                      + ", ".join(f"{k}:{v * 1e3:.0f}ms" for k, v in sweep.items()) + " on A.X)",
            "ms_per_step": t * 1e3, "step_times_s": times}
    return base, parity


def cpu_extrapolated(layout, cfg, fracs=(0.02, 0.04)) -> dict:
    """C4-size CPU baseline: the oracle CF step on uniformly subsampled edge sets (all N rows kept),
    extrapolated linearly in E to the full graph ("extrapolated").  At 10M rows the step is dominated by
    the dense per-row work, so two whole-step times differ by less than their noise (a fitted slope
    came out negative once); the per-edge slope is therefore taken from the sparse product itself:
    A . X timed at both subsamples (best of 3), times the step's 2 * sum_l d_in(l) / d0 products'
    worth of gathered width (forward + backward of every layer)."""
    from oracle import kgat_cpu as K

    n = layout.n_nodes
    rows, cols, vals = layout.coo()
    rng = np.random.default_rng(5)
    pts = []
    ax = []  # A . X seconds (d0 wide) per subsample
    threads = None
    for f in fracs:
        keep = np.flatnonzero(rng.random(rows.size) < f)
        A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows[keep], cols[keep]])),
                                    torch.from_numpy(vals[keep]), (n, n)).coalesce()
        if threads is None:
            threads, _ = _sweep_threads(A, n, cfg["dim"])
            torch.set_num_threads(threads)
        Xp = torch.randn(n, cfg["dim"])
        best = float("inf")
        for _ in range(3):
            t0 = time.perf_counter()
            torch.sparse.mm(A, Xp)
            best = min(best, time.perf_counter() - t0)
        ax.append(best)
        del Xp
        P = _oracle_params(layout, cfg, None)
        g = torch.Generator().manual_seed(2)
        ts = []
        for it in range(2):  # warm-up + one timed step
            log(f"  CPU baseline: {f:.0%} edge subsample, {'warm-up' if it == 0 else 'timed'} step ...")
            u, p, q = (torch.randint(0, n // 10, (cfg["batch"],), generator=g) for _ in range(3))
            t0 = time.perf_counter()
            leaves = {k: v.requires_grad_(True) for k, v in P.items()}
            loss = K.cf_loss(torch.cat(K.propagate(leaves, A, dropout=[0.1] * len(cfg["layers"]), generator=g), 1),
                             u, p, q)
            loss.backward()
            grads = {k: v.grad for k, v in leaves.items()}
            P = {k: v.detach() for k, v in leaves.items()}
            K.AdamOracle(lr=1e-3).step(P, grads)
            ts.append(time.perf_counter() - t0)
        pts.append((A._nnz(), ts[-1]))
        del A
    (e1, t1), (e2, t2) = pts
    b_fit = (t2 - t1) / max(e2 - e1, 1)
    dims_in = [cfg["dim"]] + list(cfg["layers"][:-1])
    widths = 2.0 * sum(dims_in) / cfg["dim"]
    b_ax = max(ax[1] - ax[0], 0.0) / max(e2 - e1, 1)
    b = b_ax * widths
    t = max(t1, t2) + b * (layout.nnz - e2)
    L = len(cfg["layers"])
    return {"value": layout.nnz * L / t, "unit": "layer-edges/s", "cores": threads, "kind": "port",
            "extrapolated": True, "ms_per_step": t * 1e3, "per_edge_s": b, "per_edge_s_step_fit": b_fit,
            "sample": f"oracle/kgat_cpu.py CF step on {', '.join(f'{e:,}' for e, _ in pts)}-edge uniform subsamples "
                      f"of the {cfg['workload']} graph (all {n:,} rows; {', '.join(f'{s:.1f}' for _, s in pts)} s/step "
                      f"after 1 warm-up each), + the remaining {layout.nnz - e2:,} edges at the A.X per-edge cost "
                      f"({', '.join(f'{x * 1e3:.0f}' for x in ax)} ms per d0-wide product at the two subsamples) x "
                      f"{widths:g} products' width per step; threads={threads}"}


# --------------------------------------------------------------------------- roofline
def roofline(events, cfg_name: str, n: int, nnz: int, d0: int, steps: int, kernel: str) -> tuple[dict, dict]:
    fwd = []  # (ms, d, algorithmic bytes, compulsory bytes) per forward launch
    for e0, e1, d, tr, acc in events:
        if tr or acc is True or acc in ("masked",):
            continue
        if isinstance(acc, tuple):  # ("block", rows, nnz[, accumulate])
            a = bool(acc[3]) if len(acc) > 3 else False
            fwd.append((e0.elapsed_time(e1), d, spmm_bytes(acc[1], acc[2], d, a), compulsory_bytes(acc[1], acc[2], d)))
        elif acc is False:
            fwd.append((e0.elapsed_time(e1), d, spmm_bytes(n, nnz, d, False), compulsory_bytes(n, nnz, d)))
    bwd = [(e0.elapsed_time(e1), d) for e0, e1, d, tr, acc in events if tr and acc not in ("masked", "fused_adam")]
    masked = [e0.elapsed_time(e1) for e0, e1, d, tr, acc in events if acc in ("masked", "fused_adam")]
    fused = [(e0.elapsed_time(e1), d) for e0, e1, d, tr, acc in events if acc == "fused_adam"]
    # the layer-0 launches (d0 wide; the row-sharded mode's gathered column chunks are narrower)
    fwd_d0 = [x for x in fwd if x[1] == d0] or [x for x in fwd if x[1] == max(y[1] for y in fwd)]
    avg_ms = float(np.mean([x[0] for x in fwd_d0]))
    algo = float(np.mean([x[2] for x in fwd_d0]))
    comp = float(np.mean([x[3] for x in fwd_d0]))
    t_prop = sum(x[0] for x in fwd) / steps
    traffic, pmc_src, rec = None, None, {}
    pmc = ROOT / "profiles" / f"pmc_{cfg_name}.json"
    if pmc.exists():
        try:
            rec = json.loads(pmc.read_text())
            # the counters are per launch of this config at full size: a scaled or sharded rehearsal
            # (other n / nnz per launch) must not borrow them
            if rec.get("nodes", n) == n and rec.get("nnz", nnz) == nnz:
                traffic = rec.get("spmm_fwd_hbm_bytes_per_launch")
                pmc_src = str(pmc.relative_to(ROOT))
        except Exception:  # noqa: BLE001
            traffic = None
    algo_gbs = algo / (avg_ms * 1e-3) / 1e9
    if traffic:
        achieved, basis = traffic / (avg_ms * 1e-3) / 1e9, "counters"
    else:  # no PMC pass for this config: the bytes the launch cannot avoid (a lower bound, <= 1 by construction)
        achieved, basis = comp / (avg_ms * 1e-3) / 1e9, "compulsory (lower bound; no PMC pass for this config)"
    roof = {"bound": "hbm", "kernel": kernel, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "basis": basis, "pmc_source": pmc_src,
            "avg_launch_ms": avg_ms,
            "algorithmic_bytes_per_launch": algo, "algorithmic_GBps": algo_gbs,
            "algorithmic_frac": algo_gbs / HBM_PEAK_GBS,
            "compulsory_bytes_per_launch": comp, "compulsory_frac": comp / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "note": "achieved = counter-measured bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, rocprofv3 --pmc on "
                    "this kernel build) / live HIP-event launch time; the SURVEY §8d algorithmic formula prices "
                    "every gathered row as an HBM read although Zipf hub rows are served from L2 / the Infinity "
                    "Cache, so algorithmic_frac can exceed 1; compulsory = each source row read once"}
    if 4 * n * d0 <= CACHE_RESIDENT_BYTES:
        # a table this small stays in the XCDs' L2s and the Infinity Cache: the gathers never reach HBM
        # after the first touch, so the HBM fraction says nothing; the bound is the cache's row-gather rate
        roof["cache_roofline"] = {
            "level": "L2 / Infinity Cache", "achieved": algo_gbs, "peak": L2_GATHER_PEAK_GBS, "unit": "GB/s",
            "frac": algo_gbs / L2_GATHER_PEAK_GBS, "table_bytes": 4 * n * d0,
            "peak_source": "MI355X_MICROARCH.md 'Indexed rows: gather into LDS': rows shared by every workgroup "
                           "(the XCD's L2) 16.8-18.8 TB/s chip-wide; the upper figure is the peak used"}
    spmm = {"fwd_launches": len(fwd), "bwd_launches": len(bwd), "fwd_avg_ms": avg_ms,
            "bwd_avg_ms": float(np.mean([t for t, _ in bwd])) if bwd else None,
            "bwd_masked_launches": len(masked), "bwd_masked_ms_per_step": sum(masked) / steps,
            "fwd_spmm_ms_per_step": t_prop, "fwd_spmm_layer_edges_per_s": None}
    if fused:
        # the layer-0 A^T product fused with the table's Adam step: HBM-bound on the Adam stream
        # (read + write of p, m, v: 24 B / parameter) plus the product's index scan; counter bytes
        # from the same PMC file when it has them
        ms = float(np.mean([t for t, _ in fused]))
        d = fused[0][1]
        adam_b = 24 * n * d
        scan_b = 8 * (n + 1) + 8 * nnz
        tu = {"kernel": f"spmm_main_kernel<{d}, 4> (+fixup): masked A^T.dS0 + table Adam", "avg_launch_ms": ms,
              "launches_per_step": len(fused) / steps, "adam_bytes": adam_b, "scan_bytes": scan_b,
              "min_bytes_GBps": (adam_b + scan_b) / (ms * 1e-3) / 1e9}
        tu["min_bytes_frac"] = tu["min_bytes_GBps"] / HBM_PEAK_GBS
        tb = rec.get("table_update_hbm_bytes_per_launch") if traffic else None
        if tb:
            tu["traffic"] = tb
            tu["counter_GBps"] = tb / (ms * 1e-3) / 1e9
            tu["counter_frac"] = tu["counter_GBps"] / HBM_PEAK_GBS
        spmm["table_update"] = tu
    return roof, spmm


# --------------------------------------------------------------------------- timing
def timed(step, batches, warmup: int, steps: int, world: int, dev, wire_log=None):
    """Warm-up steps, then ``steps`` timed steps (max over ranks).  ``wire_log`` (comm.WireLog): its byte
    counts are taken over the timed steps only (``timed.wire_bytes``)."""
    kernels = importlib.import_module(PKG + ".kernels")
    for i in range(warmup):
        step(batches[i])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    if wire_log is not None:
        wire_log.reset()
    # HIP events around the SpMM launches of every EVENT_EVERY-th timed step (each record costs the
    # stream a few us; --event-every 1 instruments every step)
    events_all = []
    timed.instrumented = 0
    t0 = time.perf_counter()
    loss = None
    host = []  # host time of each step's launches (the GPU runs behind; no synchronisation inside)
    for i in range(steps):
        on = i % EVENT_EVERY == 0
        kernels.SPMM_EVENTS = events_all if on else None
        timed.instrumented += int(on)
        h0 = time.perf_counter()
        loss = step(batches[warmup + i])
        host.append(time.perf_counter() - h0)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    events, kernels.SPMM_EVENTS = events_all, None
    if world > 1:
        tt = torch.tensor([elapsed], device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(tt.item())
    timed.host_ms_per_step = float(np.median(host)) * 1e3
    timed.wire_bytes = dict(wire_log.bytes) if wire_log is not None else None
    return elapsed, events, float(loss.item())


def run_dp(args, cfg, world: int, rank: int, dev) -> dict:
    """c2 / c4: every rank holds the whole graph; data-parallel replicas for N > 1."""
    pkg = importlib.import_module(PKG)
    graph_mod = importlib.import_module(PKG + ".graph")
    replicas = importlib.import_module(PKG + ".replicas")
    t0 = time.perf_counter()
    log(f"generating the synthetic CKG ({cfg['workload']}) ...")
    ds = None
    if cfg.get("codeforces"):
        # C3: the Codeforces-shaped dataset driver.py trains on (no real data here), its train split
        driver = importlib.import_module(PKG + ".driver")
        ci, trip, E = driver.synthetic_codeforces(users=cfg["users"], seed=2024)
        U = cfg["users"]
        tr, va, te = driver.split_interactions(ci, U)
        ds = driver.Dataset(U, E, 9500, tr, va, te, trip)
        inter = tr
    else:
        U, E, inter, trip = graph_mod.synthetic_ckg(cfg["nodes"], cfg["triples"], seed=2024)
    log(f"  {time.perf_counter() - t0:.1f}s; building the layout ...")
    layout = graph_mod.build_layout(U, E, inter, trip)
    log(f"graph: N={layout.n_nodes} interactions={len(inter)} kg={len(trip)} nnz={layout.nnz} "
        f"({time.perf_counter() - t0:.1f}s host build)")
    torch.manual_seed(2024 + rank)
    L = len(cfg["layers"])
    model = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(layout.rel_order),
                                  cf_embedding_dim=cfg["dim"], kg_embedding_dim=cfg["dim"], layer_size=cfg["layers"],
                                  message_dropout=[0.1] * L))
    log("attaching the graph (device CSR, transpose, refresh plan) ...")
    model.attach_graph(layout, dev)
    log(f"  attached ({time.perf_counter() - t0:.1f}s)")
    replicas.broadcast_parameters(model)  # identical replicas (no-op at N=1)
    model.train()
    model.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    # the table gradient's layer-0 A^T product runs fused with the table's Adam step inside
    # update_cf_weights (same bits; --no-fused-update: product and Adam as two passes)
    model.fuse_table_update = not args.no_fused_update
    model.direct_backward = True  # the timed loop's plain loss.backward() (no DDP wrapper; model._StepLoss)
    B = cfg["batch"]
    # batches (host sampling is outside the hot path, main.py:300-305): uniform users,
    # a positive from the user's interactions, a uniform negative item
    rng = np.random.default_rng(7 + rank)
    order = np.argsort(inter[:, 0], kind="stable")
    su = inter[order]
    ustart = np.searchsorted(su[:, 0], np.arange(U + 1))
    have = np.nonzero(np.diff(ustart) > 0)[0]
    n_items = ds.item_num if ds is not None else max(1, int(E * 0.1))
    batches = []
    for _ in range(args.warmup + args.steps):
        u = rng.choice(have, B, replace=len(have) < B)
        k = ustart[u] + (rng.random(B) * (ustart[u + 1] - ustart[u])).astype(np.int64)
        batches.append([torch.from_numpy(x.astype(np.int64)).to(dev)
                        for x in (u, su[k, 1], rng.integers(0, n_items, B))])
    params = [p for p in model.parameters() if not p.is_sparse and p.requires_grad]
    dp_mode = args.dp if args.dp != "auto" else ("replicated" if L <= 2 else "sharded")
    # sharded mode: each owner's block Adam + broadcast pipelined inside the backward (ShardedGradSync.pipeline)
    sync = replicas.ShardedGradSync(params, replicate_table=dp_mode == "replicated", force=args.exchange_at_1,
                                    pipeline=dp_mode == "sharded").attach(model)

    def step(b):
        loss = model(*b, mode=pkg.KGATMode.TRAIN_CF)
        loss.backward()
        # RCCL over xGMI (no-op at N=1): the table-gradient exchange of --dp, small gradients in
        # one flat all-reduce
        model.update_cf_weights(row_ranges=sync.reduce())
        sync.gather()
        return loss

    elapsed, events, final_loss = timed(step, batches, args.warmup, args.steps, world, dev)
    exchange_steps = dict(sync.stats)  # the full-propagation run's table exchanges (warm-up + timed)
    ms = elapsed / args.steps * 1e3
    n, nnz, d0 = layout.n_nodes, layout.nnz, cfg["dim"]
    roof, spmm = roofline(events, args.config, n, nnz, d0, timed.instrumented,
                          f"spmm_main_kernel<{d0}, 0> (+fixup), forward A.X")
    spmm["fwd_spmm_layer_edges_per_s"] = nnz * L / (spmm["fwd_spmm_ms_per_step"] * 1e-3)
    spmm["event_steps"] = timed.instrumented  # timed steps whose SpMM launches carry HIP events
    result = {
        "value": world * nnz * L / (ms * 1e-3), "n_gpus": world, "ms_per_step": ms, "scaling": "weak",
        "config": {"workload": cfg["workload"], "nodes": n, "nnz": nnz, "interactions": int(len(inter)),
                   "kg_triples": int(len(trip)), "embed_dim": d0, "layer_size": cfg["layers"],
                   "global_batch": B * world, "parallelism": f"dp{world}" if world > 1 else "single",
                   "dp_exchange": dp_mode if world > 1 else None, "mode": "train (dropout 0.1)",
                   "table_update": "unfused" if args.no_fused_update else "fused layer-0 A^T product + Adam"},
        "bpr_pairs_per_s": B * world / (ms * 1e-3), "final_loss": final_loss, "spmm": spmm, "roofline": roof,
        "host_launch_ms_per_step": timed.host_ms_per_step,
        "cpu_baseline": None,
    }
    if L <= 3 and not args.no_frontier_leg and not args.exchange_at_1:
        # the same CF step with KGAT.frontier_forward (each layer's forward on the rows the loss can
        # reach only: same loss, gradients and updates bit for bit, tested) -- the training step as
        # driver.py runs it; `value` above stays the full-propagation step.  N > 1: the replicas'
        # replicated hop-set exchange composes with it (both mark the same first hop before the
        # propagation); its BPR pairs/s is the data-parallel training throughput.
        model.frontier_forward = True
        before = dict(sync.stats)
        fel, _, _ = timed(step, batches, args.warmup, args.steps, world, dev)
        model.frontier_forward = False
        fr_exchange = {k: v - before.get(k, 0) for k, v in sync.stats.items()}
        fms = fel / args.steps * 1e3
        # bit identity vs the full forward: checked here at N = 1 (and, with the exchange, in tests/dp_worker.py)
        same = frontier_matches_full(model, pkg, batches[0]) if world == 1 else None
        est = getattr(model.graph(), "_hop_est", {}).get(L - 2)  # pinned count of the last step's first hop
        result["frontier_forward"] = {
            "ms_per_step": fms, "bpr_pairs_per_s": B * world / (fms * 1e-3), "speedup_vs_full": ms / fms,
            "first_hop_rows_last_step": int(est[0][0]) if est is not None and L >= 2 else None,
            "host_launch_ms_per_step": timed.host_ms_per_step,
            "bit_identical_to_full": same,
            "note": "TRAIN_CF forward restricted to the rows the BPR loss reaches (layer L-2 on the first hop "
                    "F + N(F), the last layer on the batch rows F, layer 0 of 3 whole); not counted in value (it "
                    "does not visit every edge)"}
        if world > 1:
            result["frontier_forward"]["dp_table_exchange_steps"] = fr_exchange
    result["value_note"] = ("value = n_gpus x nnz x L / t_step: each data-parallel replica runs the reference step's "
                            "full propagation over every edge for its own 256-pair batch (weak scaling; replicas "
                            "repeat the same graph's work); bpr_pairs_per_s (and frontier_forward.bpr_pairs_per_s, "
                            "the training step driver.py runs) is the job's training throughput")
    if world > 1 or args.exchange_at_1:
        result["dp_table_exchange_steps"] = exchange_steps
    if args.exchange_at_1:
        result["config"]["dp_exchange"] = dp_mode
        result["rehearsal"] = ("the N-rank table exchange forced at world 1 over RCCL (collectives move no data "
                               "between GPUs): its GPU + host overhead per step, not a scaling measurement")
    if world == 1 and not args.no_kg_leg and not args.exchange_at_1:
        cf_ms = result.get("frontier_forward", {}).get("ms_per_step", ms)
        result["kg_refresh"] = kg_refresh_legs(model, pkg, layout, cfg, args, dev, len(inter), cf_ms)
    if ds is not None and cfg.get("nfm") and world == 1:
        result["nfm"] = nfm_legs(ds, cfg, args, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if cfg.get("nodes", 0) > 2_000_000:
            log("timing the CPU baseline (oracle restatement on subsampled edge sets, extrapolated) ...")
            result["cpu_baseline"] = cpu_extrapolated(layout, cfg)
        else:
            parity_in = None
            if not args.no_parity:
                log("bench-scale parity: eval-mode propagation / CF loss / table gradient on the GPU ...")
                parity_in = gpu_parity_inputs(model, pkg, batches[0])
            log("timing the CPU baseline (oracle restatement; warm-up step = the parity check) ...")
            base, parity = cpu_leg(layout, cfg, args.cpu_steps, *(parity_in or (None, None, None)))
            result["cpu_baseline"] = base
            result["parity"] = parity
    return result


FP32_MFMA_PEAK_TFS = 157.3  # MI355X dense fp32 matrix peak (MI355X_MICROARCH.md chip table)


def _event_ms(evs: dict, name: str) -> list[float]:
    return [a.elapsed_time(b) for a, b in evs.get(name, [])]


def kg_refresh_legs(model, pkg, layout, cfg, args, dev, n_interactions: int, cf_ms: float) -> dict:
    """The reference epoch's other two phases at this config:
    TRAIN_KG + update_kg_weights at the reference's B = 512 (main.py:324-345) -- with the fused KG
    table update (the table's Adam from TransR's compact rows, kgat_adam_rows_f32) and without it
    (dense [N, d] gradient + Adam, the reference's arithmetic) -- and UPDATE_ATTENTION (main.py:350-361,
    train mode: MHA dropout on, as the reference runs it).  Kernel times come from HIP events on the
    launch stream (kernels.KERNEL_EVENTS); rooflines: the table Adam against HBM (24 B per parameter
    + 4 B per row fused, 28 B per parameter dense), the edge scorer against the fp32 MFMA peak
    (6 d^2 flop per edge: e_t W_r, W_v, W_o).  epoch_estimate = (interactions // 256 + 1) CF steps
    (the training step: frontier forward when measured) + (edges // 512 + 1) KG steps + 1 refresh
    (main.py:297, 324)."""
    kernels = importlib.import_module(PKG + ".kernels")
    B = 512
    n, d = layout.n_nodes, cfg["dim"]
    E = int(layout.heads.size)
    rng = np.random.default_rng(11)
    # a KG step is ~0.1-0.3 ms: time at least 100 of them (the default 20 would be ~3 ms of work, short
    # enough for the clock ramp after the previous leg's sync to show); 32 distinct batches, cycled
    steps = max(args.steps, 100)
    batches = []
    for _ in range(32):
        e = rng.integers(0, E, B)
        batches.append([torch.from_numpy(np.asarray(x, np.int64)).to(dev)
                        for x in (layout.heads[e], layout.rels[e], layout.tails[e], rng.integers(0, n, B))])

    def kg_step(b):
        loss = model(*b, mode=pkg.KGATMode.TRAIN_KG)
        loss.backward()
        model.update_kg_weights()
        return loss

    out = {"batch": B}
    for tag, fused, lazy, cap in (("captured", True, True, True), ("lazy", True, True, False),
                                  ("fused", True, False, False), ("unfused", False, False, False)):
        model.fuse_kg_table_update = fused
        model.lazy_kg_adam = lazy
        model.capture_kg_step = cap
        for i in range(args.warmup):
            kg_step(batches[i % 32])
        torch.cuda.synchronize()
        # the step time without instrumentation (an event pair around every kernel costs the stream
        # and the host ~10-20 us each: it would be most of a 0.3 ms step), then the kernels' own times
        # from an instrumented pass over the same batches
        t0 = time.perf_counter()
        for i in range(steps):
            kg_step(batches[(args.warmup + i) % 32])
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps * 1e3
        kernels.KERNEL_EVENTS = {}
        for i in range(8):
            kg_step(batches[(args.warmup + i) % 32])
        torch.cuda.synchronize()
        evs, kernels.KERNEL_EVENTS = kernels.KERNEL_EVENTS, None
        leg = {"ms_per_step": el, "kg_pairs_per_s": B / (el * 1e-3)}
        if cap:
            leg["graph_replays"] = model._kg_graph.replays
            model.capture_kg_step = False
        if lazy:
            # the flush that brings every row current (before the next CF step): here after the leg's
            # warmup + 2 x steps KG steps, i.e. that many zero-gradient steps replayed for almost every row
            pend = args.warmup + steps + 8
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            model.flush_kg_table()
            torch.cuda.synchronize()
            leg["flush_ms"] = (time.perf_counter() - t1) * 1e3
            leg["flush_steps_pending"] = pend
            model.lazy_kg_adam = False
        for k in ("transr_fwd", "transr_bwd", "adam_rows", "adam_multi"):
            t = _event_ms(evs, k)
            if t:
                leg[f"{k}_avg_ms"] = float(np.mean(t))
        if fused:
            t = leg.get("adam_rows_avg_ms")
            if t:
                by = 24 * n * d + 4 * n
                leg["roofline"] = {"kernel": "adam_rows_kernel (table Adam from the compact TransR rows)", "bound": "hbm",
                                   "bytes_per_launch": by, "achieved": by / (t * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": by / (t * 1e-3) / 1e9 / HBM_PEAK_GBS}
        else:
            t = leg.get("adam_multi_avg_ms")
            if t:
                # the KG step's gradients: table, relation embeddings, trans matrices (model.py:414-419)
                by = 28 * (n * d + model._relation_embedding.weight.numel() + model._trans_matrix.numel())
                leg["roofline"] = {"kernel": "adam_multi_kernel<2> (dense table gradient)", "bound": "hbm",
                                   "bytes_per_launch": by, "achieved": by / (t * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": by / (t * 1e-3) / 1e9 / HBM_PEAK_GBS}
        out[tag] = leg
    model.fuse_kg_table_update = True
    out["speedup_fused"] = out["unfused"]["ms_per_step"] / out["fused"]["ms_per_step"]
    # UPDATE_ATTENTION on the whole edge list; A's values are restored afterwards (later legs compare
    # the timed model with the oracle on the layout's initial values)
    g = model.graph()
    saved = g.A.val.detach().clone()
    att = [torch.from_numpy(np.asarray(x, np.int64)).to(dev) for x in (layout.heads, layout.rels, layout.tails)]
    att.append(torch.tensor(layout.rel_order))
    model.train()
    model(*att, mode=pkg.KGATMode.UPDATE_ATTENTION)  # warm-up (builds the refresh plan)
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        model(*att, mode=pkg.KGATMode.UPDATE_ATTENTION)
    torch.cuda.synchronize()
    rms = (time.perf_counter() - t0) / reps * 1e3
    kernels.KERNEL_EVENTS = {}
    model(*att, mode=pkg.KGATMode.UPDATE_ATTENTION)
    torch.cuda.synchronize()
    evs, kernels.KERNEL_EVENTS = kernels.KERNEL_EVENTS, None
    g = model.graph()
    g.A.val.copy_(saved)
    g.refresh_transpose()
    ref = {"ms_per_call": rms, "edges": E, "edges_per_s": E / (rms * 1e-3)}
    t = _event_ms(evs, "edge_scores")
    if t:
        flops = 6.0 * d * d * E
        ref["edge_scores_avg_ms"] = float(np.mean(t))
        ref["roofline"] = {"kernel": "edge scorer (e_t W_r, W_v, W_o on the fp32 MFMA)", "bound": "mfma",
                           "flops_per_launch": flops, "achieved": flops / (float(np.mean(t)) * 1e-3) / 1e12,
                           "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                           "frac": flops / (float(np.mean(t)) * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFS}
    t = _event_ms(evs, "row_softmax")
    if t:
        by = 8 * g.nnz + 8 * n  # logits read + values written per edge, row pointers
        ref["row_softmax_avg_ms"] = float(np.mean(t))
        ref["row_softmax_GBps"] = by / (float(np.mean(t)) * 1e-3) / 1e9
    out["refresh"] = ref
    n_cf, n_kg = n_interactions // 256 + 1, E // 512 + 1
    lz = out["captured"]
    # a row's pending zero-gradient steps at the phase's end: ~ the steps since the batch last drew it
    # (n / 1,536 rows per step on average, at most the phase): the end-of-phase flush scales from the
    # measured one by that over its pending steps
    pend_epoch = min(n_kg, n / (3 * B))
    lz["epoch_flush_ms_estimate"] = lz["flush_ms"] * pend_epoch / lz["flush_steps_pending"]
    kg_lazy_s = n_kg * lz["ms_per_step"] + lz["epoch_flush_ms_estimate"]
    ep_fused = n_cf * cf_ms + n_kg * out["fused"]["ms_per_step"] + rms
    out["epoch_estimate"] = {
        "cf_steps": n_cf, "kg_steps": n_kg, "cf_ms_per_step": cf_ms, "kg_ms_per_step": lz["ms_per_step"],
        "kg_flush_ms": lz["epoch_flush_ms_estimate"], "refresh_ms": rms,
        "seconds": (n_cf * cf_ms + kg_lazy_s + rms) / 1e3, "seconds_fused_kg_dense_adam": ep_fused / 1e3,
        "what": "one reference epoch (main.py:290-361: CF phase, KG phase, attention refresh; no evaluation) at the "
                "measured per-step times, as driver.py trains: frontier-forward CF steps, KG steps with "
                "KGAT.lazy_kg_adam and KGAT.capture_kg_step (the step replayed as HIP graphs; its end-of-phase flush "
                "included); seconds_eager_lazy_kg: the same KG steps launched eagerly; seconds_fused_kg_dense_adam: "
                "the KG steps with the whole-table Adam every step"}
    out["epoch_estimate"]["seconds_eager_lazy_kg"] = (n_cf * cf_ms + n_kg * out["lazy"]["ms_per_step"]
                                                       + lz["epoch_flush_ms_estimate"] + rms) / 1e3
    return out


def nfm_legs(ds, cfg, args, dev) -> dict:
    """C3's NFM head (src/model/NFM/main.py:281-301, model.py:73-129) on the same Codeforces-shaped data:
    the train step (B pairs: positive and negative feature batches, loss, backward, Adam) and PREDICT on
    the users x all items grid of NFM/preprocess.py:309-334, batches built on the device (NFMBatcher)
    before timing.  Parity: loss, every gradient and a grid's scores vs oracle/kgat_cpu.py on the same
    weights and rows.  Rooflines: the PREDICT kernel (nfm_fwd: feature pooling + MLP + heads) against the
    fp32 MFMA peak (2 sum d_l d_(l+1) flop per row) and against HBM (k (4d + 8) + 4d bytes per
    row at k gathered features).  CPU baseline: the oracle's train step and PREDICT."""
    pkg = importlib.import_module(PKG)
    from oracle import kgat_cpu as K

    nc = cfg["nfm"]
    B, d, hidden = nc["batch"], nc["embedding_dim"], nc["hidden_dim"]
    U, I, E = ds.user_num, ds.item_num, ds.entity_num
    trip = ds.triplets
    fh, ft = trip[trip[:, 0] < I, 0], trip[trip[:, 0] < I, 2]  # problem-headed triplets (NFM/preprocess.py:166)
    batcher = pkg.NFMBatcher(U, I, E, fh, ft, ds.interaction_dict("train"), dev, train_batch_size=B, seed=2024)
    torch.manual_seed(2024)
    model = pkg.NFM(pkg.NFMArgs(user_num=U, item_num=I, entity_num=E, embedding_dim=d, hidden_dim=hidden,
                                message_dropout=[0.1] * len(hidden))).to(dev)
    model.build_optimizer(lr=1e-4)  # NFM/main.py:33-38
    model.train()
    train = [batcher.generate_train_batch() for _ in range(args.warmup + args.steps)]
    users = list(range(nc["predict_users"]))
    grid = batcher.generate_test_batch(users)
    rows = grid.shape[0]
    nnz_grid = int(grid.rowptr[-1].item())

    def step(b):
        loss = model(b[0], b[1], mode=pkg.NFMMode.TRAIN)
        loss.backward()
        model.update_weights()
        return loss

    for b in train[:args.warmup]:
        step(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in train[args.warmup:]:
        loss = step(b)
    torch.cuda.synchronize()
    tr_ms = (time.perf_counter() - t0) / args.steps * 1e3
    model.eval()
    with torch.no_grad():
        model(grid, mode=pkg.NFMMode.PREDICT)  # warm-up
        torch.cuda.synchronize()
        reps = 10
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            model(grid, mode=pkg.NFMMode.PREDICT)
        e1.record()
        torch.cuda.synchronize()
    pr_ms = e0.elapsed_time(e1) / reps
    dims = [d, *hidden]
    flops_row = 2 * sum(a * b for a, b in zip(dims[:-1], dims[1:])) + 2 * dims[-1]
    k_row = nnz_grid / rows
    bytes_row = k_row * (4 * d + 8) + 4 * d
    out = {"config": {"embedding_dim": d, "hidden_dim": hidden, "train_batch": B, "users": U, "items": I,
                      "features": U + E, "predict_rows": rows, "predict_users": len(users),
                      "features_per_row": k_row},
           "train": {"ms_per_step": tr_ms, "pairs_per_s": B / (tr_ms * 1e-3), "final_loss": float(loss.item()),
                     "what": "NFM TRAIN step (pos + neg batches of B rows, loss, backward, Adam; dropout 0.1), "
                             "batches pre-built on the device"},
           "predict": {"ms_per_call": pr_ms, "rows_per_s": rows / (pr_ms * 1e-3),
                       "roofline": {"kernel": "nfm_fwd_kernel (pooling + MLP + heads)", "bound": "mfma",
                                    "flops_per_row": flops_row, "achieved": flops_row * rows / (pr_ms * 1e-3) / 1e12,
                                    "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                                    "frac": flops_row * rows / (pr_ms * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFS,
                                    "hbm_bytes_per_row": bytes_row,
                                    "hbm_frac": bytes_row * rows / (pr_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                    "note": "the call's HIP-event time (one kernel launch + its output allocation); "
                                            "the feature table (%.0f MB) is L2 / Infinity-Cache resident, so the gather "
                                            "bytes are an upper bound on HBM traffic" % ((U + E) * d * 4 / 1e6)}}}
    # parity: the timed model's weights, one train batch (eval mode: dropout off) and 4 users' grid rows
    params = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in model.named_parameters()}
    xp, xn = (x.to_sparse_coo().cpu() for x in train[0])
    ref = K.nfm_loss(params, xp, xn, lam=1e-5)
    ref.backward()
    model.zero_grad(set_to_none=True)
    got = model(train[0][0], train[0][1], mode=pkg.NFMMode.TRAIN)
    got.backward()
    gerr = max(float((p.grad.cpu() - params[k].grad).abs().max()) for k, p in model.named_parameters())
    gscale = max(float(params[k].grad.abs().max()) for k in params)
    small = batcher.generate_test_batch(users[:4])
    with torch.no_grad():
        sc = model(small, mode=pkg.NFMMode.PREDICT).cpu()
        want = K.nfm_score({k: v.detach() for k, v in params.items()}, small.to_sparse_coo().cpu())
    serr = float((sc - want).abs().max())
    lrel = abs(float(got) - float(ref)) / max(abs(float(ref)), 1e-30)
    model.zero_grad(set_to_none=True)
    out["parity"] = {"loss_rel": lrel, "max_abs_grad": gerr, "max_abs_grad_ref": gscale, "max_abs_score": serr,
                     "tolerance": {"loss_rel": 1e-4, "grad_rel_to_max": 1e-4, "score": 1e-4},
                     "pass": bool(lrel <= 1e-4 and gerr <= 1e-4 * max(gscale, 1e-30) + 1e-7 and serr <= 1e-4),
                     "what": "eval-mode NFM loss + every gradient on one B-pair train batch and PREDICT scores of 4 "
                             "users x all items vs oracle/kgat_cpu.py (nfm_loss / nfm_score) on the timed weights"}
    if not args.no_cpu_baseline:
        torch.set_num_threads(min(64, os.cpu_count() or 1))
        ts = []
        for b in train[:3]:
            xp, xn = (x.to_sparse_coo().cpu() for x in b)
            pc = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
            t1 = time.perf_counter()
            K.nfm_loss(pc, xp, xn).backward()
            ts.append(time.perf_counter() - t1)
        gx = grid.to_sparse_coo().cpu()
        t1 = time.perf_counter()
        with torch.no_grad():
            K.nfm_score({k: v.detach() for k, v in params.items()}, gx)
        pcpu = time.perf_counter() - t1
        out["cpu_baseline"] = {"train_ms_per_step": float(np.median(ts)) * 1e3, "predict_ms_per_call": pcpu * 1e3,
                               "cores": torch.get_num_threads(), "kind": "port",
                               "sample": "oracle/kgat_cpu.py nfm_loss + backward on 3 of the timed train batches "
                                         "(median; no optimiser step) and nfm_score on the timed PREDICT grid"}
    model.train()
    return out


def frontier_matches_full(model, pkg, batch) -> dict:
    """One train-mode CF loss + backward of the timed model on the full graph, with and without
    KGAT.frontier_forward (same dropout seeds, no optimizer step): loss, table gradient and every
    aggregator weight gradient compared bit for bit."""
    fused = model.fuse_table_update
    model.fuse_table_update = False
    outs = []
    for frontier in (False, True):
        model.zero_grad(set_to_none=True)
        model.frontier_forward = frontier
        torch.manual_seed(11)
        loss = model(*batch, mode=pkg.KGATMode.TRAIN_CF)
        loss.backward()
        outs.append([loss.detach().clone()] + [p.grad.detach().clone() for p in model.parameters()
                                               if not p.is_sparse and p.grad is not None])
    model.frontier_forward = False
    model.zero_grad(set_to_none=True)
    model.fuse_table_update = fused
    a, b = outs
    return {"pass": len(a) == len(b) and all(torch.equal(x, y) for x, y in zip(a, b)), "tensors": len(a),
            "what": "loss + table and aggregator gradients of one train-mode CF step on the full graph"}


def gpu_parity_inputs(model, pkg, batch):
    """The timed model's weights, one eval-mode CF loss + table gradient and its propagated tables."""
    model.eval()
    state = {k: v.detach().clone() for k, v in model.state_dict().items() if not v.is_sparse}
    state = {k: v for k, v in state.items() if k == "_user_entity_embedding.weight" or k.startswith("_aggregator")}
    tables = [t.cpu() for t in model.propagate()]
    loss = model(*batch, mode=pkg.KGATMode.TRAIN_CF)
    loss.backward()
    model.materialize_table_grad()  # fuse_table_update leaves it to update_cf_weights otherwise
    grad = model._user_entity_embedding.weight.grad.detach().cpu()
    for p in model.parameters():
        p.grad = None
    torch.cuda.synchronize()
    model.train()
    return state, [t.cpu() for t in batch], {"tables": tables, "table_grad": grad, "loss": float(loss)}


class ShareComm:
    """--rank-share K [--share-rank r]: rank r of a K-rank row-sharded run, alone on its GPU.  Every collective
    keeps only this rank's part: a gathered layer buffer holds this rank's rows (the other ranks' rows are
    whatever the buffer held), all-reduces are the identity, all-gathers hand back this rank's tensor for every
    rank -- except the global batch ids, for which the bench supplies the other K - 1 ranks' batches
    (``peer_ids``).  The step then runs rank r's whole compute on the full-size shapes (its rows of A and A^T,
    the [N, d] gathered inputs, the global batch's frontier) with no data moving: the per-rank compute of
    DESIGN §6.2's budget, not the wire (whose bytes comm.WireLog counts as the K-rank run would send them).
    A timing harness only (sharded.Comm's interface)."""

    host = False
    force = False
    active = True

    def __init__(self, world: int, bounds, rank: int = 0):
        self.rank, self.world = int(rank), int(world)
        self.bounds = [int(x) for x in bounds]
        self.peer_ids = None

    def gather_at(self, send, out, starts, sizes):
        sh = importlib.import_module(PKG + ".sharded")
        r = self.rank
        lo, n_own = int(starts[r]), int(sizes[r])
        _comm_mod().count_gather(self, out, n_own)  # what this rank would send to its share's K - 1 peers
        own = out[lo:lo + n_own]
        if n_own and send.data_ptr() != own.data_ptr():
            own.copy_(send)
        if out.dtype == torch.int32 and out.dim() == 1:
            # a gathered id list (the hop layer's global hop rows): the peers' blocks must be ids their rows
            # hold -- evenly spaced distinct rows of each peer's range (ascending, as the real gather's)
            for k in (k for k in range(self.world) if k != r):
                s0, n = int(starts[k]), int(sizes[k])
                if n:
                    b0, b1 = self.bounds[k], self.bounds[k + 1]
                    stride = max(1, (b1 - b0) // n)
                    ids = torch.arange(n, dtype=torch.int64, device=out.device) * stride + b0
                    out[s0:s0 + n].copy_(ids.clamp_(max=b1 - 1))
        return sh._Pending([])

    def gather_v(self, send, out, bounds):
        b = [int(x) for x in bounds]
        return self.gather_at(send, out, b[:-1], [hi - lo for lo, hi in zip(b[:-1], b[1:])])

    def exchange(self, send, recv):
        _comm_mod().wire(self).add(send.numel() * send.element_size())
        return importlib.import_module(PKG + ".sharded")._Pending([])

    def all_to_all_v(self, send, send_off, recv, recv_off):
        r = self.rank
        mine = int(send_off[r + 1]) - int(send_off[r])
        _comm_mod().wire(self).add(send.element_size() * (int(send_off[-1]) - int(send_off[0]) - mine))
        recv[int(recv_off[r]):int(recv_off[r + 1])].copy_(send[int(send_off[r]):int(send_off[r + 1])])

    def all_reduce_(self, t):
        _comm_mod().count_all_reduce(self, t)
        return t

    def all_gather(self, t):
        _comm_mod().count_all_gather(self, t)
        peers = self.peer_ids
        if peers is not None and t.dtype == torch.int64 and tuple(t.shape) == tuple(peers[0].shape):
            self.peer_ids = None
            ps = [p.to(t.device) for p in peers]  # the other ranks' batches, rank order without this one
            return torch.stack(ps[:self.rank] + [t] + ps[self.rank:])
        return t.unsqueeze(0).expand(self.world, *t.shape).contiguous()


def _comm_mod():
    return importlib.import_module(PKG + ".comm")


_CKG_CACHE: dict = {}


def wire_per_step(counts: dict | None, steps: int, world: int, dev) -> dict | None:
    """comm.WireLog counts over the timed steps -> bytes per step and rank by phase ("forward", "backward",
    "other"); at world > 1 every rank's totals and the max over ranks (the wire-bound rank)."""
    if counts is None:
        return None
    out = {k: v / steps for k, v in sorted(counts.items())}
    total = sum(out.values())
    out["total"] = total
    if world > 1:
        t = torch.tensor([float(out.get("forward", 0.0)), float(out.get("backward", 0.0)), total], device=dev)
        allr = [torch.empty_like(t) for _ in range(world)]
        torch.distributed.all_gather(allr, t)
        per = torch.stack(allr).cpu().numpy()
        out["per_rank_total"] = [float(x) for x in per[:, 2]]
        out["max_rank_forward"] = float(per[:, 0].max())
        out["max_rank_total"] = float(per[:, 2].max())
    out["what"] = ("bytes this rank sends per CF step (comm.WireLog: a row gather = its rows x (G-1) peers, "
                   "a ring all-reduce 2(G-1)/G of the buffer, an all-gather (G-1) x its part)")
    return out


def run_sharded(args, cfg, world: int, rank: int, dev) -> dict:
    """c5: the table row-sharded over the ranks; each rank builds only its own rows of the graph.
    ``--rank-share K`` (one process): rank 0 of K alone (ShareComm), the per-rank compute at full size."""
    pkg = importlib.import_module(PKG)
    graph_mod = importlib.import_module(PKG + ".graph")
    sh = importlib.import_module(PKG + ".sharded")
    share = int(getattr(args, "rank_share", 0) or 0)
    if share and world != 1:
        raise RuntimeError("--rank-share runs one process (rank 0 of K alone)")
    parts = share or world
    t0 = time.perf_counter()
    threads = max(1, min(16, (os.cpu_count() or 1) // max(world, 1)))
    key = (cfg["nodes"], cfg["triples"])
    ckg = _CKG_CACHE.get(key)
    if ckg is None:  # (several --share-rank shares of one graph: drawn once per process)
        log(f"generating the synthetic CKG ({cfg['workload']}) row-sharded over {parts} ranks, {threads} threads "
            f"each ...")
        ckg = _CKG_CACHE[key] = graph_mod.HashedCKG(cfg["nodes"], cfg["triples"], seed=2024, threads=threads)
        log(f"  distinct triples drawn ({time.perf_counter() - t0:.1f}s)")
    rw = getattr(args, "row_weight", None)
    # the cost model's item-row factor (sharded.HUB_EDGE_SCALE; --hub-edge-scale 1 = edges and rows only)
    hub = sh.HUB_EDGE_SCALE if args.hub_edge_scale is None else args.hub_edge_scale
    bounds = sh.shard_bounds(ckg.row_offsets(), parts, **({} if rw is None else {"row_weight": rw}),
                             edge_scale=[(ckg.user_num, ckg.user_num + ckg.item_num, hub)])
    if share:
        # the share's rank: a number, or the rank with the most rows / the most entries of A
        sr = str(getattr(args, "share_rank_current", 0))
        rows_per, nnz_per = np.diff(bounds), np.diff(ckg.row_offsets()[bounds])
        rank = int(np.argmax(rows_per) if sr == "maxrows" else np.argmax(nnz_per) if sr == "maxedges" else int(sr))
        if not 0 <= rank < share:
            raise ValueError(f"--share-rank {sr}: not a rank of {share}")
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    rowptr, col, val = ckg.shard(lo, hi)
    log(f"  rank {rank} rows [{lo}, {hi}): {col.size:,} entries ({time.perf_counter() - t0:.1f}s)")
    shard = sh.RowShard(rowptr, col, val, bounds, rank, dev, local=True, transpose=ckg.shard(lo, hi, transpose=True))
    whole = (rowptr, col, val) if parts == 1 and not args.no_parity else None  # the oracle's graph (parity leg)
    del rowptr, col, val
    comm = ShareComm(share, bounds, rank) if share else sh.Comm()
    nnz_t = torch.tensor([shard.nnz], dtype=torch.int64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(nnz_t)
    nnz = int(nnz_t.item()) if not share else 2 * ckg.n_triples  # rank share: the whole graph's E (~2T)
    log(f"  device shards built ({time.perf_counter() - t0:.1f}s); total nnz {nnz:,}")
    log(f"graph: N={ckg.n_nodes} interactions={ckg.n_interactions} kg={ckg.n_kg} nnz={nnz}")
    if share:  # the key tools/pmc_parse.py files a rank share's counters under
        log(f"share graph: N={shard.n} nnz={shard.nnz} (rank {rank} of {share})")
    L = len(cfg["layers"])
    torch.manual_seed(2024)
    model = sh.RowShardedKGAT(pkg.KGATArgs(user_num=ckg.user_num, entity_num=ckg.entity_num, relation_num=10,
                                           cf_embedding_dim=cfg["dim"], kg_embedding_dim=cfg["dim"],
                                           layer_size=cfg["layers"], message_dropout=[0.1] * L),
                              None, comm, dev, shard=shard)
    model.train()
    model.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    model.fuse_table_update = not args.no_fused_update  # layer 0's table product fused with the shard's Adam
    B = cfg["batch"]
    rng = np.random.default_rng(7 + rank)
    batches, peer_batches = [], []
    for _ in range(args.warmup + args.steps):
        u, it = ckg.sample_interactions(rng, B)  # positives: drawn interactions (raw item ids, main.py:89)
        batches.append([torch.from_numpy(x.astype(np.int64)).to(dev)
                        for x in (u, it, rng.integers(0, ckg.item_num, B))])
        if share:  # the other ranks' batches of the same step (their own rng streams, as their processes)
            peers = []
            for k in (k for k in range(share) if k != rank):
                pr = np.random.default_rng(10_000 * (len(batches)) + 7 + k)
                pu, pit = ckg.sample_interactions(pr, B)
                peers.append(torch.from_numpy(np.stack([pu, pit, pr.integers(0, ckg.item_num, B)]).astype(np.int64)))
            peer_batches.append(peers)

    def step(b):
        if share:
            comm.peer_ids = peer_batches[next(i for i, x in enumerate(batches) if x is b)]
        loss = model(*b, mode=pkg.KGATMode.TRAIN_CF)
        loss.backward()
        model.update_cf_weights()
        return loss

    wlog = _comm_mod().wire(comm)
    elapsed, events, final_loss = timed(step, batches, args.warmup, args.steps, world, dev, wire_log=wlog)
    wire_full = wire_per_step(timed.wire_bytes, args.steps, world, dev)
    ms = elapsed / args.steps * 1e3
    if args.timeline:
        # one more step with the pipelined forward's block marks (sharded.TIMELINE): per rank, GPU time of
        # each block's compute, host time of its post and of each post's landing, relative to the first mark
        sh.TIMELINE = []
        step(batches[0])
        torch.cuda.synchronize()
        marks, sh.TIMELINE = sh.TIMELINE, None
        if marks:
            e0, h0 = marks[0][1], marks[0][2]
            lines = [f"# rank {rank} of {world}: gpu ms (event) | host ms | mark -- one CF step, pipelined forward "
                     f"({getattr(model, 'pipeline_blocks', '?')} row blocks per layer)"]
            lines += [f"{e0.elapsed_time(e):9.3f} {1e3 * (h - h0):9.3f}  {what}" for what, e, h in marks]
            out = ROOT / "gpurun_out"
            out.mkdir(exist_ok=True)
            (out / f"c5_timeline_rank{rank}.txt").write_text("\n".join(lines) + "\n")
    d0 = cfg["dim"]
    chunked = comm.active and d0 > sh.GATHER_CHUNK > 0
    # a rank share's counters are its own (profiles/pmc_c5_share.json, keyed by the share's rows / entries of A)
    roof, spmm = roofline(events, "c5_share" if share else args.config, ckg.n_nodes if parts == 1 else shard.n,
                          nnz if parts == 1 else (shard.nnz if share else 0), d0, timed.instrumented,
                          f"spmm_main_kernel<{sh.GATHER_CHUNK if chunked else d0}, 0> on the local rows of A "
                          f"(all-peer gathered layer input{', column chunks' if chunked else ''})")
    spmm["fwd_spmm_layer_edges_per_s_rank0"] = shard.nnz * L / (spmm["fwd_spmm_ms_per_step"] * 1e-3)
    if share:
        torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated(dev)
    res = {
        "value": nnz * L / (ms * 1e-3), "n_gpus": world, "ms_per_step": ms, "scaling": "strong",
        "config": {"workload": cfg["workload"], "nodes": ckg.n_nodes, "nnz": nnz, "interactions": ckg.n_interactions,
                   "kg_triples": ckg.n_kg, "embed_dim": d0, "layer_size": cfg["layers"], "global_batch": B * world,
                   "parallelism": f"row-sharded x{world}", "shard_rows": [int(x) for x in np.diff(bounds)],
                   "mode": "train (dropout 0.1)",
                   "graph": f"graph.HashedCKG (per-rank rows; {ckg.n_triples:,} distinct triples, repeats redrawn: "
                            f"E = {nnz:,} = {nnz / max(2 * ckg.n_triples, 1):.4f} x 2T)"},
        "bpr_pairs_per_s": B * world / (ms * 1e-3), "final_loss": final_loss, "spmm": spmm, "roofline": roof,
        "wire_bytes_per_step": wire_full,
        "cpu_baseline": None,
        "cpu_baseline_note": "not run: the row-sharded config never runs at N = 1 and its CPU step "
                             "(50M x 704 fp32 tables + autograd state) exceeds host RAM",
    }
    if not args.no_frontier_leg:
        # the same step with RowShardedKGAT.frontier_forward: the last layer on the batch rows F, layer L-2
        # on the first hop F + N(F) (this rank's part, marked from its A^T rows), the lower layers whole --
        # the rows the loss reads, with the whole-shard forward's bits (checked below); not in `value`
        model.frontier_forward = True
        sh.ROW_SET_STATS.clear()
        fel, fev, _ = timed(step, batches, args.warmup, args.steps, world, dev, wire_log=wlog)
        model.frontier_forward = False
        fms = fel / args.steps * 1e3
        res["frontier_forward"] = {
            "ms_per_step": fms, "bpr_pairs_per_s": B * world / (fms * 1e-3), "speedup_vs_full": ms / fms,
            "wire_bytes_per_step": wire_per_step(timed.wire_bytes, args.steps, world, dev),
            "row_sets": dict(sh.ROW_SET_STATS),
            "bit_identical_to_full": sharded_frontier_matches_full(model, pkg, batches[0]) if not share else {
                "pass": None, "what": "not checked in a rank share: the peers' rows of every gathered buffer are "
                                      "never computed, so the two forwards read different (uninitialised) rows"},
            "note": "TRAIN_CF forward restricted to the rows the BPR loss reaches (layer L-1 on the batch rows, "
                    "layer L-2 on F + N(F)); not counted in value (it does not visit every edge)"}
    if whole is not None and rank == 0:
        log("bench-scale parity: eval-mode propagation / CF loss / table gradient vs the oracle on the CPU ...")
        res["parity"] = sharded_parity(model, pkg, batches[0], whole, ckg.n_nodes, cfg)
    if share:
        res["rank_share"] = {
            "ranks": share, "rank": rank, "shard_rows": int(shard.n), "shard_nnz_A": int(shard.nnz),
            "shard_nnz_AT": int(shard.AT.col.numel()), "step_ms": ms,
            "frontier_step_ms": res.get("frontier_forward", {}).get("ms_per_step"),
            "hbm_peak_bytes": int(peak), "hbm_planned_bytes": float(sharded_bytes_per_gpu(cfg, share)),
            "design_budget_ms": 220.0,
            "note": f"rank {rank} of {share} alone on one GPU (ShareComm): its rows of A / A^T, the full [N, d] gathered "
                    f"layer buffers and the global batch, every collective local -- the per-rank compute of one "
                    f"row-sharded step at full size, no wire; `value` = the whole graph's layer-edges over this "
                    f"rank's step (the wire-hidden bound), not a measurement of {share} GPUs"}
        res["rehearsal"] = res["rank_share"]["note"]
        res["n_gpus"] = 1
    return res


def sharded_frontier_matches_full(model, pkg, batch) -> dict:
    """One train-mode CF loss + backward of the row-sharded model with and without frontier_forward (the
    same step counter, so the same dropout seeds; no optimizer step): the loss, this rank's table
    gradient rows and every aggregator weight gradient compared bit for bit."""
    outs, step0 = [], model._step
    for frontier in (False, True):
        model.zero_grad(set_to_none=True)
        model.frontier_forward = frontier
        model._step = step0
        loss = model(*batch, mode=pkg.KGATMode.TRAIN_CF)
        loss.backward()
        model.materialize_table_grad()  # fuse_table_update leaves it to update_cf_weights otherwise
        outs.append([loss.detach().clone()] + [p.grad.detach().clone() for p in model.parameters()
                                               if not p.is_sparse and p.grad is not None])
    model.frontier_forward = False
    model.zero_grad(set_to_none=True)
    a, b = outs
    return {"pass": len(a) == len(b) and all(torch.equal(x, y) for x, y in zip(a, b)), "tensors": len(a),
            "what": "loss + table-shard and aggregator gradients of one train-mode CF step"}


def sharded_parity(model, pkg, batch, whole, n: int, cfg: dict) -> dict:
    """The timed row-sharded model (world 1: its shard is the whole graph) after the timed steps vs
    oracle/kgat_cpu.py on the same graph and weights: eval-mode propagation of every layer, one CF loss
    and its table gradient (the C5 shape, d = 256, layers [256, 128, 64], at the rehearsal's scale)."""
    from oracle import kgat_cpu as K

    model.eval()
    tables = [t.cpu() for t in model.propagate()]
    loss = model(*batch, mode=pkg.KGATMode.TRAIN_CF)
    loss.backward()
    model.materialize_table_grad()
    grad = model._user_entity_embedding_shard.grad.detach().cpu()
    state = {k: v.detach().float().cpu().clone() for k, v in model.state_dict().items()
             if k.startswith("_aggregator")}
    state["_user_entity_embedding.weight"] = model._user_entity_embedding_shard.detach().cpu().clone()
    for p in model.parameters():
        p.grad = None
    model.train()
    rowptr, col, val = whole
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rowptr))
    A = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, col.astype(np.int64)])), torch.from_numpy(val),
                                (n, n)).coalesce()
    del rows
    torch.set_num_threads(min(64, os.cpu_count() or 1))
    leaves = {k: v.requires_grad_(True) for k, v in state.items()}
    outs = K.propagate(leaves, A)
    u, p, q = (t.cpu() for t in batch)
    ref = K.cf_loss(torch.cat(outs, 1), u, p, q)
    ref.backward()
    emb = max(float((o.detach() - g).abs().max()) for o, g in zip(outs, tables))
    gref = leaves["_user_entity_embedding.weight"].grad
    gerr = float((gref - grad).abs().max())
    lrel = abs(float(ref) - float(loss)) / max(abs(float(ref)), 1e-30)
    return {"max_abs_emb": emb, "max_abs_grad": gerr, "max_abs_grad_ref": float(gref.abs().max()), "loss_rel": lrel,
            "loss": float(loss), "loss_oracle": float(ref), "tolerance": PARITY_TOL,
            "pass": bool(emb <= PARITY_TOL["emb"] and gerr <= PARITY_TOL["grad"] and lrel <= PARITY_TOL["loss_rel"]),
            "what": f"eval-mode propagation of every layer, CF loss and table gradient of the timed row-sharded "
                    f"model (after the timed steps) vs oracle/kgat_cpu.py on the whole {n:,}-node graph, d = "
                    f"{cfg['dim']}, layers {cfg['layers']}, one {batch[0].numel()}-pair batch"}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--scale", type=float, default=1.0, help="shrink nodes and triples (rehearsals)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--event-every", type=int, default=10,
                    help="HIP events (the roofline's live kernel times) around the SpMMs of every k-th timed step "
                         "(each record costs the stream ~5 us between two kernels: tools/event_gap_probe.py)")
    ap.add_argument("--exchange-at-1", action="store_true",
                    help="c2/c4 at N=1: run the N-rank table exchange anyway (RCCL world 1) to time its overhead")
    ap.add_argument("--no-frontier-leg", action="store_true",
                    help="skip the second timed run with KGAT.frontier_forward (training-step speed)")
    ap.add_argument("--timeline", action="store_true",
                    help="row-sharded configs: record one step's pipelined-forward block marks per rank "
                         "(gpurun_out/c5_timeline_rank*.txt)")
    ap.add_argument("--no-kg-leg", action="store_true",
                    help="skip the KG-step / attention-refresh legs and the epoch estimate (c2/c4, N = 1)")
    ap.add_argument("--no-fused-update", action="store_true",
                    help="c2/c4: materialise the table gradient and run Adam as its own pass")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch the ranks and join the process group (gloo, no GPU), report, exit")
    ap.add_argument("--rank-share", type=int, default=0,
                    help="c5, one process: time rank r of K row-sharded ranks alone (per-rank compute, no wire)")
    ap.add_argument("--share-rank", default="0",
                    help="--rank-share's rank(s): comma-separated numbers, 'maxrows' or 'maxedges'; several run "
                         "one after another on one drawn graph, the line reports the slowest (max over ranks)")
    ap.add_argument("--row-weight", type=float, default=None,
                    help="c5: shard_bounds' per-row weight in edges (default: sharded.SHARD_ROW_WEIGHT)")
    ap.add_argument("--hub-edge-scale", type=float, default=None,
                    help="c5: shard_bounds' weight of an item row's entry (default: sharded.HUB_EDGE_SCALE)")
    ap.add_argument("--dp", choices=("auto", "replicated", "sharded"), default="auto",
                    help="N>1 table-gradient exchange (c2/c4): replicated = all-gather of the compact layer-0 "
                         "hop-set terms, every rank computes the mean gradient and full Adam; sharded = row-block "
                         "reduce-scatter, owned-row Adam, all-gather; auto = replicated for 2-layer configs")
    args = ap.parse_args()
    global EVENT_EVERY
    EVENT_EVERY = max(1, args.event_every)
    cfg = dict(CONFIGS[args.config])
    if args.scale != 1.0 and cfg.get("codeforces"):
        cfg["users"] = max(100, int(cfg["users"] * args.scale))
        cfg["workload"] += f" scaled x{args.scale:g} ({cfg['users']:,} users)"
    elif args.scale != 1.0:
        cfg["nodes"] = max(1000, int(cfg["nodes"] * args.scale))
        cfg["triples"] = max(5000, int(cfg["triples"] * args.scale))
        cfg["workload"] += f" scaled x{args.scale:g} ({cfg['nodes']:,} nodes / {cfg['triples']:,} triples)"

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    if cfg["mode"] == "sharded" and world < min_gpus(cfg) and args.rank_share < min_gpus(cfg):
        need = min_gpus(cfg)
        print(f"bench.py: config {args.config} needs >= {need} GPUs (row-sharded: planned "
              f"{sharded_bytes_per_gpu(cfg, world) / 1e9:.0f} GB per GPU at N={world}, budget "
              f"{GPU_BUDGET / 1e9:.0f} GB); run it as --gpus {need} or more", file=sys.stderr)
        return 2

    if args.dry_run:
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            joined = int(t.item())
        else:
            joined = 1
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_joined": joined, "config": args.config,
                              "mode": cfg["mode"], "min_gpus": min_gpus(cfg) if cfg["mode"] == "sharded" else 1}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0

    import torch.distributed as dist
    # KGAT_BENCH_BACKEND=gloo: rehearse the N-rank path with every rank on the GPUs there are (ranks
    # share a device round-robin; host-staged collectives) -- tests only, never a measurement
    backend = os.environ.get("KGAT_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        print(f"bench.py: KGAT_BENCH_BACKEND={backend} (nccl or gloo)", file=sys.stderr)
        return 2
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    if world > 1 or cfg["mode"] == "sharded" or args.exchange_at_1:  # (row-sharded: always a process group)
        torch.cuda.set_device(local)
        kw = {} if "MASTER_ADDR" in os.environ else dict(init_method=f"tcp://127.0.0.1:{free_port()}", rank=0,
                                                           world_size=1)
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
        if dist.get_world_size() != args.gpus:
            raise RuntimeError(f"{dist.get_world_size()} ranks joined, --gpus {args.gpus}")
    dev = torch.device("cuda", local)
    run = run_sharded if cfg["mode"] == "sharded" else run_dp
    if cfg["mode"] == "sharded" and args.rank_share and "," in args.share_rank:
        shares = []
        for sr in args.share_rank.split(","):
            args.share_rank_current = sr.strip()
            shares.append(run(args, cfg, world, rank, dev))
            gc.collect()
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(dev)
        res = max(shares, key=lambda x: x["ms_per_step"])  # the per-rank compute bound: the slowest rank
        res["rank_share_all"] = [dict(x["rank_share"], wire_bytes_per_step=x.get("wire_bytes_per_step"),
                                      frontier_wire_bytes_per_step=x.get("frontier_forward", {}).get(
                                          "wire_bytes_per_step"),
                                      row_sets=x.get("frontier_forward", {}).get("row_sets"),
                                      roofline_frac=x["roofline"]["frac"],
                                      fwd_spmm_ms_per_step=x["spmm"]["fwd_spmm_ms_per_step"]) for x in shares]
    else:
        args.share_rank_current = args.share_rank
        res = run(args, cfg, world, rank, dev)
    result = {
        "metric": "CKG edges/sec (KGAT propagation step) + BPR pairs/sec at 1/2/4/8 MI355X",
        "value": res.pop("value"), "unit": "layer-edges/s", "n_gpus": res.pop("n_gpus"), "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": res.pop("ms_per_step"), "higher_is_better": True,
        "scaling": res.pop("scaling"), "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded CKG per SURVEY §8d; random-init weights; no dataset download)",
    }
    result.update(res)
    if backend != "nccl":
        result["rehearsal"] = f"{backend} backend, ranks sharing {torch.cuda.device_count()} GPU(s): not a measurement"
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
