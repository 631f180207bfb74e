"""The frontier chain's set sizes at full C5 (graph.HashedCKG, N = 50M, 500M triples), on the host: the global
batch F of G ranks x 256 pairs (users, positives, uniform negatives, as bench.py draws them), the first hop
F + N_A(F) and the second hop -- the rows each row-set gather of the row-sharded frontier forward moves
(sharded._frontier_sets), per rank of shard_bounds(row_weight).  usage: python tools/c5_hop_fractions.py
[scale] [G] [threads] -> JSON (profiles/r06_c5_hop_fractions.json)"""
import importlib
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
PKG = "problem-recommender-system-using-kgat-in-codeforces_amd"


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    graph = importlib.import_module(PKG + ".graph")
    sh = importlib.import_module(PKG + ".sharded")
    t0 = time.perf_counter()
    ckg = graph.HashedCKG(int(50_000_000 * scale), int(500_000_000 * scale), seed=2024, threads=threads)
    N = ckg.n_nodes
    print(f"graph drawn {time.perf_counter() - t0:.0f}s", file=sys.stderr, flush=True)
    rowptr, col, _ = ckg.shard(0, N)
    print(f"CSR built {time.perf_counter() - t0:.0f}s nnz {col.size:,}", file=sys.stderr, flush=True)
    B = 256
    F = []
    for k in range(G):
        rng = np.random.default_rng(7 + k)
        u, it = ckg.sample_interactions(rng, B)
        F += [u, it, rng.integers(0, ckg.item_num, B)]
    F = np.unique(np.concatenate(F).astype(np.int64))

    def expand(rows):
        mark = np.zeros(N, bool)
        mark[rows] = True
        starts, ends = rowptr[rows], rowptr[rows + 1]
        tot = int((ends - starts).sum())
        idx = np.repeat(starts - np.concatenate([[0], np.cumsum(ends - starts)[:-1]]), ends - starts) + np.arange(tot)
        mark[col[idx]] = True
        return np.flatnonzero(mark)

    hop1 = expand(F)
    hop2 = expand(hop1)
    hop3 = expand(hop2)
    print(f"hops {hop1.size} {hop2.size} {hop3.size} ({time.perf_counter() - t0:.0f}s)", file=sys.stderr, flush=True)
    out = {"nodes": N, "nnz": int(col.size), "G": G, "batch_rows": int(F.size), "hop1": int(hop1.size),
           "hop2": int(hop2.size), "hop3": int(hop3.size), "hop1_frac": hop1.size / N, "hop2_frac": hop2.size / N,
           "hop3_frac": hop3.size / N}
    dims = [256, 256, 128]  # the inputs of layers 0, 1, 2 at C5
    hops = [hop3, hop2, hop1]  # the rows layer 0 / 1 / 2 reads its input on (sharded._frontier_sets)
    items = [(ckg.user_num, ckg.user_num + ckg.item_num, sh.HUB_EDGE_SCALE)]
    for name, kw in (("mean_degree", dict(row_weight=float(rowptr[-1] / N))), ("row_weight_48", {}),
                     ("cost_model", dict(edge_scale=items))):
        b = sh.shard_bounds(rowptr, G, **kw)
        ranks = []
        for r in range(G):
            lo, hi = int(b[r]), int(b[r + 1])
            own = [int(((h >= lo) & (h < hi)).sum()) for h in hops]
            rec = {"rows": hi - lo, "edges": int(rowptr[hi] - rowptr[lo]), "hop1": own[2], "hop2": own[1],
                   "hop3": own[0]}
            # the frontier forward's sends (G - 1 peers): each layer input on its hop's rows while the global hop
            # holds <= COMPACT_FRACTION of the nodes, else the whole shard
            fwd = 0
            for h, o, d in zip(hops, own, dims):
                fwd += (o if h.size <= sh.COMPACT_FRACTION * N else hi - lo) * 4 * d * (G - 1)
            rec["frontier_forward_wire_bytes"] = fwd
            rec["whole_forward_wire_bytes"] = (hi - lo) * 4 * sum(dims) * (G - 1)
            ranks.append(rec)
        out[f"ranks_{name}"] = ranks
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
