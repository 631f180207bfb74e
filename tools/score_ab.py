"""A/B of the edge scorer's tiles-per-wave (KGAT_SCORE_P=1 vs 2 vs 4, an env switch the launcher read during the
round-6 measurement and no longer has) on the C2 graph at d = 64 and 128: bit-identity of the logits (eval and
train-mode dropout) and interleaved HIP-event timings.  Results: gpurun_out/score_ab2.log, DESIGN.md round 6 #8.
Without the switch every variant runs the built one (P = 2 from d = 64), so it now reports one timing.

    python tools/score_ab.py [--dims 64,128] [--reps 5]
"""
import argparse
import importlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
PKG = "problem-recommender-system-using-kgat-in-codeforces_amd"


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", default="64,128")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--triples", type=int, default=10_000_000)
    args = ap.parse_args()
    pkg = importlib.import_module(PKG)
    graph = importlib.import_module(PKG + ".graph")
    K = importlib.import_module(PKG + ".kernels")
    dev = torch.device("cuda", 0)
    t0 = time.time()
    U, E, inter, trip = graph.synthetic_ckg(args.nodes, args.triples, seed=2024)
    lay = graph.build_layout(U, E, inter, trip)
    print(f"graph built {time.time() - t0:.1f}s, edges {lay.heads.size}", flush=True)
    out = {}
    for d in (int(x) for x in args.dims.split(",")):
        torch.manual_seed(0)
        m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[d // 2],
                                  cf_embedding_dim=d, kg_embedding_dim=d))
        g = m.attach_graph(lay, dev)
        h, r, t = (torch.from_numpy(x).to(dev) for x in (lay.heads, lay.rels, lay.tails))
        plan = g.refresh_plan(h, r, t)
        mha = m._multi_head_attention
        w = [m._user_entity_embedding.weight.detach(), m._trans_matrix.detach(), mha._value_weight.weight.detach(),
             mha._value_weight.bias.detach(), mha._output.weight.detach(), mha._output.bias.detach(),
             mha._layer_norm.weight.detach(), mha._layer_norm.bias.detach()]
        res = {}
        PS = ("1", "2", "4") if d <= 64 else ("1", "2")
        for p_drop in (0.0, 0.1):
            outs = {}
            for P in PS:
                os.environ["KGAT_SCORE_P"] = P
                outs[P] = K.edge_logits(g, plan, *w, dropout_p=p_drop, seed=11).clone()
            res[f"bit_identical_p{p_drop}"] = all(bool(torch.equal(outs["1"], outs[P])) for P in PS)
        flop = 6.0 * d * d * lay.heads.size
        ms = {P: [] for P in PS}
        for _ in range(3):  # interleaved pairs
            for P in PS:
                os.environ["KGAT_SCORE_P"] = P
                ms[P].append(timeit(lambda: K.edge_logits(g, plan, *w), args.reps))
        for P in ms:
            best = min(ms[P])
            res[f"P{P}_ms"] = [round(x, 3) for x in ms[P]]
            res[f"P{P}_mfma_frac"] = round(flop / (best * 1e-3) / 157.3e12, 3)
        out[d] = res
        print(json.dumps({d: res}), flush=True)
        del m, g, plan, w
        torch.cuda.empty_cache()
    os.environ.pop("KGAT_SCORE_P", None)


if __name__ == "__main__":
    main()
