"""Host-side profile of the CF training step (python tools/host_profile.py [--full] [--kg [--unfused | --lazy |
--captured]]: the KG step instead): cProfile over
200 steps of a small synthetic graph (host launch cost does not depend on the graph size), printing
the functions with the most own time.  Used to find Python / ctypes overhead in the step's launches."""
import cProfile
import importlib
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
PKG = "problem-recommender-system-using-kgat-in-codeforces_amd"


def main():
    full = "--full" in sys.argv
    pkg = importlib.import_module(PKG)
    graph_mod = importlib.import_module(PKG + ".graph")
    dev = torch.device("cuda:0")
    U, E, inter, trip = graph_mod.synthetic_ckg(100_000, 1_000_000, seed=3)
    lay = graph_mod.build_layout(U, E, inter, trip)
    torch.manual_seed(0)
    m = pkg.KGAT(pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32],
                              message_dropout=[0.1, 0.1]))
    m.attach_graph(lay, dev)
    m.train()
    m.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    m.fuse_table_update = True
    m.direct_backward = True
    m.frontier_forward = not full
    rng = np.random.default_rng(1)
    batches = [[torch.from_numpy(rng.integers(0, hi, 256)).to(dev) for hi in (U, int(E * 0.1), int(E * 0.1))]
               for _ in range(16)]

    kg = "--kg" in sys.argv
    if kg:  # the KG phase's step (main.py:324-345) at the reference's B = 512, fused table update
        m.fuse_kg_table_update = "--unfused" not in sys.argv
        m.lazy_kg_adam = "--lazy" in sys.argv or "--captured" in sys.argv
        m.capture_kg_step = "--captured" in sys.argv
        n = U + E
        batches = [[torch.from_numpy(x).to(dev) for x in (lay.heads[e], lay.rels[e], lay.tails[e],
                                                          rng.integers(0, n, 512))]
                   for e in (rng.integers(0, lay.heads.size, 512) for _ in range(16))]

    def step(b):
        if kg:
            loss = m(*b, mode=pkg.KGATMode.TRAIN_KG)
            loss.backward()
            m.update_kg_weights()
            return
        loss = m(*b, mode=pkg.KGATMode.TRAIN_CF)
        loss.backward()
        m.update_cf_weights()

    for i in range(20):
        step(batches[i % 16])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(200):
        step(batches[i % 16])
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"{'kg' if kg else ('full' if full else 'frontier')}: host {host / 200 * 1e3:.3f} ms/step, wall {wall / 200 * 1e3:.3f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for i in range(200):
        step(batches[i % 16])
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
