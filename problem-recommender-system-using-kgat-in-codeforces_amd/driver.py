"""The reference's ``make train`` / ``make predict`` / ``make recommend`` entry points on the HIP path.

Mirrors src/model/KGAT/main.py (train 234-489, predict 491-538, recommend 541-636,
early_stopping 173-195, save_model / load_model 197-231) and its Makefile targets
(train-sm, train, predict-sm, predict, recommend-sm): the same epoch structure
(all CF batches, all KG batches, UPDATE_ATTENTION, evaluation on the training
and validation splits, early stopping on validation recall@20 after 10 epochs
without improvement), the same constants and the same checkpoint file
(``result/model/kgat.pth`` = ``{"model_state_dict": state_dict}``).

Data: the reference reads Codeforces JSON dumps through its DataLoader /
Preprocess (absent here, .MISSING_LARGE_BLOBS).  ``--dataset FILE.npz`` takes the
preprocessed arrays (user_num, entity_num, item_num, train / validation / test
(user, problem) pairs, KG triplets (head, relation, tail) in entity ids);
without it a seeded Codeforces-shaped synthetic dataset is generated
(``synthetic_codeforces``: ``--sm`` = 500 users as users-sm.json, 9.5k problems,
1,913 contests, 37 tags, 28 ratings; otherwise 10x the users).  The per-user
80/20 then 90/10 train/test/validation split follows preprocess.py:55-111.
Plots and visualisers are not rebuilt (outside the hot path).
"""
from __future__ import annotations

import argparse
import json
import logging
import math
import time
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

from . import evaluation
from .graph import build_layout
from .model import KGAT, KGATArgs, KGATMode
from .sampler import BatchSampler

logger = logging.getLogger("kgat_amd")

SEED = 2024  # src/constants.py:4
EPOCH_NUM = 500  # main.py:44-54
STOP_STEPS = 10
TRAIN_CF_BATCH_SIZE = 256
TRAIN_KG_BATCH_SIZE = 512
TEST_BATCH_SIZE = 256
CF_LEARNING_RATE = 0.001
KG_LEARNING_RATE = 0.0001
METRICS_K_LIST = [20, 40, 60, 80, 100]
# src/type.py:90-94
TAGGED, HAS_DIFFICULTY, IN_CONTEST, HAS_CONTEST_DIVISION = 0, 1, 2, 3


@dataclass
class Dataset:
    user_num: int
    entity_num: int
    item_num: int
    train: np.ndarray       # int64 [M, 2] (user, problem)
    validation: np.ndarray
    test: np.ndarray
    triplets: np.ndarray    # int64 [T, 3] (head, relation, tail), entity ids

    def interaction_dict(self, split: str) -> dict[int, list[int]]:
        """user -> problems of a split, every user present (preprocess.py:_get_interaction_matrix)."""
        pairs = getattr(self, split)
        out: dict[int, list[int]] = {u: [] for u in range(self.user_num)}
        for u, i in pairs:
            out[int(u)].append(int(i))
        return out

    def save(self, path: str | Path) -> None:
        np.savez(path, user_num=self.user_num, entity_num=self.entity_num, item_num=self.item_num, train=self.train,
                 validation=self.validation, test=self.test, triplets=self.triplets)

    @classmethod
    def load(cls, path: str | Path) -> "Dataset":
        z = np.load(path)  # allow_pickle=False: plain arrays only
        return cls(int(z["user_num"]), int(z["entity_num"]), int(z["item_num"]),
                   *(np.asarray(z[k], np.int64) for k in ("train", "validation", "test", "triplets")))


def synthetic_codeforces(users: int = 500, problems: int = 9500, contests: int = 1913, tags: int = 37,
                         ratings: int = 28, divisions: int = 6, per_user=(10, 2000), seed: int = SEED):
    """(interactions [M, 2], triplets [T, 3], entity_num): the reference's KG layout
    (kg_triplets_generator.py:136-197) -- entity ids = problems first (= problem ids), then contests,
    divisions, tags, ratings; problem -> contest / 0-3 tags / rating (80 %), contest -> division
    (75 %) -- and per-user distinct solved problems with Zipf(0.8) popularity."""
    rng = np.random.default_rng(seed)
    c0 = problems
    d0, t0 = c0 + contests, c0 + contests + divisions
    r0 = t0 + tags
    entity_num = r0 + ratings
    p = np.arange(problems, dtype=np.int64)
    parts = [np.stack([p, np.full(problems, IN_CONTEST), c0 + rng.integers(0, contests, problems)], 1)]
    ntag = rng.integers(0, 4, problems)
    for j in range(3):
        sel = ntag > j
        parts.append(np.stack([p[sel], np.full(sel.sum(), TAGGED), t0 + rng.integers(0, tags, sel.sum())], 1))
    sel = rng.random(problems) < 0.8
    parts.append(np.stack([p[sel], np.full(sel.sum(), HAS_DIFFICULTY), r0 + rng.integers(0, ratings, sel.sum())], 1))
    c = np.arange(contests, dtype=np.int64)
    sel = rng.random(contests) < 0.75
    parts.append(np.stack([c0 + c[sel], np.full(sel.sum(), HAS_CONTEST_DIVISION),
                           d0 + rng.integers(0, divisions, sel.sum())], 1))
    trip = np.unique(np.concatenate(parts).astype(np.int64), axis=0)  # duplicate tags dropped
    pop = 1.0 / np.arange(1, problems + 1) ** 0.8
    pop = pop[rng.permutation(problems)]
    pop /= pop.sum()
    inter = []
    for u in range(users):
        k = int(min(problems, rng.integers(per_user[0], per_user[1] + 1)))
        it = np.sort(rng.choice(problems, size=k, replace=False, p=pop))
        inter.append(np.stack([np.full(k, u, np.int64), it], 1))
    return np.concatenate(inter), trip, entity_num


def split_interactions(inter: np.ndarray, user_num: int, seed: int = SEED):
    """Per user: shuffle, test = ceil(20 %), then validation = ceil(10 %) of the rest
    (preprocess.py:55-111, sklearn train_test_split sizes)."""
    rng = np.random.default_rng(seed)
    order = np.argsort(inter[:, 0], kind="stable")
    inter = inter[order]
    starts = np.searchsorted(inter[:, 0], np.arange(user_num + 1))
    tr, va, te = [], [], []
    for u in range(user_num):
        rows = inter[starts[u]:starts[u + 1]]
        rows = rows[rng.permutation(len(rows))]
        n_test = math.ceil(0.2 * len(rows))
        rest, test = rows[:len(rows) - n_test], rows[len(rows) - n_test:]
        n_val = math.ceil(0.1 * len(rest))
        tr.append(rest[:len(rest) - n_val])
        va.append(rest[len(rest) - n_val:])
        te.append(test)
    return tuple(np.concatenate(x) if x else np.zeros((0, 2), np.int64) for x in (tr, va, te))


def load_dataset(args) -> Dataset:
    if getattr(args, "dataset", None):
        return Dataset.load(args.dataset)
    users = 500 if args.sm else 5000
    inter, trip, entity_num = synthetic_codeforces(users=users, seed=SEED)
    tr, va, te = split_interactions(inter, users)
    return Dataset(users, entity_num, 9500, tr, va, te, trip)


def early_stopping(recalls: list[float]) -> tuple[float, bool]:
    """main.py:173-195."""
    best = max(recalls)
    return best, len(recalls) - recalls.index(best) - 1 >= STOP_STEPS


def save_model(model: KGAT, save_dir: str | Path) -> None:
    Path(save_dir).mkdir(parents=True, exist_ok=True)
    torch.save({"model_state_dict": model.state_dict()}, Path(save_dir) / "kgat.pth")


def load_model(model: KGAT, load_dir: str | Path) -> KGAT:
    ck = torch.load(Path(load_dir) / "kgat.pth", map_location="cpu", weights_only=True)
    model.load_state_dict(ck["model_state_dict"])
    model.eval()
    return model


def _model_args(ds: Dataset, layout_rel_num: int, args) -> KGATArgs:
    dim = int(getattr(args, "dim", 64))
    layers = list(getattr(args, "layers", None) or [dim, dim // 2, dim // 4])
    return KGATArgs(user_num=ds.user_num, entity_num=ds.entity_num, relation_num=layout_rel_num,
                    cf_embedding_dim=dim, kg_embedding_dim=dim, layer_size=layers,
                    message_dropout=[0.1] * len(layers))


def train(args) -> dict:
    """main.py:234-489 on the HIP path; returns the per-epoch history."""
    dev = torch.device("cuda")
    torch.manual_seed(SEED)
    ds = load_dataset(args)
    t0 = time.perf_counter()
    layout = build_layout(ds.user_num, ds.entity_num, ds.train, ds.triplets)
    logger.info("graph: %d nodes, %d nonzeros (%.1f s)", layout.n_nodes, layout.nnz, time.perf_counter() - t0)
    sampler = BatchSampler.from_arrays(ds.train, ds.item_num, layout, cf_batch_size=TRAIN_CF_BATCH_SIZE,
                                       kg_batch_size=TRAIN_KG_BATCH_SIZE, seed=SEED)
    model = KGAT(_model_args(ds, len(layout.rel_order), args))
    model.attach_graph(layout, dev)
    model.build_optimizer(cf_lr=CF_LEARNING_RATE, kg_lr=KG_LEARNING_RATE)
    model.fuse_table_update = True  # the loop below only ever steps right after backward (main.py:312-313)
    model.frontier_forward = True  # TRAIN_CF's forward on the rows its loss reaches (same bits)
    model.fuse_kg_table_update = True  # the KG step's table Adam from TransR's compact rows (same bits)
    # ... on the batch rows only, the skipped zero-gradient steps replayed when a row is next read (same bits;
    # every whole-table reader -- the CF phase, evaluation, state_dict -- flushes first)
    model.lazy_kg_adam = True
    model.capture_kg_step = True  # each KG step's forward / backward / update replays a captured HIP graph (same bits)
    model.direct_backward = True  # this loop's plain loss.backward() without the autograd engine (no DDP hooks here)
    refresh = [torch.from_numpy(np.asarray(x, np.int64)).to(dev)
               for x in (layout.heads, layout.rels, layout.tails, layout.rel_order)]
    train_dict, val_dict = ds.interaction_dict("train"), ds.interaction_dict("validation")
    test_dict = ds.interaction_dict("test")
    cf_batches = len(ds.train) // TRAIN_CF_BATCH_SIZE + 1
    kg_batches = len(layout.heads) // TRAIN_KG_BATCH_SIZE + 1
    if getattr(args, "max_batches", None):
        cf_batches, kg_batches = min(cf_batches, args.max_batches), min(kg_batches, args.max_batches)
    k_min = min(METRICS_K_LIST)
    hist: dict = {"cf_loss": [], "kg_loss": [], "training": [], "validation": [], "epoch_s": []}
    for epoch in range(1, int(getattr(args, "epochs", EPOCH_NUM)) + 1):
        model.train()
        te = time.perf_counter()
        cf_sum = torch.zeros((), device=dev)  # summed on the device: one host read per epoch
        for _ in range(cf_batches):
            u, p, n = (x.to(dev, non_blocking=True) for x in sampler.generate_cf_batch())
            loss = model(u, p, n, mode=KGATMode.TRAIN_CF)
            loss.backward()
            model.update_cf_weights()
            cf_sum += loss.detach()
        kg_sum = torch.zeros((), device=dev)
        for _ in range(kg_batches):
            h, r, pt, nt = (x.to(dev, non_blocking=True) for x in sampler.generate_kg_batch())
            loss = model(h, r, pt, nt, mode=KGATMode.TRAIN_KG)
            loss.backward()
            model.update_kg_weights()
            kg_sum += loss.detach()
        model(*refresh, mode=KGATMode.UPDATE_ATTENTION)
        torch.cuda.synchronize()
        hist["epoch_s"].append(time.perf_counter() - te)
        hist["cf_loss"].append(float(cf_sum) / cf_batches)
        hist["kg_loss"].append(float(kg_sum) / kg_batches)
        _, m_tr = evaluation.evaluate(model, train_dict, test_dict, ds.item_num, METRICS_K_LIST, TEST_BATCH_SIZE,
                                      return_scores=False)
        _, m_va = evaluation.evaluate(model, train_dict, val_dict, ds.item_num, METRICS_K_LIST, TEST_BATCH_SIZE,
                                      return_scores=False)
        hist["training"].append(m_tr)
        hist["validation"].append(m_va)
        logger.info("epoch %d: CF loss %.4f, KG loss %.4f, recall@20 train %.4f / validation %.4f (%.2f s train)",
                    epoch, hist["cf_loss"][-1], hist["kg_loss"][-1], m_tr[k_min]["recall"], m_va[k_min]["recall"],
                    hist["epoch_s"][-1])
        _, stop = early_stopping([m[k_min]["recall"] for m in hist["validation"]])
        if stop:
            logger.info("Early stopping!")
            break
    out = Path(getattr(args, "result_dir", "result"))
    save_model(model, out / "model")
    (out / "metrics").mkdir(parents=True, exist_ok=True)
    for name in ("training", "validation"):
        best = {k: {m: max(e[k][m] for e in hist[name]) for m in evaluation.METRICS} for k in METRICS_K_LIST}
        (out / "metrics" / f"{name}-metrics.json").write_text(json.dumps({"per_epoch": hist[name], "best": best},
                                                                         default=float))
    return hist


def _loaded_model(args):
    ds = load_dataset(args)
    layout = build_layout(ds.user_num, ds.entity_num, ds.train, ds.triplets)
    model = load_model(KGAT(_model_args(ds, len(layout.rel_order), args)),
                       Path(getattr(args, "result_dir", "result")) / "model")
    model.to(torch.device("cuda"))  # the checkpoint's attentive matrix becomes the device graph
    return ds, model


def predict(args) -> dict:
    """main.py:491-538: test-split metrics of the saved model."""
    ds, model = _loaded_model(args)
    _, res = evaluation.evaluate(model, ds.interaction_dict("train"), ds.interaction_dict("test"), ds.item_num,
                                 METRICS_K_LIST, TEST_BATCH_SIZE, return_scores=False)
    for k in METRICS_K_LIST:
        logger.info("@%d precision %.4f recall %.4f nDCG %.4f", k, res[k]["precision"], res[k]["recall"],
                    res[k]["ndcg"])
    return res


def recommend(args, k: int = 20) -> torch.Tensor:
    """main.py:541-636: top-20 problems per user, solved (test split) and train problems masked."""
    ds, model = _loaded_model(args)
    tr, te = ds.interaction_dict("train"), ds.interaction_dict("test")
    exclude = {u: set(tr[u]) | set(te[u]) for u in range(ds.user_num)}
    top = evaluation.recommend_topk(model, list(range(ds.user_num)), ds.item_num, exclude, k=k,
                                    batch_size=TEST_BATCH_SIZE)
    out = Path(getattr(args, "result_dir", "result"))
    out.mkdir(parents=True, exist_ok=True)
    np.savetxt(out / "recommendations.txt", top.numpy(), fmt="%d")
    counts = np.bincount(top.numpy().ravel(), minlength=ds.item_num)
    logger.info("recommended %d users; %d distinct problems", ds.user_num, int((counts > 0).sum()))
    return top


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--sm", action="store_true", help="small dataset shape (users-sm.json)")
    ap.add_argument("--predict", action="store_true")
    ap.add_argument("--recommend", action="store_true")
    ap.add_argument("--dataset", help="preprocessed dataset .npz (Dataset.save); default: synthetic")
    ap.add_argument("--epochs", type=int, default=EPOCH_NUM)
    ap.add_argument("--max-batches", type=int, default=None, help="cap CF/KG batches per epoch (smoke runs)")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--layers", type=int, nargs="*", default=None)
    ap.add_argument("--result-dir", default="result")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(message)s")
    if args.predict:
        predict(args)
    elif args.recommend:
        recommend(args)
    else:
        train(args)
