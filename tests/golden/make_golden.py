"""Generate the golden parity fixtures by running the REFERENCE classes.

Run in the build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own model/preprocess/metrics modules from
/root/reference (read-only) and records inputs + outputs as small .npz files.
Nothing of the reference's source is copied: only numbers are stored.

The reference needs two 3.11-only stdlib names on this 3.10 interpreter
(``enum.StrEnum`` for src/utils/metrics_calculator.py:1, ``datetime.UTC`` for
src/utils/json_writer.py:6); the shim below provides them.  The real
Codeforces ``--sm`` data is absent (.MISSING_LARGE_BLOBS:1-2), so the inputs
are seeded synthetic CKGs with the reference's entity / relation layout.
"""
from __future__ import annotations

import datetime
import enum
import os
import sys
from pathlib import Path

import numpy as np
import torch

REF = Path(os.environ.get("KGAT_REFERENCE", "/root/reference"))
OUT = Path(__file__).resolve().parent

# ---- stdlib shim for the 3.11 names the reference imports -----------------
if not hasattr(enum, "StrEnum"):
    class StrEnum(str, enum.Enum):  # noqa: D101
        def __str__(self) -> str:
            return str(self.value)
    enum.StrEnum = StrEnum
if not hasattr(datetime, "UTC"):
    datetime.UTC = datetime.timezone.utc
sys.path.insert(0, str(REF))

from src.model.KGAT.model import KGAT, KGATArgs, KGATMode  # noqa: E402
from src.model.KGAT.preprocess import Preprocess as KGATPreprocess  # noqa: E402
from src.model.NFM.model import NFM, NFMArgs, NFMMode  # noqa: E402
from src.model.NFM.preprocess import Preprocess as NFMPreprocess  # noqa: E402
from src.type import Entity, Relation, RelationType, Triplet  # noqa: E402
from src.utils.metrics_calculator import metrics_at_k  # noqa: E402

SEED = 2024  # src/constants.py:4


def synthetic_codeforces(rng: np.random.Generator, users: int, problems: int, contests: int,
                         tags: int, ratings: int):
    """A small CKG with the reference's layout (kg_triplets_generator.py:136-197).

    Entity ids: problems first (= problem ids), then contests, divisions, tags,
    ratings.  Returns (interactions [M,2] user,problem), triplets [T,3]
    (head, relation, tail), entity target types, entity_num.
    """
    divisions = 5
    c0 = problems
    d0 = c0 + contests
    t0 = d0 + divisions
    r0 = t0 + tags
    entity_num = r0 + ratings
    types = (["problem"] * problems + ["contest"] * contests + ["contest_division"] * divisions
             + ["tag"] * tags + ["rating"] * ratings)
    trip = set()
    for p in range(problems):
        trip.add((p, RelationType.IN_CONTEST.value, c0 + int(rng.integers(contests))))
        for tg in rng.choice(tags, size=int(rng.integers(0, 4)), replace=False):
            trip.add((p, RelationType.TAGGED.value, t0 + int(tg)))
        if rng.random() < 0.8:
            trip.add((p, RelationType.HAS_DIFFICULTY.value, r0 + int(rng.integers(ratings))))
    for c in range(contests):
        if rng.random() < 0.75:
            trip.add((c0 + c, RelationType.HAS_CONTEST_DIVISION.value, d0 + int(rng.integers(divisions))))
    # Zipf-ish problem popularity, each user 6..24 distinct problems
    pop = 1.0 / np.arange(1, problems + 1) ** 0.8
    pop = pop[rng.permutation(problems)]
    pop /= pop.sum()
    inter = []
    for u in range(users):
        k = int(rng.integers(6, 25))
        for p in rng.choice(problems, size=k, replace=False, p=pop):
            inter.append((u, int(p)))
    return np.array(inter, np.int64), np.array(sorted(trip), np.int64), types, entity_num


def reference_graph(user_num, entity_num, interactions, triplets):
    """Drive the reference Preprocess graph methods on injected state."""
    pp = KGATPreprocess.__new__(KGATPreprocess)
    pp.user_num = user_num
    pp.entity_num = entity_num
    pp.interaction_matrix = interactions
    pp._relations = [Relation(id=r.value, name=r.name) for r in RelationType]
    pp.relation_num = len(pp._relations)
    pp.triplets = [Triplet(head=int(h), relation=int(r), tail=int(t)) for h, r, t in triplets]
    pp._adjacency_matrices, pp.adjacency_relations = pp._get_adjacency_matrices()
    pp.laplacian_matrices = pp._get_bi_norm_laplacian_matrices()
    heads, rels, tails, vals = pp._get_kg_data()
    total = sum(pp.laplacian_matrices).tocoo()
    A = torch.sparse_coo_tensor(torch.LongTensor(np.vstack((total.row, total.col))),
                                torch.FloatTensor(total.data), torch.Size(total.shape))
    return pp, A, (np.array(heads), np.array(rels), np.array(tails), np.array(vals, np.float32))


def split(rng, interactions, users):
    """Per-user 80/20 train/test split of the interaction list (host-side stand-in)."""
    train, test = {}, {}
    for u in range(users):
        items = interactions[interactions[:, 0] == u, 1]
        items = items[rng.permutation(len(items))]
        k = max(1, int(round(0.8 * len(items))))
        train[u], test[u] = sorted(items[:k].tolist()), sorted(items[k:].tolist())
    return train, test


def dense_state(model) -> dict[str, np.ndarray]:
    return {k: v.detach().numpy().copy() for k, v in model.state_dict().items() if not v.is_sparse}


CHECKPOINTS_ONLY = "--checkpoints" in sys.argv  # write only the *_ckpt.pth fixtures


def make_kgat_case(name: str, users: int, problems: int, contests: int, tags: int, ratings: int,
                   dim: int, layers: list[int], cf_steps: int = 3, kg_steps: int = 2) -> None:
    rng = np.random.default_rng(SEED + len(name))
    inter, trip, _types, entity_num = synthetic_codeforces(rng, users, problems, contests, tags, ratings)
    pp, A, (heads, rels, tails, vals) = reference_graph(users, entity_num, inter, trip)
    n = users + entity_num
    rec: dict[str, np.ndarray] = {
        "user_num": np.array(users), "item_num": np.array(problems), "entity_num": np.array(entity_num),
        "dim": np.array(dim), "layers": np.array(layers), "interactions": inter, "triplets": trip,
        "adjacency_relations": np.array(pp.adjacency_relations), "kg_heads": heads, "kg_rels": rels,
        "kg_tails": tails, "kg_vals": vals,
    }
    Ac = A.coalesce()
    rec["A_idx"], rec["A_val"] = Ac.indices().numpy(), Ac.values().numpy()

    torch.manual_seed(SEED)
    model = KGAT(KGATArgs(user_num=users, entity_num=entity_num, relation_num=len(pp.adjacency_relations),
                          cf_embedding_dim=dim, kg_embedding_dim=dim, attentive_matrix=A,
                          layer_size=layers, message_dropout=[0.1] * len(layers)))
    model.eval()  # dropout off: the parity mode (SURVEY §8 trap 4)
    for k, v in dense_state(model).items():
        rec["init/" + k] = v
    with torch.no_grad():
        rec["all_emb"] = model._build_cf_embeddings().numpy()

    model.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    named = dict(model.named_parameters())
    for s in range(cf_steps):
        u = torch.LongTensor(rng.choice(users, size=min(64, users), replace=False))
        p = torch.LongTensor(rng.integers(0, problems, size=len(u)))
        q = torch.LongTensor(rng.integers(0, problems, size=len(u)))
        loss = model(u, p, q, mode=KGATMode.TRAIN_CF)
        loss.backward()
        rec[f"cf{s}/users"], rec[f"cf{s}/pos"], rec[f"cf{s}/neg"] = u.numpy(), p.numpy(), q.numpy()
        rec[f"cf{s}/loss"] = np.array(loss.item(), np.float32)
        for k, prm in named.items():
            if prm.grad is not None:
                rec[f"cf{s}/grad/{k}"] = prm.grad.numpy().copy()
        model.update_cf_weights()
    for k, v in dense_state(model).items():
        if not np.array_equal(v, rec.get("init/" + k)):   # only what the CF Adam moved
            rec["after_cf/" + k] = v

    E = len(heads)
    for s in range(kg_steps):
        pick = rng.integers(0, E, size=min(128, E))
        h = torch.tensor(heads[pick])
        r = torch.tensor(rels[pick])
        tp = torch.tensor(tails[pick])
        tn = torch.tensor(rng.integers(0, n, size=len(pick)))
        loss = model(h, r, tp, tn, mode=KGATMode.TRAIN_KG)
        loss.backward()
        rec[f"kg{s}/heads"], rec[f"kg{s}/rels"] = h.numpy(), r.numpy()
        rec[f"kg{s}/pos"], rec[f"kg{s}/neg"] = tp.numpy(), tn.numpy()
        rec[f"kg{s}/loss"] = np.array(loss.item(), np.float32)
        for k, prm in named.items():
            if prm.grad is not None:
                rec[f"kg{s}/grad/{k}"] = prm.grad.numpy().copy()
        model.update_kg_weights()
    for k, v in dense_state(model).items():
        prev = rec.get("after_cf/" + k, rec.get("init/" + k))
        if not np.array_equal(v, prev):                    # only what the KG Adam moved
            rec["after_kg/" + k] = v

    # attention refresh, exactly as main.py:351-361 drives it (eval => MHA dropout off)
    model(torch.tensor(heads), torch.tensor(rels), torch.tensor(tails),
          torch.tensor(pp.adjacency_relations), mode=KGATMode.UPDATE_ATTENTION)
    att = model.attentive_matrix.data.coalesce()
    rec["att_idx"], rec["att_val"] = att.indices().numpy(), att.values().numpy()

    # predict + ranking metrics (main.py:70-130, metrics_calculator.py:84-131)
    train, test = split(rng, inter, users)
    eval_users = np.array([u for u in range(users) if test[u]], np.int64)
    items = torch.arange(problems)
    with torch.no_grad():
        sc = model(torch.LongTensor(eval_users), items, mode=KGATMode.PREDICT)
    rec["eval_users"], rec["scores"] = eval_users, sc.numpy()
    ks = [20, 40]
    met = metrics_at_k(sc.clone(), train, test, eval_users, items.numpy(), ks)
    masked = sc.clone()
    for i, u in enumerate(eval_users):
        masked[i, train[int(u)]] = -np.inf
    rec["topk20"] = torch.topk(masked, k=20, dim=1).indices.numpy()
    for k in ks:
        for m, v in met[k].items():
            rec[f"metrics/{k}/{m.value}"] = np.asarray(v, np.float64)
    rec["train_flat"] = np.array([(u, i) for u in train for i in train[u]], np.int64)
    rec["test_flat"] = np.array([(u, i) for u in test for i in test[u]], np.int64)
    if name == "L2_d64":
        # the reference's own checkpoint format (main.py:197-210) at the state the scores above came from
        torch.save({"model_state_dict": model.state_dict()}, OUT / f"kgat_{name}_ckpt.pth")
    if CHECKPOINTS_ONLY:
        return
    np.savez_compressed(OUT / f"kgat_{name}.npz", **rec)
    print(f"kgat_{name}: N={n} E={len(heads)} nnz(A)={rec['A_val'].size} "
          f"-> {(OUT / f'kgat_{name}.npz').stat().st_size / 1e6:.2f} MB")


def make_c1_case(name: str = "C1_sm", users: int = 500, problems: int = 9500, contests: int = 1913, tags: int = 37,
                 ratings: int = 28, cf_steps: int = 2) -> None:
    """BASELINE configs[0] shape (the --sm dataset: 500 users, ~9.5k problems, 1,913 contests, 37 tags,
    28 ratings; 1 KGAT layer, d = 64), ~1M nnz: heavy users with hundreds of solved problems.
    Records only what a GPU run cannot recompute: the reference's CF losses (eval mode), its top-20
    after an attention refresh, the 21 largest masked scores per user (the near-tie rule) and its own
    precision / recall / nDCG@20 per user.  Initial weights are torch.manual_seed(2024)'s (the HIP
    module creates its parameters in the reference's order, tested)."""
    rng = np.random.default_rng(SEED + 1000)
    divisions = 5
    c0, d0 = problems, problems + contests
    t0 = d0 + divisions
    r0 = t0 + tags
    entity_num = r0 + ratings
    trip = set()
    for p in range(problems):
        trip.add((p, RelationType.IN_CONTEST.value, c0 + int(rng.integers(contests))))
        for tg in rng.choice(tags, size=int(rng.integers(0, 5)), replace=False):
            trip.add((p, RelationType.TAGGED.value, t0 + int(tg)))
        if rng.random() < 0.85:
            trip.add((p, RelationType.HAS_DIFFICULTY.value, r0 + int(rng.integers(ratings))))
    for c in range(contests):
        if rng.random() < 0.77:
            trip.add((c0 + c, RelationType.HAS_CONTEST_DIVISION.value, d0 + int(rng.integers(divisions))))
    pop = 1.0 / np.arange(1, problems + 1) ** 0.9
    pop = pop[rng.permutation(problems)]
    pop /= pop.sum()
    inter = []
    for u in range(users):
        k = int(min(problems - 1, max(10, rng.lognormal(6.8, 0.6))))  # >= 10 per user (the scraper's floor)
        inter += [(u, int(p)) for p in rng.choice(problems, size=k, replace=False, p=pop)]
    inter = np.array(inter, np.int64)
    trip = np.array(sorted(trip), np.int64)
    pp, A, (heads, rels, tails, vals) = reference_graph(users, entity_num, inter, trip)
    n = users + entity_num
    train, test = split(rng, inter, users)
    in_test = np.zeros(len(inter), bool)
    test_keys = {(u, i) for u in test for i in test[u]}
    for j, (u, i) in enumerate(inter):
        in_test[j] = (int(u), int(i)) in test_keys
    rec = {"user_num": np.array(users), "item_num": np.array(problems), "entity_num": np.array(entity_num),
           "interactions": inter.astype(np.int32), "triplets": trip.astype(np.int32),
           "test_mask": np.packbits(in_test), "nnz": np.array(A.coalesce().values().numel())}
    torch.manual_seed(SEED)
    model = KGAT(KGATArgs(user_num=users, entity_num=entity_num, relation_num=len(pp.adjacency_relations),
                          cf_embedding_dim=64, kg_embedding_dim=64, attentive_matrix=A, layer_size=[64],
                          message_dropout=[0.1]))
    model.eval()
    model.build_optimizer(cf_lr=1e-3, kg_lr=1e-4)
    for s in range(cf_steps):
        u = torch.LongTensor(rng.choice(users, size=256, replace=False))
        p = torch.LongTensor([int(rng.choice(train[int(x)])) for x in u])
        q = torch.LongTensor(rng.integers(0, problems, size=256))
        loss = model(u, p, q, mode=KGATMode.TRAIN_CF)
        loss.backward()
        model.update_cf_weights()
        rec[f"cf{s}/users"], rec[f"cf{s}/pos"], rec[f"cf{s}/neg"] = u.numpy(), p.numpy(), q.numpy()
        rec[f"cf{s}/loss"] = np.array(loss.item(), np.float32)
    model(torch.tensor(heads), torch.tensor(rels), torch.tensor(tails), torch.tensor(pp.adjacency_relations),
          mode=KGATMode.UPDATE_ATTENTION)
    eval_users = np.array([u for u in range(users) if test[u]], np.int64)
    items = torch.arange(problems)
    with torch.no_grad():
        sc = model(torch.LongTensor(eval_users), items, mode=KGATMode.PREDICT)
    met = metrics_at_k(sc.clone(), train, test, eval_users, items.numpy(), [20])
    masked = sc.clone()
    for i, u in enumerate(eval_users):
        masked[i, train[int(u)]] = -np.inf
    top = torch.topk(masked, k=21, dim=1)
    rec["eval_users"] = eval_users
    rec["topk20"] = top.indices[:, :20].numpy().astype(np.int32)
    rec["top21_scores"] = top.values.numpy()
    for m, v in met[20].items():
        rec[f"metrics/20/{m.value}"] = np.asarray(v, np.float64)
    rec["recall20_mean"] = np.array(float(np.mean(met[20][[m for m in met[20] if m.value == "recall"][0]])))
    np.savez_compressed(OUT / f"kgat_{name}.npz", **rec)
    print(f"kgat_{name}: N={n} interactions={len(inter)} E={len(heads)} nnz(A)={int(rec['nnz'])} "
          f"recall@20={float(rec['recall20_mean']):.4f} -> {(OUT / f'kgat_{name}.npz').stat().st_size / 1e6:.2f} MB")


def make_nfm_case(name: str, users: int, problems: int, contests: int, tags: int, ratings: int,
                  dim: int, hidden: list[int]) -> None:
    rng = np.random.default_rng(SEED + 100 + len(name))
    inter, trip, types, entity_num = synthetic_codeforces(rng, users, problems, contests, tags, ratings)
    pp = NFMPreprocess.__new__(NFMPreprocess)
    pp.user_num, pp.item_num, pp.entity_num = users, problems, entity_num
    pp._entities = [Entity(id=i, target_type=t, target_id=i) for i, t in enumerate(types)]
    pp._triplets = [Triplet(head=int(h), relation=int(r), tail=int(t)) for h, r, t in trip]
    user_m, feat_m = pp._get_user_and_feature_matrices()
    pp._user_matrix, pp._feature_matrix = user_m, feat_m
    fc = feat_m.tocoo()
    rec = {"user_num": np.array(users), "item_num": np.array(problems), "entity_num": np.array(entity_num),
           "dim": np.array(dim), "hidden": np.array(hidden), "triplets": trip, "interactions": inter,
           "feat_row": fc.row.astype(np.int64), "feat_col": fc.col.astype(np.int64),
           "feat_val": fc.data.astype(np.float32)}
    torch.manual_seed(SEED)
    model = NFM(NFMArgs(user_num=users, item_num=problems, entity_num=entity_num, embedding_dim=dim,
                        hidden_dim=hidden, message_dropout=[0.1] * len(hidden)))
    model.eval()
    for k, v in dense_state(model).items():
        rec["init/" + k] = v
    import scipy.sparse as sp
    model.build_optimizer(lr=1e-4)
    named = dict(model.named_parameters())
    for s in range(2):
        u = rng.choice(users, size=min(96, users), replace=False)
        p = rng.integers(0, problems, size=len(u))
        q = rng.integers(0, problems, size=len(u))
        xp = pp._convert_to_tensor(sp.hstack([user_m[u], feat_m[p]]).tocoo())
        xn = pp._convert_to_tensor(sp.hstack([user_m[u], feat_m[q]]).tocoo())
        loss = model(xp, xn, mode=NFMMode.TRAIN)
        loss.backward()
        rec[f"tr{s}/users"], rec[f"tr{s}/pos"], rec[f"tr{s}/neg"] = u, p, q
        rec[f"tr{s}/loss"] = np.array(loss.item(), np.float32)
        for k, prm in named.items():
            if prm.grad is not None:
                rec[f"tr{s}/grad/{k}"] = prm.grad.numpy().copy()
        model.update_weights()
    for k, v in dense_state(model).items():
        rec["after/" + k] = v
    test_users = torch.LongTensor(np.arange(min(4, users)))
    pp._user_matrix = user_m
    x = NFMPreprocess.generate_test_batch(pp, test_users)
    with torch.no_grad():
        sc = model(x, mode=NFMMode.PREDICT)
    rec["pred_users"], rec["pred_scores"] = test_users.numpy(), sc.numpy()
    torch.save({"model_state_dict": model.state_dict()}, OUT / f"nfm_{name}_ckpt.pth")  # NFM/main.py:186-198
    if CHECKPOINTS_ONLY:
        return
    np.savez_compressed(OUT / f"nfm_{name}.npz", **rec)
    print(f"nfm_{name}: F={users + entity_num} -> {(OUT / f'nfm_{name}.npz').stat().st_size / 1e6:.2f} MB")


if __name__ == "__main__":
    torch.set_num_threads(4)
    if "--c1" in sys.argv:  # the C1 (--sm shaped) ranking fixture only
        make_c1_case()
        sys.exit(0)
    make_kgat_case("L1_d64", users=96, problems=200, contests=40, tags=16, ratings=8, dim=64, layers=[64])
    make_kgat_case("L3_d64", users=96, problems=200, contests=40, tags=16, ratings=8, dim=64,
                   layers=[64, 32, 16])
    make_kgat_case("L2_d64", users=120, problems=260, contests=50, tags=20, ratings=10, dim=64,
                   layers=[64, 32])
    make_kgat_case("L3_d128", users=64, problems=120, contests=24, tags=12, ratings=6, dim=128,
                   layers=[128, 64, 32], cf_steps=1, kg_steps=1)
    make_nfm_case("h3_d64", users=64, problems=150, contests=30, tags=12, ratings=8, dim=64,
                  hidden=[64, 32, 16])
