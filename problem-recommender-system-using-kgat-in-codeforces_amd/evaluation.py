"""Evaluation and recommendation ranking on the GPU.

Mirrors the reference's ranking code path for path:
- ``metrics_at_k``: src/utils/metrics_calculator.py:84-131 (same signature and
  result layout: ``{k: {"precision" | "recall" | "ndcg": ndarray[n_users]}}``;
  the keys equal the reference's ``Metrics`` StrEnum members).  Like the
  reference it writes -inf into ``cf_scores`` at the train items (in place).
- ``evaluate``: src/model/KGAT/main.py:70-130 -- but the graph is propagated
  ONCE per evaluation (the reference re-propagates per 256-user batch; the
  scores are identical because PREDICT does not change the model).
- ``recommend_topk``: the masked ``torch.topk(k=20)`` of main.py:576-605.

Arithmetic: kgat_score_f32 (fused gather + MFMA GEMM), kgat_mask_rows_f32,
kgat_topk_f32 (radix select + bitonic sort) and kgat_rank_metrics_f32 -- all
in csrc/.  Equal scores rank by ascending item id; the reference's torch.sort
leaves their order unspecified, which can only matter for ties at the k-th rank.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Mapping, Sequence

import numpy as np
import torch

from . import _lib, kernels
from .graph import stream_ptr

METRICS = ("precision", "recall", "ndcg")
METRICS_K_LIST = [20, 40, 60, 80, 100]  # main.py:53
TEST_BATCH_SIZE = 256                   # main.py:48


def _csr(lists: Sequence[Iterable[int]], device, unique: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
    """int64 rowptr [len+1] + int32 indices of per-row id lists (sorted + unique when asked)."""
    rows = []
    for ids in lists:
        a = np.asarray(list(ids), dtype=np.int64)
        if unique:
            a = np.unique(a)
        rows.append(a)
    lens = np.array([a.size for a in rows], np.int64)
    rowptr = np.zeros(len(rows) + 1, np.int64)
    np.cumsum(lens, out=rowptr[1:])
    idx = np.concatenate(rows).astype(np.int32) if rows and rowptr[-1] > 0 else np.zeros(1, np.int32)
    return (torch.from_numpy(rowptr).to(device), torch.from_numpy(idx).to(device))


def mask_rows(scores: torch.Tensor, rowptr: torch.Tensor, idx: torch.Tensor, value: float = float("-inf")) -> None:
    kernels._req(scores, "scores", dim=2)
    if scores.stride(1) != 1:
        raise ValueError("scores must be row-contiguous")
    rows, cols = scores.shape
    _lib.call("kgat_mask_rows_f32", scores.data_ptr(), scores.stride(0), rows, cols, rowptr.data_ptr(),
              idx.data_ptr(), ctypes.c_float(value), stream_ptr(scores.device))


def topk(scores: torch.Tensor, k: int, values: bool = False):
    """Top-k columns per row, descending (ties: ascending column). int64 [rows, k] (+ values)."""
    kernels._req(scores, "scores", dim=2)
    if scores.stride(1) != 1:
        raise ValueError("scores must be row-contiguous")
    rows, cols = scores.shape
    if not 1 <= k <= min(cols, 1024):
        raise ValueError(f"k must be in [1, min(cols, 1024)], got {k}")
    idx = torch.empty(rows, k, dtype=torch.int32, device=scores.device)
    val = torch.empty(rows, k, dtype=torch.float32, device=scores.device) if values else None
    _lib.call("kgat_topk_f32", scores.data_ptr(), scores.stride(0), rows, cols, k, idx.data_ptr(),
              val.data_ptr() if val is not None else None, stream_ptr(scores.device))
    return (idx.long(), val) if values else idx.long()


def rank_metrics(top: torch.Tensor, test_rowptr: torch.Tensor, test_idx: torch.Tensor,
                 k_list: Sequence[int]) -> torch.Tensor:
    """float32 [len(k_list), 3, rows]: precision / recall / ndcg @k (metrics_calculator.py:17-81)."""
    top32 = top.to(torch.int32).contiguous()
    rows, kmax = top32.shape
    ks = (ctypes.c_int32 * len(k_list))(*[int(k) for k in k_list])
    out = torch.empty(len(k_list), 3, rows, dtype=torch.float32, device=top.device)
    _lib.call("kgat_rank_metrics_f32", top32.data_ptr(), rows, kmax, test_rowptr.data_ptr(), test_idx.data_ptr(),
              ctypes.cast(ks, ctypes.c_void_p), len(k_list), out.data_ptr(), stream_ptr(top.device))
    return out


def metrics_at_k(cf_scores: torch.Tensor, train_interaction_dict: Mapping[int, Sequence[int]],
                 test_interaction_dict: Mapping[int, Sequence[int]], user_ids, item_ids,
                 k_list: Sequence[int]) -> dict[int, dict[str, np.ndarray]]:
    """metrics_calculator.py:84-131 on the GPU.  cf_scores: [len(user_ids), len(item_ids)] on the
    GPU, columns = item ids 0..I-1 (as the reference builds them)."""
    user_ids = np.asarray(user_ids).reshape(-1)
    n_items = len(item_ids)
    if cf_scores.shape != (user_ids.size, n_items):
        raise ValueError("cf_scores must be [len(user_ids), len(item_ids)]")
    dev = cf_scores.device
    tr_ptr, tr_idx = _csr([train_interaction_dict[int(u)] for u in user_ids], dev)
    te_ptr, te_idx = _csr([test_interaction_dict[int(u)] for u in user_ids], dev, unique=True)
    mask_rows(cf_scores, tr_ptr, tr_idx)
    kmax = max(k_list)
    top = topk(cf_scores, kmax)
    m = rank_metrics(top, te_ptr, te_idx, k_list).cpu().numpy()
    return {int(k): {name: m[t, j].copy() for j, name in enumerate(METRICS)} for t, k in enumerate(k_list)}


@torch.no_grad()
def evaluate(model, train_interaction_dict: Mapping[int, Sequence[int]],
             eval_interaction_dict: Mapping[int, Sequence[int]], item_num: int,
             k_list: Sequence[int] = METRICS_K_LIST, batch_size: int = TEST_BATCH_SIZE,
             return_scores: bool = True, return_per_user: bool = False):
    """main.py:70-130: returns (scores [n_eval_users, item_num] on the host or None,
    {k: {metric: mean over users}}) -- plus, with return_per_user, {k: {metric: ndarray[n_eval_users]}}
    in the eval dict's user order (what the reference averages, metrics_calculator.py:124-131)."""
    model.eval()
    tables = model.propagate()
    dev = tables[0].device
    test_user_ids = list(eval_interaction_dict.keys())
    items = torch.arange(item_num, dtype=torch.long, device=dev)
    per_k = {int(k): {m: [] for m in METRICS} for k in k_list}
    all_scores = []
    for i in range(0, len(test_user_ids), batch_size):
        users = np.asarray(test_user_ids[i:i + batch_size], np.int64)
        sc = kernels.scores(tables, torch.from_numpy(users).to(dev), items)
        if return_scores:
            all_scores.append(sc.cpu())  # before masking, as main.py:103-115 keeps them
        met = metrics_at_k(sc, train_interaction_dict, eval_interaction_dict, users, np.arange(item_num), k_list)
        for k in per_k:
            for m in METRICS:
                per_k[k][m].append(met[k][m])
    per_user = {k: {m: np.concatenate(per_k[k][m]) for m in METRICS} for k in per_k}
    result = {k: {m: float(per_user[k][m].mean()) for m in METRICS} for k in per_k}
    scores = torch.cat(all_scores) if return_scores else None
    return (scores, result, per_user) if return_per_user else (scores, result)


@torch.no_grad()
def recommend_topk(model, user_ids: Sequence[int], item_num: int, exclude: Mapping[int, Iterable[int]],
                   k: int = 20, batch_size: int = TEST_BATCH_SIZE) -> torch.Tensor:
    """main.py:576-605: top-k items per user with ``exclude[user]`` masked to -inf; int64 [U, k] on the host."""
    tables = model.propagate()
    dev = tables[0].device
    items = torch.arange(item_num, dtype=torch.long, device=dev)
    out = []
    for i in range(0, len(user_ids), batch_size):
        users = np.asarray(user_ids[i:i + batch_size], np.int64)
        sc = kernels.scores(tables, torch.from_numpy(users).to(dev), items)
        ptr, idx = _csr([sorted(set(exclude.get(int(u), ()))) for u in users], dev)
        mask_rows(sc, ptr, idx)
        out.append(topk(sc, k).cpu())
    return torch.cat(out)
