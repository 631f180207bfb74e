"""CF / KG batch sampling on the host in native code.

Mirrors the reference's ``Preprocess.generate_cf_batch`` / ``generate_kg_batch``
(src/model/KGAT/preprocess.py:328-525): the same draws (users / heads without
replacement unless the batch is larger than the population, one positive per
row uniform over the row's interactions / edges, one negative by rejection),
computed by kgat_sample_cf_batch / kgat_sample_kg_batch (csrc/sampler.cpp)
instead of per-sample Python loops.  The reference's module-level ``rng`` is
unseeded; here a batch is a function of (seed, step), so runs reproduce.
"""
from __future__ import annotations

from typing import Mapping, Sequence

import numpy as np
import torch

from . import _lib


class BatchSampler:
    """Samplers over a user -> items map and the CKG edge list (head, relation, tail)."""

    def __init__(self, interaction_dict: Mapping[int, Sequence[int]], item_num: int, kg_heads: np.ndarray,
                 kg_rels: np.ndarray, kg_tails: np.ndarray, n_nodes: int, cf_batch_size: int = 256,
                 kg_batch_size: int = 512, seed: int = 2024, pin_memory: bool = True):
        self.item_num, self.n_nodes = int(item_num), int(n_nodes)
        self._cf_batch_size, self._kg_batch_size = int(cf_batch_size), int(kg_batch_size)
        self.seed = int(seed)
        # batches land in pinned host memory so the caller's .to(device, non_blocking=True) is a true
        # async copy (a pageable source makes the copy wait for the device queue to drain)
        self.pin_memory = bool(pin_memory) and torch.cuda.is_available()
        self._cf_step = self._kg_step = 0
        users = np.array(sorted(u for u, v in interaction_dict.items() if len(v)), np.int64)
        rows = [np.unique(np.asarray(interaction_dict[int(u)], np.int64)) for u in users]
        self._cf_users = users
        self._cf_rowptr = np.zeros(users.size + 1, np.int64)
        np.cumsum([r.size for r in rows], out=self._cf_rowptr[1:])
        self._cf_items = np.concatenate(rows) if rows else np.zeros(1, np.int64)
        h = np.asarray(kg_heads, np.int64)
        key = np.asarray(kg_rels, np.int64) * self.n_nodes + np.asarray(kg_tails, np.int64)
        order = np.lexsort((key, h))
        h, key = h[order], key[order]
        keep = np.ones(h.size, bool)
        keep[1:] = (h[1:] != h[:-1]) | (key[1:] != key[:-1])  # duplicate (h, r, t) edges
        h, key = h[keep], key[keep]
        self._kg_heads, starts = np.unique(h, return_index=True)
        self._kg_rowptr = np.append(starts, h.size).astype(np.int64)
        self._kg_rel_tail = key if key.size else np.zeros(1, np.int64)

    @classmethod
    def from_arrays(cls, interactions: np.ndarray, item_num: int, layout, **kw) -> "BatchSampler":
        """From (user, item) pairs and a graph.GraphLayout (its kg edge arrays)."""
        inter = np.asarray(interactions, np.int64)
        order = np.argsort(inter[:, 0], kind="stable")
        u, i = inter[order, 0], inter[order, 1]
        bounds = np.flatnonzero(np.diff(u)) + 1
        d = {int(uu[0]): ii for uu, ii in zip(np.split(u, bounds), np.split(i, bounds)) if uu.size}
        return cls(d, item_num, layout.heads, layout.rels, layout.tails, layout.n_nodes, **kw)

    def generate_cf_batch(self) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(user_ids, positive_problem_ids, negative_problem_ids) -- LongTensors (preprocess.py:381-409)."""
        B = self._cf_batch_size
        out = self._buffers(3, B)
        self._cf_step += 1
        _lib.call("kgat_sample_cf_batch", self._cf_users.ctypes.data, self._cf_users.size, self._cf_rowptr.ctypes.data,
                  self._cf_items.ctypes.data, self.item_num, B, self.seed, self._cf_step,
                  *[o.data_ptr() for o in out])
        return tuple(out)

    def _buffers(self, k: int, B: int) -> list[torch.Tensor]:
        # torch's pinned-memory cache keeps a block out of reuse until the copies reading it are done
        return [torch.empty(B, dtype=torch.int64, pin_memory=self.pin_memory) for _ in range(k)]

    def generate_kg_batch(self) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
        """(heads, relations, positive_tails, negative_tails) (preprocess.py:486-525; LongTensors)."""
        B = self._kg_batch_size
        out = self._buffers(4, B)
        self._kg_step += 1
        _lib.call("kgat_sample_kg_batch", self._kg_heads.ctypes.data, self._kg_heads.size, self._kg_rowptr.ctypes.data,
                  self._kg_rel_tail.ctypes.data, self.n_nodes, B, self.seed, self._kg_step,
                  *[o.data_ptr() for o in out])
        return tuple(out)
