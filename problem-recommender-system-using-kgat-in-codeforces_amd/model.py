"""Drop-in KGAT model on the MI355X HIP path.

Mirrors the reference module API of src/model/KGAT/model.py:13-431: the same
``KGATArgs`` fields and defaults, the same ``KGATMode`` values, the same
parameter names / creation order (so ``torch.manual_seed`` gives the same
initial weights and ``state_dict`` keys -- including the sparse COO
``attentive_matrix`` -- interoperate with reference checkpoints), and the same
``forward(*args, mode=...)``, ``build_optimizer``, ``update_cf_weights``,
``update_kg_weights`` calls.  The arithmetic never runs on torch ops: every
mode calls the hand-written gfx950 kernels of libkgat_hip.so.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import IntEnum
from typing import Any

import ctypes
import math

import numpy as np
import torch
from torch import nn

from . import _lib, kernels
from .graph import DeviceGraph, GraphLayout, csr_from_coo, stream_ptr
from .optim import FusedAdam


@dataclass
class KGATArgs:
    """Same fields/defaults as the reference (model.py:13-23)."""

    user_num: int
    entity_num: int
    relation_num: int
    cf_embedding_dim: int = 64
    kg_embedding_dim: int = 64
    attentive_matrix: torch.Tensor | None = None
    message_dropout: list[float] = field(default_factory=lambda: [0.1, 0.1, 0.1])
    layer_size: list[int] = field(default_factory=lambda: [64, 32, 16])
    regularization_params: list[float] = field(default_factory=lambda: [1e-5, 1e-5])


class KGATMode(IntEnum):
    TRAIN_CF = 0
    TRAIN_KG = 1
    UPDATE_ATTENTION = 2
    PREDICT = 3


class Aggregator(nn.Module):
    """Parameter holder of one bi-interaction layer (aggregator.py:15-35).

    Same submodule names and initialisation order as the reference; the
    arithmetic is the fused HIP kernel (csrc/biinter.hip).
    """

    def __init__(self, input_dim: int, output_dim: int, dropout: float) -> None:
        super().__init__()
        self.dropout = float(dropout)
        self.linear1 = nn.Linear(input_dim, output_dim)
        self.linear2 = nn.Linear(input_dim, output_dim)
        nn.init.xavier_uniform_(self.linear1.weight)
        nn.init.xavier_uniform_(self.linear2.weight)

    def weights(self) -> list[torch.Tensor]:
        return [self.linear1.weight, self.linear1.bias, self.linear2.weight, self.linear2.bias]


class MultiHeadAttention(nn.Module):
    """Parameter holder of the knowledge-aware attention (multi_head_attention.py:5-30)."""

    def __init__(self, cf_embedding_dim: int, kg_embedding_dim: int, head_num: int = 8, dropout: float = 0.1):
        super().__init__()
        self._head_num = head_num
        self.dropout = dropout
        self._query_weight = nn.Linear(cf_embedding_dim, kg_embedding_dim)
        self._key_weight = nn.Linear(cf_embedding_dim, kg_embedding_dim)
        self._value_weight = nn.Linear(cf_embedding_dim, kg_embedding_dim)
        self._output = nn.Linear(kg_embedding_dim, kg_embedding_dim)
        self._layer_norm = nn.LayerNorm(kg_embedding_dim)
        for lin in (self._query_weight, self._key_weight, self._value_weight, self._output):
            nn.init.xavier_uniform_(lin.weight)


# The backward's hop chain runs a layer on its hop set while that set holds at most this
# fraction of the nodes (beyond it the dense kernels stream the rows faster).
HOP_DENSE_FRACTION = 0.4


def _hop_estimate(graph, l: int):
    """Layer l's hop-set size at a previous step (None before any listing was launched): read from the
    pinned mirror as it stands -- the listing kernels store it through to memory themselves, so the
    newest completed count is there without an event (an older one while the GPU runs behind)."""
    ent = getattr(graph, "_hop_est", {}).get(l)
    if ent is None:
        return None
    return int(ent[0][0])


def _hop_small(graph, l: int, n_nodes: int) -> bool:
    """Run layer l on its hop set: its size at the previous step (unknown: yes) is at most
    HOP_DENSE_FRACTION of the nodes."""
    est = _hop_estimate(graph, l)
    return est is None or est <= HOP_DENSE_FRACTION * n_nodes


def _hop_host(graph, l: int) -> torch.Tensor:
    """Layer l's pinned hop-count mirror: the kernel that lists the hop set (kgat_frontier_hop /
    kgat_hop_compact) writes the count there itself (host-mapped memory, no copy launch)."""
    est = graph.__dict__.setdefault("_hop_est", {})
    ent = est.get(l)
    if ent is None:
        ent = est[l] = (torch.zeros(1, dtype=torch.int32, pin_memory=True), torch.cuda.Event())
    return ent[0]


def _hop_record(graph, l: int, exact: bool = False) -> None:
    """Layer l's hop set was just listed.  ``exact``: this step's backward reads the count on the host (a wide
    layer sizing its compact problem) -- an event is recorded behind the listing for that read; otherwise
    none (each record costs the stream ~5 us between two kernels), the estimate reads the mirror as is."""
    if exact:
        graph._hop_est[l][1].record()
    graph.__dict__.setdefault("_hop_exact", {})[l] = exact


# A layer that went dense on its last-known hop-set size re-measures the set every this many dense steps.
HOP_REPROBE_STEPS = 8


def _hop_reprobe(graph, l: int) -> None:
    """Layer l runs densely because its hop set was large at a previous step; no hop listing refreshes the
    estimate then, so every HOP_REPROBE_STEPS-th such step lists the set anyway from the row flags the
    previous product left (kgat_hop_compact: the count lands in the pinned mirror, no host sync; the dense
    path reads none of its outputs) -- a set that shrank takes the layer back to the hop chain."""
    cnt = graph.__dict__.setdefault("_hop_dense_steps", {})
    cnt[l] = cnt.get(l, 0) + 1
    if cnt[l] % HOP_REPROBE_STEPS == 0:
        kernels.hop_compact(graph, count_host=_hop_host(graph, l))
        _hop_record(graph, l)


class _IdGuard:
    """Ids are range-checked before any kernel indexes a table with them (the reference's
    nn.Embedding gathers raise IndexError, model.py:188-191, 219-222, 389-391).

    Host ids are checked on the host, at once.  Device ids are checked on the device without
    a host synchronisation (kgat_ids_check_ex: one launch copies them, zeroes any id outside
    [0, bound) so no kernel reads out of range, and sets a flag in pinned host memory and one in
    device memory); the host flag is read after the call's event and IndexError is raised at the
    model's next call (or by ``raise_pending(block=True)``) -- the way PyTorch reports a
    device-side index error.  The device flag is the optimiser kernels' skip flag
    (``update_cf_weights`` / ``update_kg_weights`` pass it): a step whose ids were bad moves no
    parameter and no Adam moment, although the host learns of it only later; it is cleared when
    the error is raised."""

    def __init__(self):
        self._host = self._event = self._dev = None
        self._pending = None
        self._tag = 0  # the last tag a TRAIN_CF check (kgat_cf_begin_ex) was launched with
        self._tag_stream = None  # its stream, while that check is the pending one (no event behind it)

    def skip_flag(self) -> torch.Tensor | None:
        """The device int32 flag the optimiser kernels read (None before any device-id check)."""
        return self._dev

    def _ensure(self, device) -> None:
        if self._host is None:
            # pinned host words written by the check kernels themselves (host-mapped: no copy launch per
            # call): [0] the bad-id flag (every check kernel sets it; cleared here), [1] kgat_cf_begin_ex's tag
            self._host = torch.zeros(2, dtype=torch.int32, pin_memory=True)
            self._event = torch.cuda.Event()
            self._dev = torch.zeros(1, dtype=torch.int32, device=device)

    def raise_pending(self, block: bool = False) -> None:
        if self._pending is None:
            return
        if self._tag_stream is not None:
            # a TRAIN_CF check: done when its tag is in the word (stored through to memory by the kernel)
            if int(self._host[1]) != self._tag:
                if not block:
                    return
                self._tag_stream.synchronize()
        else:
            if not block and not self._event.query():
                return
            self._event.synchronize()
        what = self._pending
        self._pending = self._tag_stream = None
        if int(self._host[0]):
            # every check launched so far is complete (the pending one was the last): no kernel writes the flag
            self._host[0] = 0
            if self._dev is not None:
                kernels.fill(self._dev.view(torch.float32), 0.0)  # int32 0 == float 0.0 bits
            raise IndexError(f"{what}: id out of range (detected on the device; the call ran with it zeroed, "
                             f"and no optimiser step after it moved a parameter)")

    def check(self, what: str, ids, bound: int, device, more=(), outs=None) -> list[torch.Tensor]:
        """int64 device copies of ``ids`` (each as given, flattened), validated against [0, bound);
        ``more`` = further (ids, bound) groups of the same call, checked under the same flag so a
        call raises (for an earlier call's device ids) at most once, before it runs.  ``outs``: one
        preallocated int64 buffer per group (device ids; a captured step's static inputs)."""
        self.raise_pending()
        groups = [(list(ids), int(bound))] + [(list(i), int(b)) for i, b in more]
        flat = [torch.as_tensor(t) for g, _ in groups for t in g]
        if all(t.device.type == "cpu" for t in flat):
            for g, b in groups:
                for t in map(torch.as_tensor, g):
                    if t.numel() and (int(t.min()) < 0 or int(t.max()) >= b):
                        raise IndexError(f"{what}: id out of range [0, {b}) (min {int(t.min())}, max {int(t.max())})")
            return [t.to(device).long().reshape(-1).contiguous() for t in flat]
        self._ensure(device)
        given, outs = outs, []
        for gi, (g, b) in enumerate(groups):
            src = [torch.as_tensor(t).to(device).long().reshape(-1).contiguous() for t in g]
            sizes = [t.numel() for t in src]
            if given is not None:
                out = given[gi]
                if out.dtype != torch.int64 or not out.is_contiguous() or out.numel() < sum(sizes):
                    raise ValueError("id check: preallocated buffer too small")
            else:
                out = torch.empty(max(sum(sizes), 1), dtype=torch.int64, device=device)
            for i in range(0, len(src), _lib.KGAT_IDS_MAX):
                part = src[i:i + _lib.KGAT_IDS_MAX]
                d = _lib.Ids()
                for k, t in enumerate(part):
                    d.ptr[k], d.n[k] = t.data_ptr(), t.numel()
                d.count = len(part)
                off = sum(sizes[:i])
                _lib.call("kgat_ids_check_ex", ctypes.byref(d), b, out.data_ptr() + 8 * off, self._host.data_ptr(),
                          self._dev.data_ptr(), stream_ptr(device))
            outs += list(out[:sum(sizes)].split(sizes))
        self._event.record()
        self._pending, self._tag_stream = what, None
        return outs

    def check_cf(self, what: str, ids, bound: int, device, node_map: torch.Tensor, clear=None, mark=None):
        """TRAIN_CF's ids checked (the rules of ``check``) and numbered as the batch frontier in one launch
        (kgat_cf_begin_ex: kgat_ids_check_ex + kgat_frontier_build, a bitmap pair zeroed when ``clear`` =
        (bits0, bits1, words), and the batch's first hop marked in the pair ``mark`` = (graph, (bits0, bits1))
        -- kernels.hop_bitmaps_next).  Returns ((users, pos, neg), rows, count) or None when the ids do not
        take this path (sizes differ, 3B > 4096, an id array is empty)."""
        ts = [torch.as_tensor(t) for t in ids]
        B = ts[0].numel()
        if B == 0 or 3 * B > 4096 or any(t.numel() != B for t in ts):
            return None
        self.raise_pending()
        if all(t.device.type == "cpu" for t in ts):
            for t in ts:
                if int(t.min()) < 0 or int(t.max()) >= bound:
                    raise IndexError(f"{what}: id out of range [0, {bound}) (min {int(t.min())}, max {int(t.max())})")
        self._ensure(device)
        src = [t.to(device).long().reshape(-1).contiguous() for t in ts]
        tag = self._tag % ((1 << 29) - 1) + 1
        # the completion tag instead of an event record (~5 us of GPU time per record between two kernels)
        out, rows, count = kernels.cf_begin(*src, bound, self._host, self._dev, node_map, clear, tag=tag, mark=mark)
        self._tag = tag  # launched: the tag the host now waits for
        self._pending, self._tag_stream = what, torch.cuda.current_stream(src[0].device)
        return tuple(out.split(B)), rows, count

    def check_multi(self, what: str, ts, bounds, out: torch.Tensor, device) -> None:
        """The captured KG step's check: ``ts`` (<= KGAT_IDS_MAX int64 contiguous 1-D device tensors) checked
        against their own bounds (a ctypes int64 array) and copied, concatenated, into the preallocated ``out``
        in one launch (kgat_ids_check_multi)."""
        self.raise_pending()
        self._ensure(device)
        d = _lib.Ids()
        for k, t in enumerate(ts):
            d.ptr[k], d.n[k] = t.data_ptr(), t.numel()
        d.count = len(ts)
        _lib.call("kgat_ids_check_multi", ctypes.byref(d), bounds, out.data_ptr(), self._host.data_ptr(),
                  self._dev.data_ptr(), stream_ptr(device))
        self._event.record()
        self._pending, self._tag_stream = what, None


class _TableUpdate:
    """The CF step's table gradient left unmaterialised until ``update_cf_weights`` (opt-in:
    ``KGAT.fuse_table_update = True``).

    The reference step is ``loss.backward(); model.update_cf_weights()`` (main.py:312-313):
    backward writes the dense [N, d] table gradient, Adam reads it back (model.py:404-413).
    With the hop chain that gradient is one masked product, A^T . dS_0 + dXd_0, of compact
    hop-set terms; deferred, ``update_cf_weights`` runs it fused with the table's Adam step
    (kgat_spmm_csr_masked_adam_f32): the product's latency-bound gather and Adam's streaming
    p / m / v traffic share one pass and the 2 x 4 B/param gradient write + read disappears.
    Same bits as the unfused step.  Meanwhile ``table.grad`` stays None; anything that needs
    it (a second backward, a KG step, UPDATE_ATTENTION -- which rewrites A's values --, an
    explicit ``materialize_table_grad()``) materialises it first."""

    def __init__(self, param: torch.Tensor):
        self.param = param
        self.enabled = False
        self.pending = None

    def defer(self, graph, src_map, Xc, Yc, rank) -> bool:
        if not self.enabled or self.param.grad is not None or self.pending is not None:
            return False
        self.pending = (graph, src_map, Xc, Yc, rank)
        return True

    @torch.no_grad()
    def materialize(self) -> None:
        if self.pending is None:
            return
        graph, src_map, Xc, Yc, rank = self.pending
        self.pending = None
        g = kernels.spmm_masked(graph, src_map, Xc, Yc_init=Yc, transpose=True, src_rank=rank)
        if self.param.grad is None:
            self.param.grad = g
        else:
            kernels.add_(self.param.grad, g)

    def discard(self) -> None:
        """Drop the pending gradient (a step whose update is abandoned: update_cf_weights raised)."""
        self.pending = None

    def launch(self):
        """The fused product + Adam of the pending gradient (FusedAdam.step(fused=...))."""
        graph, src_map, Xc, Yc, rank = self.pending
        self.pending = None
        p = self.param.data

        def run(m, v, step_size, bc2s, b1, b2, eps, skip=None, extra=None):
            kernels.spmm_masked_adam(graph, src_map, Xc, Yc, rank, p, m, v, step_size, b1, b2, bc2s, eps, skip,
                                     extra=extra)
        run.takes_extra = True  # FusedAdam.step may hand it the step's other tensors (their Adam in its fix-up)
        return run


class _KGTableUpdate:
    """The KG step's table gradient kept compact until ``update_kg_weights`` (opt-in:
    ``KGAT.fuse_kg_table_update = True``).

    The reference KG step is ``loss.backward(); model.update_kg_weights()`` (main.py:334-342):
    nn.Embedding's dense backward writes a [N, d] table gradient that is zero except on the <= 3B
    rows TransR gathered (model.py:211-221), and Adam reads it back (model.py:414-419).  Here the
    TransR backward writes those rows compactly (kgat_transr_bwd_ex_f32, rows numbered by
    kgat_frontier_build's map) and ``update_kg_weights`` runs the table's Adam with row r's gradient
    looked up through the map, 0 elsewhere (kgat_adam_rows_f32): the same bits as the dense step,
    without writing, zeroing or re-reading the [N, d] gradient.  Anything that needs the gradient
    first materialises it (a second backward, the next forward, ``materialize_table_grad()``)."""

    def __init__(self, param: torch.Tensor):
        self.param = param
        self.enabled = False
        self.pending = None
        self._map = None
        self.marked = None  # the batch rows a TRAIN_KG forward numbered in the map, for its backward

    def node_map(self) -> torch.Tensor:
        """node -> compact row of the batch ids (-1 between steps), allocated once."""
        n = self.param.shape[0]
        if self._map is None or self._map.numel() != n or self._map.device != self.param.device:
            self._map = torch.full((n,), -1, dtype=torch.int32, device=self.param.device)
        return self._map

    def wants(self, batch: int) -> bool:
        # kgat_frontier_build numbers at most 4096 slots (3 per sample)
        return self.enabled and self.pending is None and self.param.grad is None and 3 * batch <= 4096

    def defer(self, rows: torch.Tensor, Gc: torch.Tensor) -> None:
        self.pending = (rows, Gc)

    def mark(self, heads, pos, neg) -> torch.Tensor:
        """Number the batch rows in the map (kgat_frontier_build) in the forward -- the lazy Adam's
        catch-up and the backward's compact gradient use the same rows; a forward whose backward never
        ran releases its marks here first."""
        self.release()
        rows, _ = kernels.frontier_build(heads, pos, neg, self.node_map())
        self.marked = rows
        return rows

    def release(self) -> None:
        if self.marked is not None:
            kernels.frontier_reset(self.marked, self._map)
            self.marked = None

    @torch.no_grad()
    def materialize(self) -> None:
        if self.pending is None:
            return
        rows, Gc = self.pending
        self.pending = None
        g = kernels.zeros(tuple(self.param.shape), self.param.device)
        kernels.scatter_rows(g, rows, Gc[:rows.numel()], accumulate=False)
        kernels.frontier_reset(rows, self._map)
        if self.param.grad is None:
            self.param.grad = g
        else:
            kernels.add_(self.param.grad, g)

    def discard(self) -> None:
        """Drop the pending rows (update_kg_weights raised); the node map is reset for the next step."""
        if self.pending is None:
            return
        rows, _ = self.pending
        self.pending = None
        kernels.frontier_reset(rows, self._map)

    def launch(self, lazy: "_LazyKGAdam | None" = None, opt=None):
        """The table's Adam step on the compact gradient (FusedAdam.step(fused=...)); with ``lazy`` on the
        batch rows only (_LazyKGAdam)."""
        rows, Gc = self.pending
        self.pending = None
        p, row_map = self.param.data, self._map
        if lazy is not None:
            return lazy.launch(opt, rows, Gc, row_map)

        def run(m, v, step_size, bc2s, b1, b2, eps, skip=None):
            kernels.adam_rows(p, m, v, row_map, Gc, step_size, b1, b2, bc2s, eps, skip)
            kernels.frontier_reset(rows, row_map)
        return run


class _LazyKGAdam:
    """The KG phase's table Adam on the batch rows only (opt-in: ``KGAT.lazy_kg_adam``; needs the fused KG
    table update's compact rows).

    The reference's KG step (main.py:334-342, model.py:414-419) runs Adam over the whole table every
    step: nn.Embedding's dense gradient is zero outside the <= 3B batch rows, yet those rows still move
    (their moments decay and p takes the step m / (sqrt(v) + eps)).  At C4 that is 24 B of HBM per
    parameter per step (5 ms) for 1,536 touched rows.  Here each row records the last KG step applied to
    it and its skipped zero-gradient steps are replayed, in order and with each step's own step size,
    bias correction and skip flag (a device history), when the row is next read or updated
    (kgat_adam_lazy_catchup_f32 / kgat_adam_lazy_rows_f32) -- the dense step's exact sequence of
    adam_elem operations per element, so the same bits.  Anything that reads the whole table (a CF,
    PREDICT or UPDATE_ATTENTION forward, the CF update, state_dict, propagate) flushes first: every row
    is brought up to the current step.  Between a KG step and a flush the table's rows outside recent
    batches and the KG optimiser's moments are behind: call ``KGAT.flush_kg_table()`` before reading
    ``_user_entity_embedding.weight`` or the KG optimiser's state directly."""

    CAP = 1 << 20  # history entries (steps); a flush is forced before any row falls this far behind

    def __init__(self, param: torch.Tensor):
        self.param = param
        self.enabled = False
        self.last = None
        self.hist = None
        self.flushed_at = 0
        self.dirty = False  # rows behind the current step (a lazy step since the last flush)

    def _t(self, opt) -> int:
        st = opt.state.get(id(self.param))
        return int(st["step"]) if st is not None else 0

    def ensure(self, opt) -> None:
        n = self.param.shape[0]
        if self.last is None or self.last.numel() != n or self.last.device != self.param.device:
            dev = self.param.device
            t = self._t(opt)
            self.last = torch.full((n,), t, dtype=torch.int32, device=dev)
            if self.hist is None or self.hist[0].device != dev:
                # entries are written by the step that owns them before any replay reads them
                self.hist = (torch.zeros(self.CAP, dtype=torch.float32, device=dev),
                             torch.zeros(self.CAP, dtype=torch.float32, device=dev),
                             torch.zeros(self.CAP, dtype=torch.int32, device=dev))
            self.flushed_at = t

    def catch_up(self, opt, rows: torch.Tensor | None = None) -> None:
        """Bring the listed rows (None: every row) up to the optimiser's current step."""
        st = opt.state.get(id(self.param))
        if self.last is None or st is None or (rows is None and not self.dirty):
            return
        t = int(st["step"])
        p = self.param.data
        n, d = p.shape
        hs, hb, hk = self.hist
        _lib.call("kgat_adam_lazy_catchup_f32", p.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                  n, d, rows.data_ptr() if rows is not None else None, rows.numel() if rows is not None else 0,
                  self.last.data_ptr(), t, hs.data_ptr(), hb.data_ptr(), hk.data_ptr(), self.CAP, opt.beta1,
                  opt.beta2, opt.eps, stream_ptr(p.device))
        if rows is None:
            self.flushed_at = t
            self.dirty = False

    def launch(self, opt, rows: torch.Tensor, Gc: torch.Tensor, row_map: torch.Tensor):
        """FusedAdam's fused launch for the table: step t on the batch rows only."""
        p = self.param.data

        def run(m, v, step_size, bc2s, b1, b2, eps, skip=None):
            t = self._t(opt)
            self.dirty = True
            hs, hb, hk = self.hist
            _lib.call("kgat_adam_lazy_rows_f32", p.data_ptr(), m.data_ptr(), v.data_ptr(), p.shape[1], rows.data_ptr(),
                      rows.numel(), Gc.data_ptr(), Gc.stride(0), self.last.data_ptr(), t, hs.data_ptr(), hb.data_ptr(),
                      hk.data_ptr(), self.CAP, step_size, b1, b2, bc2s, eps,
                      skip.data_ptr() if skip is not None else None, stream_ptr(p.device))
            kernels.frontier_reset(rows, row_map)
        return run

    def dense_step_done(self, opt) -> None:
        """A dense step t was just applied to every row (each caught up before it): every row is current at
        t, so the per-row record restarts there (the next lazy step re-creates it, ``ensure``).  Keeping the
        old record would leave every row's last[] at its pre-dense value, and after 2^20 such steps the ring
        slots a replay still needs would be overwritten."""
        self.last = None
        self.dirty = False


class _KGStepGraph:
    """The KG step captured as HIP graphs (opt-in: ``KGAT.capture_kg_step``; with the fused KG table update
    and the lazy KG Adam, as driver.py trains).

    The reference KG step is ``loss = model(h, r, t+, t-, mode=TRAIN_KG); loss.backward();
    model.update_kg_weights()`` (main.py:334-342; model.py:204-261, 414-419).  Eagerly that is ~13
    launches wrapped in ~0.2 ms of Python, ctypes and autograd work for ~0.12 ms of kernels at C2.
    Here the forward and the update each replay one graph captured once per shape:
      forward -- frontier_build (the batch rows' map), the lazy Adam catch-up of those rows, TransR
                 forward (loss + the backward's work buffer);
      update  -- TransR backward (the table gradient's compact rows, d_rel, d_trans), the lazy table Adam
                 on the batch rows (which also resets their map entries), the Adam of the relation
                 embeddings and trans matrices (the two advance the device step counter between them).
    ``loss.backward()`` only copies its upstream gradient into the graphs' input (the backward kernels
    run in the update graph, so one replay fewer); a third graph -- the TransR backward alone -- serves
    anything that needs the gradients before the update (``materialize``).  Outside the graphs: one id
    check (kgat_ids_check_multi: the caller's ids checked and copied into the static inputs) and the loss
    copy.  A graph replays its captured kernel arguments, so the step's scalars live on the device:
    t_dev (advanced by the update graph) indexes schedule tables of the step size and sqrt(1 - beta2^t)
    that the host fills with FusedAdam's own expressions -- the same floats the eager launches get -- and
    the host keeps the optimiser's step counters in step.  The three parameters' ``.grad`` stay None
    between backward and update, as with the fused table updates.  Same bits as the eager step
    (tests/test_gpu_parity.py::test_captured_kg_step_bit_identical)."""

    SCHED = 1 << 16  # initial schedule entries (steps); doubled (and the graphs recaptured) when t reaches them

    def __init__(self, model: "KGAT"):
        self.model = model
        self.enabled = False
        self.key = None
        self.g = None       # {"fwd", "bwd", "upd"} graphs
        self.buf = None     # static tensors of the captured step
        self.pending = None  # "fwd" after a forward replay, "bwd" once backward copied its gradient in
        self.t_dev_value = None  # the host's view of t_dev
        self._sched = None  # (key, sz, bc)
        self._bounds = (ctypes.c_int64 * _lib.KGAT_IDS_MAX)()
        self.replays = 0

    # ---------------------------------------------------------------- eligibility
    def _states(self, opt):
        m = self.model
        ps = (m._user_entity_embedding.weight, m._relation_embedding.weight, m._trans_matrix)
        sts = [opt.state.get(id(p)) for p in ps]
        return ps, sts

    def usable(self, ids, opt):
        """The three parameters' KG optimiser states when the captured step applies, else None."""
        m = self.model
        if not (self.enabled and m._kg_table_update.enabled and m._lazy_kg.enabled and opt is not None):
            return None
        B = ids[0].numel()
        if B == 0 or not all(torch.is_tensor(t) and t.is_cuda and t.dtype == torch.int64 and t.dim() == 1
                             and t.is_contiguous() and t.numel() == B for t in ids):
            return None
        if not m._kg_table_update.wants(B) or m._lazy_kg.last is None or m._ids.skip_flag() is None:
            return None
        ps, sts = self._states(opt)
        if any(st is None for st in sts) or len({int(st["step"]) for st in sts}) != 1:
            return None  # the first KG step (and a state restored out of step) runs eagerly
        if any(p.grad is not None for p in ps):
            return None
        return ps, sts

    # ---------------------------------------------------------------- schedule + capture
    def _schedule(self, opt, dev, need: int):
        """Device tables of step t's step size and sqrt(1 - beta2^t) for t < len >= need."""
        key = (id(opt), opt.lr, opt.beta1, opt.beta2, str(dev))
        if self._sched is None or self._sched[0] != key or self._sched[1].numel() < need:
            size = self.SCHED
            while size < need:
                size *= 2
            # FusedAdam._advance's expressions, evaluated per t in Python floats, then rounded to float32 as
            # ctypes rounds the by-value arguments
            lr, b1, b2 = opt.lr, opt.beta1, opt.beta2
            sz = np.array([0.0] + [lr / (1.0 - b1 ** t) for t in range(1, size)], dtype=np.float32)
            bc = np.array([0.0] + [math.sqrt(1.0 - b2 ** t) for t in range(1, size)], dtype=np.float32)
            self._sched = (key, torch.from_numpy(sz).to(dev), torch.from_numpy(bc).to(dev))
        return self._sched[1], self._sched[2]

    def _key(self, B, opt, ps, sts):
        """Everything the graphs captured by address: a change (another optimiser, reallocated state or
        parameters, a new lazy record) recaptures them."""
        m = self.model
        lz = m._lazy_kg
        return (B, opt.beta1, opt.beta2, opt.eps, float(m._regularization_params[1]),
                self._sched[1].data_ptr(), self._sched[2].data_ptr(),
                *(p.data_ptr() for p in ps), *(st[k].data_ptr() for st in sts for k in ("exp_avg", "exp_avg_sq")),
                lz.last.data_ptr(), *(h.data_ptr() for h in lz.hist), m._kg_table_update.node_map().data_ptr(),
                m._ids.skip_flag().data_ptr())

    def _capture(self, B, opt, ps, sts):
        m = self.model
        dev = m._user_entity_embedding.weight.device
        sz, bc = self._sched[1], self._sched[2]
        emb, rel, trans = (p.data for p in ps)
        lz = m._lazy_kg
        hs, hb, hk = lz.hist
        row_map = m._kg_table_update.node_map()
        skip = m._ids.skip_flag()
        n, d = emb.shape
        n_rel, k = rel.shape
        reg = float(m._regularization_params[1])
        b = {"ids": torch.zeros(4 * B, dtype=torch.int64, device=dev),  # heads | pos | neg | relations
             "gout": torch.ones(1, dtype=torch.float32, device=dev),
             "t": torch.zeros(1, dtype=torch.int32, device=dev),
             "t_next": torch.zeros(1, dtype=torch.int32, device=dev)}
        h, p, q, r = b["ids"].split(B)
        ev = (kernels.KERNEL_EVENTS, kernels.SPMM_EVENTS)
        kernels.KERNEL_EVENTS = kernels.SPMM_EVENTS = None  # no event records inside a capture
        pool = torch.cuda.graph_pool_handle()
        g = {key: torch.cuda.CUDAGraph() for key in ("fwd", "bwd", "upd")}

        def update_kernels(Gc, d_rel, d_trans):
            st_ = stream_ptr(dev)
            # step t + 1 applied by the lazy rows' launch, its number passed on in t_next; the relation /
            # trans Adam reads it there and writes it back to t (no separate counter launch)
            _lib.call("kgat_adam_lazy_rows_sched_f32", emb.data_ptr(), sts[0]["exp_avg"].data_ptr(),
                      sts[0]["exp_avg_sq"].data_ptr(), d, rows.data_ptr(), rows.numel(), Gc.data_ptr(),
                      Gc.stride(0), lz.last.data_ptr(), hs.data_ptr(), hb.data_ptr(), hk.data_ptr(), lz.CAP,
                      b["t"].data_ptr(), sz.data_ptr(), bc.data_ptr(), opt.beta1, opt.beta2, opt.eps,
                      skip.data_ptr(), row_map.data_ptr(), 1, b["t_next"].data_ptr(), st_)  # + the map reset
            arr = (_lib.AdamTensor * 2)()
            for a, (pp, gg, stt) in zip(arr, ((rel, d_rel, sts[1]), (trans, d_trans, sts[2]))):
                a.p, a.g, a.m, a.v = pp.data_ptr(), gg.data_ptr(), stt["exp_avg"].data_ptr(), stt["exp_avg_sq"].data_ptr()
                a.n, a.step_size, a.bc2_sqrt = pp.numel(), 0.0, 0.0
            _lib.call("kgat_adam_multi_sched_f32", arr, 2, opt.beta1, opt.beta2, opt.eps, skip.data_ptr(),
                      b["t_next"].data_ptr(), sz.data_ptr(), bc.data_ptr(), 0, b["t"].data_ptr(), st_)

        try:
            torch.cuda.synchronize(dev)
            with torch.cuda.graph(g["fwd"], pool=pool):
                rows, _ = kernels.frontier_build(h, p, q, row_map)
                _lib.call("kgat_adam_lazy_catchup_sched_f32", emb.data_ptr(), sts[0]["exp_avg"].data_ptr(),
                          sts[0]["exp_avg_sq"].data_ptr(), n, d, rows.data_ptr(), rows.numel(), lz.last.data_ptr(),
                          b["t"].data_ptr(), hs.data_ptr(), hb.data_ptr(), hk.data_ptr(), lz.CAP, opt.beta1, opt.beta2,
                          opt.eps, stream_ptr(dev))
                loss, work = kernels.transr_fwd(emb, rel, trans, h, r, p, q, reg)
            with torch.cuda.graph(g["bwd"], pool=pool):
                grads = kernels.transr_bwd_compact(emb, n_rel, k, h, r, p, q, work, b["gout"], row_map, rows.numel())
            with torch.cuda.graph(g["upd"], pool=pool):
                update_kernels(*kernels.transr_bwd_compact(emb, n_rel, k, h, r, p, q, work, b["gout"], row_map,
                                                           rows.numel()))
        finally:
            kernels.KERNEL_EVENTS, kernels.SPMM_EVENTS = ev
        b.update(rows=rows, loss=loss, work=work, Gc=grads[0], d_rel=grads[1], d_trans=grads[2])
        self.g, self.buf = g, b
        self.gout_one = True  # b["gout"] starts as ones
        self.t_dev_value = None
        self.key = self._key(B, opt, ps, sts)

    # ---------------------------------------------------------------- the three calls
    def forward(self, ids, opt, ps, sts) -> torch.Tensor:
        """Replay the forward graph on the caller's ids (heads, relations, positive, negative tails)."""
        m = self.model
        B = ids[0].numel()
        t = int(sts[0]["step"])
        self._schedule(opt, m._user_entity_embedding.weight.device, t + 2)
        if self.key != self._key(B, opt, ps, sts):
            self._capture(B, opt, ps, sts)
        b = self.buf
        dev = b["t"].device
        n = m._user_num + m._entity_num
        bd = self._bounds
        bd[0] = bd[1] = bd[2] = n
        bd[3] = m._relation_num
        m._ids.check_multi("TRAIN_KG ids", (ids[0], ids[2], ids[3], ids[1]), bd, b["ids"], dev)
        if self.t_dev_value != t:
            b["t"].fill_(t)  # eager steps ran since the last replay
            self.t_dev_value = t
        self.g["fwd"].replay()
        self.pending = "fwd"
        self.replays += 1
        return b["loss"]

    def backward(self, gout: torch.Tensor | None) -> None:
        """The upstream gradient into the graphs' input; the TransR backward runs in the update graph.
        ``gout`` None: the plain ``loss.backward()`` (upstream gradient 1, written only when a scaled one
        was there before)."""
        if self.pending != "fwd":
            raise RuntimeError("TRAIN_KG backward: the captured step's forward buffers were reused by a later "
                               "TRAIN_KG forward before this backward ran")
        if gout is None:
            if not self.gout_one:
                self.buf["gout"].fill_(1.0)
                self.gout_one = True
        else:
            self.buf["gout"].copy_(gout.reshape(1))
            self.gout_one = False
        self.pending = "bwd"

    def update(self, opt) -> None:
        """The update graph (TransR backward + the three Adam steps): the host advances the optimiser
        states' step counters as FusedAdam does."""
        m = self.model
        lz = m._lazy_kg
        ps, sts = self._states(opt)
        if int(sts[0]["step"]) + 1 - lz.flushed_at >= lz.CAP:
            lz.catch_up(opt)  # no row may fall a whole history behind
        for p in ps:
            opt._advance(id(p), p.data)
        lz.dirty = True
        self.g["upd"].replay()
        self.t_dev_value = int(sts[0]["step"])
        self.pending = None

    def release(self) -> None:
        """A forward whose backward never ran (or a step abandoned after it): the batch rows' map is reset."""
        if self.pending is not None:
            kernels.frontier_reset(self.buf["rows"], self.model._kg_table_update.node_map())
            self.pending = None

    @torch.no_grad()
    def materialize(self) -> None:
        """The pending step's gradients into ``.grad`` (the backward graph; the table's compact rows
        scattered into a zero [N, d] gradient, as the fused KG update's materialisation); the map is reset."""
        if self.pending == "fwd":
            self.release()
            return
        if self.pending != "bwd":
            return
        m = self.model
        b = self.buf
        self.g["bwd"].replay()
        emb = m._user_entity_embedding.weight
        g = kernels.zeros(tuple(emb.shape), emb.device)
        kernels.scatter_rows(g, b["rows"], b["Gc"][:b["rows"].numel()], accumulate=False)
        for p, gg in ((emb, g), (m._relation_embedding.weight, b["d_rel"].clone()),
                      (m._trans_matrix, b["d_trans"].clone())):
            if p.grad is None:
                p.grad = gg
            else:
                kernels.add_(p.grad, gg)
        self.release()


class _StepLoss(torch.Tensor):
    """A step loss whose plain ``loss.backward()`` -- no gradient argument, no retain_graph / create_graph /
    inputs, the reference training loops' call (main.py:312, 340) -- runs its step's backward directly
    (``grad_fn.fast_backward``) instead of through the autograd engine: no ones_like fill launch and no
    hand-off to the engine's device thread (~30-50 us of host time per call, the bulk of a captured KG
    step's host cost).  Opt-in: the node carries a ``fast_backward`` only when the model's
    ``direct_backward`` is on (``driver.py`` and ``bench.py`` turn it on for their own loops).  It skips
    every hook the engine would run, and the hooks C++ code installs on a leaf's AccumulateGrad node (DDP's
    reducer, ``register_multi_grad_hook``) are not visible from Python -- so a model wrapped that way must
    leave ``direct_backward`` off, its default.  Even when on, the engine takes over for anything else: a
    scaled or summed loss, ``torch.autograd.backward``, ``retain_graph`` / ``create_graph`` / ``inputs``, a
    hook on the loss itself, a leaf with Python-visible gradient hooks or a non-leaf parameter -- the same
    state transitions either way; a second backward raises as the engine's would.  The direct call runs
    under ``no_grad`` as the engine's backward does.  Every other operation sees a plain tensor."""

    __torch_function__ = torch._C._disabled_torch_function_impl

    def backward(self, gradient=None, retain_graph=None, create_graph=False, inputs=None):
        node = self.grad_fn
        fast = getattr(node, "fast_backward", None) if node is not None else None
        if (fast is not None and gradient is None and not retain_graph and not create_graph and inputs is None
                and not self._backward_hooks):
            node.fast_backward = None
            try:
                with torch.no_grad():
                    fast(node)
                return None
            except _UseEngine:
                pass
        return super().backward(gradient, retain_graph, create_graph, inputs)


def _kg_fast_backward(ctx) -> None:
    if any(getattr(p, "_post_accumulate_grad_hooks", None) or getattr(p, "_backward_hooks", None)
           for p in ctx.leaves):
        ctx.fast_backward = _kg_fast_backward
        raise _UseEngine
    step, ctx.step = ctx.step, None
    if step is None:
        raise RuntimeError("Trying to backward through the graph a second time")
    step.backward(None)


class _KGGraphLoss(torch.autograd.Function):
    """The captured KG step's loss node: forward replays the forward graph (its loss copied out, so a
    kept loss survives the next step), backward hands the upstream gradient to the update graph."""

    @staticmethod
    def forward(ctx, step, ids, opt, states, emb, rel_emb, trans):
        ctx.step = step
        ctx.leaves = (emb, rel_emb, trans)
        ctx.fast_backward = _kg_fast_backward if step.model.direct_backward else None
        return step.forward(ids, opt, *states).clone().view(()).as_subclass(_StepLoss)

    @staticmethod
    def backward(ctx, gout):
        step, ctx.step = ctx.step, None
        ctx.fast_backward = None
        if step is None:
            raise RuntimeError("Trying to backward through the graph a second time")
        step.backward(gout.to(torch.float32))
        return None, None, None, None, None, None, None


class _MarkedBatch:
    """The batch rows a forward marked in ``graph.node_map`` (and, with 2 layers, the first hop it left
    in the graph's hop buffers) for its own backward -- at most one outstanding per graph."""

    def __init__(self, rows: torch.Tensor, count: torch.Tensor | None = None, cleared: int = 0):
        self.rows = rows
        self.count = count
        self.stale = False
        # kernels.PRECLEARED: kgat_cf_begin zeroed the hop bitmaps, PREMARKED: kgat_cf_begin_ex also marked the
        # batch's first hop in them -- and no kgat_frontier_hop has run since
        self.cleared = cleared

    def take_cleared(self) -> int:
        c, self.cleared = self.cleared, 0
        return c


def _release_marks(graph) -> None:
    """Undo an outstanding forward's marks (its loss was dropped, or a second forward came before its
    backward): the map is reset and that forward's backward raises instead of reading reused buffers."""
    tok = getattr(graph, "_marked", None)
    if tok is not None:
        tok.stale = True
        tok.cleared = 0  # the next step's kgat_cf_begin / kgat_frontier_hop own the bitmaps now
        kernels.frontier_reset(tok.rows, graph.node_map)
        graph._marked = None


def _mark_batch(graph, users, pos, neg, marks=None):
    """frontier_build for a forward that hands its marks to its backward: (rows, count, token); ``marks``:
    the (rows, count, token) kgat_cf_begin already made for this step."""
    if marks is not None:
        return marks
    _release_marks(graph)
    rows, fcount = kernels.frontier_build(users, pos, neg, graph.node_map)
    graph._marked = tok = _MarkedBatch(rows, fcount)
    return rows, fcount, tok


def _early_first_hop(graph, users, pos, neg, ws, L: int, hook, marks=None):
    """Data-parallel replicas exchanging the layer-0 hop-set terms (replicas.ShardedGradSync,
    replicated) with 2 layers: the layer-0 hop set is the first hop F + N(F) of the batch rows F,
    fixed by the batch and the graph alone.  It is marked here, before the propagation, and its
    size is all-gathered at once (hook.announce) -- so the host learns the exchange's sizes while
    the GPU runs the forward, instead of synchronising in the middle of the backward.  Returns
    (frontier rows, frontier_hop outputs) for the backward, or None (the backward decides then)."""
    if hook is None or not getattr(hook, "replicated", False) or L != 2 or HOP_DENSE_FRACTION <= 0:
        return None
    W1 = ws[0]
    if not kernels.saved_state_supported(W1.shape[1], W1.shape[0]) or not _hop_small(graph, 0, graph.n_nodes):
        return None
    rows, fcount, tok = _mark_batch(graph, users, pos, neg, marks)
    hop = kernels.frontier_hop(graph, rows, count_host=_hop_host(graph, 0), precleared=tok.take_cleared())
    _hop_record(graph, 0)
    hook.announce(True, hop[2])
    return rows, hop, fcount, tok


def _tile_forward_ok(din: int, dout: int) -> bool:
    """Shapes whose forward can run on a row set (kgat_biinter_fwd_list_f32 / _tiles_f32: the fused
    kernels with their saved state -- norm + sign/keep words)."""
    return kernels.fused_supported(din, dout) and dout <= 128 and (
        kernels.saved_state_supported(din, dout) or kernels.bits_supported(din, dout))


def _frontier_forward(graph, users, pos, neg, X0, ws, drops, seeds, early, marks=None):
    """The forward on the rows the loss can reach only (KGAT.frontier_forward; L = 1, 2 or 3, the
    restricted layers with the fused kernels' saved state).  The BPR loss reads the batch rows F of
    every table (model.py:189-191), so the last layer's output is needed on F only, and layer L-2's
    on the first hop F + N(F) (the last layer gathers its A rows from there) -- the same row sets the
    backward's hop chain runs on; with 3 layers layer 0 stays whole (its output is read on the second
    hop, most rows at C4).  Each restricted layer runs kgat_spmm_csr_rows_f32 on its set's rows and
    kgat_biinter_fwd_list_f32 on the 4-row quads holding them (the set's row list): every row the step
    reads gets the full forward's bits (same edges, order and dropout draws), rows outside are never
    read.  At C2 layer 0's set is 1.7 % of the rows (35 % of the edges), layer 1's the ~768 batch rows.
    Returns (tables, sides, states, early) -- early as _early_first_hop's, for the backward -- or
    None when the shapes do not qualify (the full forward runs)."""
    L = len(drops)
    if L not in (1, 2, 3) or HOP_DENSE_FRACTION <= 0:
        return None
    dims = [X0.shape[1]] + [ws[4 * l].shape[0] for l in range(L)]
    first = max(0, L - 2)  # the first restricted layer
    if not all(_tile_forward_ok(dims[l], dims[l + 1]) for l in range(first, L)):
        return None
    if L == 3 and (early is not None or not kernels.fused_supported(dims[0], dims[1])):
        return None
    if L >= 2 and early is None and not _hop_small(graph, L - 2, graph.n_nodes):
        return None
    n = graph.n_nodes
    if early is None:
        rows, fcount, tok = _mark_batch(graph, users, pos, neg, marks)
        hop = kernels.frontier_hop(graph, rows, count_host=_hop_host(graph, L - 2) if L >= 2 else None,
                                   precleared=tok.take_cleared())
        if L >= 2:
            _hop_record(graph, L - 2)
        early = (rows, hop, fcount, tok)
    rows, hop, fcount, tok = early
    hrows, _, hcount, bits1, fbits = hop
    # layer l's output row set: None = every row (layer 0 of 3), the first hop for layer L-2, the batch
    # rows F for the last layer
    sets = [None] * first + [(hrows, hcount, bits1)] * (L - 1 - first) + [(rows, fcount, fbits)]
    tables, sides, states = [X0], [], []
    x = X0
    for l in range(L):
        W1, b1, W2, b2 = ws[4 * l: 4 * l + 4]
        st = kernels.make_state(n, dims[l], dims[l + 1], x.device)
        if sets[l] is None:
            s, x = kernels.propagate_layer(graph, x, W1, b1, W2, b2, drops[l], seeds[l], state=st)
        else:
            out_rows, out_count, out_bits = sets[l]
            s = kernels.spmm_rows(graph, x, torch.empty(n, dims[l], dtype=torch.float32, device=x.device), out_rows,
                                  out_count, out_bits)
            x = kernels.biinter_fwd_list(x, s, W1, b1, W2, b2, drops[l], seeds[l],
                                         torch.empty(n, dims[l + 1], dtype=torch.float32, device=x.device),
                                         out_rows, out_count, state=st)
        sides.append(s)
        states.append(st)
        tables.append(x)
    # L = 1: the backward's last layer needs the batch rows only (no hop set is handed over)
    return tables, sides, states, (early if L >= 2 else (rows, None, fcount, tok))


def _saved(tables, states, l) -> dict:
    """Layer l's forward output + saved state for the backward (none: it recomputes)."""
    return {} if states[l] is None else {"H": tables[l + 1], "state": states[l]}


class _CFLoss(torch.autograd.Function):
    """Whole CF step as one autograd node: propagation + BPR, forward and backward.

    forward (model.py:124-140, 165-202): for each layer l
        S_l = A . X_l                       (kgat_spmm_csr_f32)
        X_{l+1} = biinter(X_l, S_l)        (kgat_biinter_fwd_f32)
      loss = BPR over the gathered rows of [X_0 | ... | X_L] (kgat_bpr_fwd_f32)
    backward: the last layer's upstream gradient is nonzero only on the
    distinct batch rows F (<= 3B, model.py:189-191 gathers nothing else), so
      dH_L[F] = scatter(dBPR) (compact), (dXd, dS, dW) = biinter_bwd on F rows,
      dX_{L-1} = dXd + A^T . dS  with the A^T gather restricted to F
    (kgat_spmm_csr_masked_ex_f32; equal to the dense product).  That product
    also flags the rows it reached: dX_{L-1} is zero outside F + N(F), the
    next "hop set".  Each lower layer runs the same way on its hop set
    (kgat_hop_compact lists it; compact biinter_bwd; masked A^T product that
    flags the next hop) while the set holds <= HOP_DENSE_FRACTION of the
    nodes -- at C2 the layer-0 hop set is 1.7 % of the rows but 35 % of the
    edges.  Once a hop set is larger, the remaining layers l run densely:
        (dXd, dS_l, dW) = biinter_bwd(...)   (kgat_biinter_bwd_f32)
        dXd += scatter(dBPR_l)               (kgat_bpr_bwd_f32)
        dX_l = dXd + A^T . dS_l              (spmm on the transposed CSR, accumulate;
                                              for l = 0 optionally by row blocks, see
                                              replicas.ShardedGradSync.attach)
    """

    @staticmethod
    def forward(ctx, users, pos, neg, cfg, X0, *ws):
        graph, drops, seeds, reg, hook, _tu, frontier, marks = cfg
        ctx.marks = marks
        ctx.early = _early_first_hop(graph, users, pos, neg, ws, len(drops), hook, marks)
        fw = _frontier_forward(graph, users, pos, neg, X0, ws, drops, seeds, ctx.early, marks) if frontier else None
        if fw is not None:
            tables, sides, states, ctx.early = fw
        else:
            tables, sides, states = [X0], [], []
            x = X0
            for l in range(len(drops)):
                W1, b1, W2, b2 = ws[4 * l: 4 * l + 4]
                st = kernels.make_state(x.shape[0], W1.shape[1], W1.shape[0], x.device)
                s, x = kernels.propagate_layer(graph, x, W1, b1, W2, b2, drops[l], seeds[l], state=st)
                sides.append(s)
                states.append(st)
                tables.append(x)
        loss, coef = kernels.bpr_fwd(tables, users, pos, neg, reg)
        ctx.cfg = cfg
        ctx.tables, ctx.sides, ctx.states, ctx.ws = tables, sides, states, ws
        ctx.ids = (users, pos, neg)
        ctx.coef = coef
        ctx.leaves = (X0, *ws)
        ctx.fast_backward = _cf_fast_backward
        return loss.view(()).as_subclass(_StepLoss)

    @staticmethod
    def backward(ctx, gout):
        ctx.fast_backward = None
        if ctx.tables is None:
            raise RuntimeError("Trying to backward through the graph a second time")
        graph, drops, seeds, reg, hook, tu, _frontier, _marks = ctx.cfg
        tables, sides, states, ws = ctx.tables, ctx.sides, ctx.states, ctx.ws
        users, pos, neg = ctx.ids
        gout = gout.reshape(1).to(torch.float32).contiguous()
        L = len(drops)
        n_nodes = graph.n_nodes
        wgrads: list[torch.Tensor | None] = [None] * (4 * L)
        hit = graph.hop_buffers()[0] if L > 1 else None
        # ---- last layer on the batch frontier
        early, ctx.early = ctx.early, None
        marks, ctx.marks = ctx.marks, None
        tok = early[3] if early is not None else (marks[2] if marks is not None else None)
        if tok is not None and tok.stale and early is None:
            tok = None  # a later forward released this step's marks (two losses, one backward): number them again
        if tok is not None:
            if tok.stale:
                raise RuntimeError("TRAIN_CF backward: a later TRAIN_CF forward on this graph reused the batch-row "
                                   "marks and hop buffers this step's forward left for it (each TRAIN_CF forward "
                                   "needs its backward before the next forward)")
            graph._marked = None  # consumed: this backward resets the marks itself
            rows, fcount = (early[0], early[2]) if early is not None else (marks[0], marks[1])
        else:
            _release_marks(graph)  # a dropped forward's marks would collide with this batch's
            rows, fcount = kernels.frontier_build(users, pos, neg, graph.node_map)
            tok = _MarkedBatch(rows, fcount)
        if early is not None and early[1] is None:
            early = None  # 1-layer frontier forward: the batch rows only
        # a rank that announced its layer-0 hop set to the replicas (forward) is committed to the hop path
        sparse = early is not None or (hit is not None and HOP_DENSE_FRACTION > 0)
        nxt = L - 2
        first_hop = early is not None or (sparse and states[nxt] is not None and states[nxt].kind == "fused"
                                          and _hop_small(graph, nxt, n_nodes))
        # The BPR loss's direct gradients of the batch rows (model.py:189-191 gathers every layer's table) in
        # one launch (kgat_bpr_bwd_multi_f32), each folded into the kernel that produces that table's
        # gradient rows: the last layer's is dH itself, layer L-1's is added by the first-hop A^T product
        # (Gc), layer L-2's by its hop-set bi-interaction backward (G), which also resets the batch-row map
        # -- instead of a zero fill, three kgat_bpr_bwd_f32 launches and a kgat_frontier_reset (same bits)
        B = users.numel()
        fold2 = first_hop and L >= 2 and states[nxt] is not None and states[nxt].kind == "fused"
        dsts: list = [None] * (L + 1)
        dsts[L] = dHc = torch.empty(rows.numel(), tables[L].shape[1], dtype=torch.float32, device=users.device)
        if first_hop:
            dsts[L - 1] = torch.empty(3 * B, tables[L - 1].shape[1], dtype=torch.float32, device=users.device)
        if fold2:
            dsts[nxt] = torch.empty(3 * B, tables[nxt].shape[1], dtype=torch.float32, device=users.device)
        t0 = min(k for k, d in enumerate(dsts) if d is not None)
        kernels.bpr_bwd_multi(tables, t0, users, pos, neg, reg, ctx.coef, gout, dsts, rows, fcount)
        l = L - 1
        dXdc, dSc, dW1, db1, dW2, db2 = kernels.biinter_bwd(tables[l], sides[l], dHc, *ws[4 * l: 4 * l + 4],
                                                            drops[l], seeds[l], rows=rows, **_saved(tables, states, l))
        bits = graph.hop_buffers()[6]
        rank = graph.hop_buffers()[9]  # rank words of the current hop set (frontier_hop / hop_compact)
        pending = None
        if first_hop:
            # first hop marked from the frontier rows' A edges (no graph scan); the A^T product is
            # computed on those rows only, compactly (kgat_spmm_csr_masked_rows_ex_f32)
            if early is not None:
                hrows, hmap, hcount, bits, fbits = early[1]
            else:
                hrows, hmap, hcount, bits, fbits = kernels.frontier_hop(graph, rows, count_host=_hop_host(graph, nxt),
                                                                        precleared=tok.take_cleared())
                _hop_record(graph, nxt, exact=states[nxt] is None or states[nxt].kind != "fused")
            # hop position -> frontier position of the batch rows (the G rows layer L-2's backward adds)
            gidx = None
            if fold2:
                gidx = getattr(graph, "_hop_src", None)
                if gidx is None or gidx.numel() != n_nodes:
                    gidx = graph._hop_src = torch.empty(n_nodes, dtype=torch.int32, device=users.device)
            dX = kernels.spmm_masked_rows(graph, graph.node_map, fbits, dSc, dXdc, hrows, hmap, hcount, bits,
                                          Gc=dsts[L - 1], out_src=gidx)
            if not fold2:
                kernels.frontier_reset(rows, graph.node_map)
            pending = (hrows, hmap, hcount)
        else:
            kernels.map_bits(graph.node_map, bits)
            dX = kernels.spmm_masked(graph, graph.node_map, dSc, Yc_init=dXdc, transpose=True, row_hit=hit,
                                     src_bits=bits)
            kernels.frontier_reset(rows, graph.node_map)
            kernels.bpr_bwd(tables, l, users, pos, neg, reg, ctx.coef, gout, dX)
        wgrads[4 * l: 4 * l + 4] = [dW1, db1, dW2, db2]
        # ---- remaining layers: on the hop set while it stays small, then densely
        for l in range(L - 2, -1, -1):
            W1, b1, W2, b2 = ws[4 * l: 4 * l + 4]
            fused = states[l] is not None and states[l].kind == "fused"
            compact_dh = pending is not None
            n_hop = None
            if compact_dh:  # dX is compact over the first hop set
                hrows, hmap, hcount = pending
                pending = None
                if not fused:  # the wide kinds size their compact problem on the host
                    est = graph._hop_est[l]
                    if graph._hop_exact.get(l):
                        est[1].synchronize()
                    else:  # listed by a forward that recorded no event (a data-parallel early first hop)
                        torch.cuda.current_stream(users.device).synchronize()
                    n_hop = int(est[0][0])
            elif sparse and fused:
                # hop size stays on the device (no host sync); the sparse/dense choice uses the
                # size this layer's hop set had at the previous step
                sparse = _hop_small(graph, l, n_nodes)
                if sparse:
                    hrows, hmap, hcount, _ = kernels.hop_compact(graph, count_host=_hop_host(graph, l))
                    _hop_record(graph, l)
                else:
                    _hop_reprobe(graph, l)
            elif sparse:
                # the wide kinds size their compact problem on the host (one synchronisation) -- taken only
                # when the layer's hop set was small at the previous step; a large one goes dense at once
                # (both paths give the same bits; C3's 3-layer step: its ~80 us stall gone)
                sparse = _hop_small(graph, l, n_nodes)
                if sparse:
                    hrows, hmap, hcount, n_hop = kernels.hop_compact(graph, sync=True,
                                                                     count_host=_hop_host(graph, l))
                    _hop_record(graph, l)
                    sparse = n_hop <= HOP_DENSE_FRACTION * n_nodes
                else:
                    _hop_reprobe(graph, l)
            if sparse:
                # dX is zero outside the hop set: the bi-interaction backward runs on its rows
                # only and the A^T product gathers from them only (kgat_spmm_csr_masked_ex_f32);
                # per row and per output element the arithmetic and order are the dense path's
                packed = None
                if fused:
                    out_rows, out = n_nodes, None
                    cap = hook.exchange_cap() if l == 0 and hook is not None and hook.replicated else None
                    if cap is not None:
                        # the replicas' exchange buffer [cap, 2d] = dS | dXd, written by the backward itself
                        din = W1.shape[1]
                        packed = torch.empty(cap, 2 * din, dtype=torch.float32, device=dX.device)
                        out_rows, out = cap, (packed[:, din:], packed[:, :din])
                    gfold = fold2 and l == nxt
                    dXdc, dSc, dW1, db1, dW2, db2 = kernels.biinter_bwd_hop(
                        tables[l], sides[l], dX, W1, W2, drops[l], hrows, hcount, tables[l + 1], states[l], out_rows,
                        dh_compact=compact_dh, out=out, G=dsts[l] if gfold else None,
                        gidx=gidx if gfold else None, gmap=graph.node_map if gfold else None)
                elif compact_dh:
                    # wide kinds after the first-hop product: dX holds the hop rows compactly
                    hr = hrows[:n_hop]
                    dXdc, dSc, dW1, db1, dW2, db2 = kernels.biinter_bwd(tables[l], sides[l], dX[:n_hop], W1, b1, W2,
                                                                        b2, drops[l], seeds[l], rows=hr,
                                                                        **_saved(tables, states, l))
                    hrows = hr
                else:
                    # wide kinds: H, dH and the state read through the hop list (X / S gathered once)
                    dXdc, dSc, dW1, db1, dW2, db2 = kernels.biinter_bwd(tables[l], sides[l], dX, W1, b1, W2, b2,
                                                                        drops[l], seeds[l], rows=hrows,
                                                                        dh_full=True, **_saved(tables, states, l))
                if not (fold2 and l == nxt):
                    kernels.bpr_bwd(tables, l, users, pos, neg, reg, ctx.coef, gout, dXdc, row_map=hmap)
                if l == 0 and hook is not None and hook.replicated:
                    # data-parallel replicas exchange the compact hop-set terms and each computes the
                    # mean table gradient A^T . mean(dS) + mean(dXd) itself (replicas.ShardedGradSync)
                    dX = hook.table_grad_hop(graph, hmap, hrows, hcount, dSc, dXdc, rank, deferral=tu, packed=packed)
                elif l == 0 and hook is not None:
                    dX = torch.empty(n_nodes, dSc.shape[1], dtype=torch.float32, device=dSc.device)
                    for k, view in enumerate(graph.transpose_row_blocks(hook.bounds)):
                        kernels.spmm_block_masked(view, hmap, dSc, dX[view.r0:view.r0 + view.n_rows],
                                                  Yc_init=dXdc, row0=view.r0, src_rank=rank)
                        hook.block_ready(k, dX)
                    # the exchange owns the table gradient now (its blocks are in flight): autograd gets
                    # none (it would copy the whole [N, d] tensor), ShardedGradSync.reduce hands it over
                    dX = None
                elif l == 0 and tu is not None and tu.defer(graph, hmap, dSc, dXdc, rank):
                    dX = None  # computed fused with the table's Adam step by update_cf_weights
                else:
                    dX = kernels.spmm_masked(graph, hmap, dSc, Yc_init=dXdc, transpose=True,
                                             row_hit=hit if l > 0 else None, src_rank=rank)
                wgrads[4 * l: 4 * l + 4] = [dW1, db1, dW2, db2]
                continue
            dXd, dS, dW1, db1, dW2, db2 = kernels.biinter_bwd(tables[l], sides[l], dX, W1, b1, W2, b2, drops[l],
                                                              seeds[l], **_saved(tables, states, l))
            kernels.bpr_bwd(tables, l, users, pos, neg, reg, ctx.coef, gout, dXd)
            if l == 0 and hook is not None and hook.replicated:
                dXd = hook.table_grad_dense(graph, dS, dXd)
            elif l == 0 and hook is not None:
                # the table gradient by row blocks: each block's exchange (replicas.ShardedGradSync)
                # starts while the next block's A^T . dS is computed
                for k, view in enumerate(graph.transpose_row_blocks(hook.bounds)):
                    kernels.spmm_block(view, dS, dXd[view.r0:view.r0 + view.n_rows], accumulate=True)
                    hook.block_ready(k, dXd)
                dXd = None  # owned by the exchange (see the hop branch)
            else:
                kernels.spmm(graph, dS, out=dXd, transpose=True, accumulate=True)
            wgrads[4 * l: 4 * l + 4] = [dW1, db1, dW2, db2]
            dX = dXd
        ctx.tables = ctx.sides = ctx.states = None
        return (None, None, None, None, dX, *wgrads)


_ONE: dict = {}  # device -> a resident fp32 1.0 (the plain backward's upstream gradient)


def _cf_fast_backward(ctx) -> None:
    """``loss.backward()`` of a TRAIN_CF loss without the engine (model._StepLoss): the node's backward with
    upstream gradient 1, its gradients accumulated into the leaves as the engine's AccumulateGrad does (set, or
    added in place).  Only reached with ``KGAT.direct_backward`` on (see _StepLoss); a non-leaf parameter or a
    leaf with Python-visible gradient hooks still sends the call through the engine."""
    leaves = ctx.leaves
    if any(not p.is_leaf or getattr(p, "_post_accumulate_grad_hooks", None) or getattr(p, "_backward_hooks", None)
           for p in leaves if p is not None):
        ctx.fast_backward = _cf_fast_backward
        raise _UseEngine
    dev = ctx.coef.device
    one = _ONE.get(dev)
    if one is None:
        one = _ONE[dev] = torch.ones((), dtype=torch.float32, device=dev)
    grads = _CFLoss.backward(ctx, one)[4:]
    with torch.no_grad():
        for p, g in zip(leaves, grads):
            if g is None or p is None or not p.requires_grad:
                continue
            if p.grad is None:
                p.grad = g.detach()
            else:
                p.grad.add_(g)


class _UseEngine(Exception):
    """A fast backward declined (model._StepLoss falls back to the autograd engine)."""


class _KGLoss(torch.autograd.Function):
    """TransR KG loss as one autograd node (model.py:204-261): kgat_transr_fwd_f32 /
    kgat_transr_bwd_f32.  Gradients: dense table (zero except the gathered rows,
    as nn.Embedding's dense backward), relation embeddings, trans matrices.  With the
    fused KG table update (_KGTableUpdate) the table's rows are handed over compactly
    instead and the table gets no .grad."""

    @staticmethod
    def forward(ctx, heads, rels, pos, neg, reg, ktu, emb, rel_emb, trans):
        loss, work = kernels.transr_fwd(emb, rel_emb, trans, heads, rels, pos, neg, reg)
        ctx.save_for_backward(heads, rels, pos, neg, work, emb)
        ctx.shape = (rel_emb.shape[0], rel_emb.shape[1])
        ctx.ktu = ktu
        ctx.rows = ktu.marked if ktu is not None else None
        return loss.view(())

    @staticmethod
    def backward(ctx, gout):
        heads, rels, pos, neg, work, emb = ctx.saved_tensors
        n_rel, k = ctx.shape
        gout = gout.reshape(1).to(torch.float32).contiguous()
        ktu, ctx.ktu = ctx.ktu, None
        rows = ctx.rows
        if ktu is not None and rows is not None and ktu.marked is rows and ktu.wants(heads.numel()):
            row_map = ktu.node_map()
            ktu.marked = None  # handed to the table update, which resets the map after its step
            Gc, d_rel, d_trans = kernels.transr_bwd_compact(emb, n_rel, k, heads, rels, pos, neg, work, gout, row_map,
                                                            rows.numel())
            ktu.defer(rows, Gc)
            return None, None, None, None, None, None, None, d_rel, d_trans
        if ktu is not None:
            ktu.release()
        d_emb, d_rel, d_trans = kernels.transr_bwd(emb, n_rel, k, heads, rels, pos, neg, work, gout)
        return None, None, None, None, None, None, d_emb, d_rel, d_trans


class KGAT(nn.Module):
    def __init__(self, args: KGATArgs) -> None:
        super().__init__()
        self._user_num = args.user_num
        self._entity_num = args.entity_num
        self._relation_num = args.relation_num
        self._message_dropout = list(args.message_dropout)
        self._layer_dims = list(args.layer_size)
        self._layer_num = len(self._layer_dims)
        self._regularization_params = list(args.regularization_params)
        self._cf_embedding_dim = args.cf_embedding_dim
        self._kg_embedding_dim = args.kg_embedding_dim
        n = self._user_num + self._entity_num
        # creation / init order as the reference (model.py:58-97) => same RNG stream
        self._user_entity_embedding = nn.Embedding(n, self._cf_embedding_dim)
        self._relation_embedding = nn.Embedding(self._relation_num, self._kg_embedding_dim)
        self._trans_matrix = nn.Parameter(torch.Tensor(self._relation_num, self._cf_embedding_dim,
                                                       self._kg_embedding_dim))
        nn.init.xavier_uniform_(self._user_entity_embedding.weight)
        nn.init.xavier_uniform_(self._relation_embedding.weight)
        nn.init.xavier_uniform_(self._trans_matrix)
        self._aggregator_layers = nn.ModuleList()
        dims = [self._cf_embedding_dim, *self._layer_dims]
        for l in range(self._layer_num):
            self._aggregator_layers.append(Aggregator(dims[l], dims[l + 1], self._message_dropout[l]))
        self.attentive_matrix = nn.Parameter(torch.sparse_coo_tensor(
            torch.empty((2, 0), dtype=torch.long), torch.empty((0,), dtype=torch.float32), (n, n)))
        if args.attentive_matrix is not None:
            self.attentive_matrix.data = args.attentive_matrix
        self.attentive_matrix.requires_grad = False
        self._multi_head_attention = MultiHeadAttention(self._cf_embedding_dim, self._kg_embedding_dim)
        self._graph: DeviceGraph | None = None
        self._graph_key = None
        self._ids = _IdGuard()
        self._table_update = _TableUpdate(self._user_entity_embedding.weight)
        self._kg_table_update = _KGTableUpdate(self._user_entity_embedding.weight)
        self._lazy_kg = _LazyKGAdam(self._user_entity_embedding.weight)
        self._kg_graph = _KGStepGraph(self)
        # Opt-in: TRAIN_CF's forward computes each layer on the rows the loss can reach only
        # (_frontier_forward) -- same loss, gradients and updates, bit for bit
        self.frontier_forward = False
        # Opt-in: a plain ``loss.backward()`` of a TRAIN_CF / captured TRAIN_KG loss runs the step's backward
        # without the autograd engine (_StepLoss).  Leave it off under wrappers that hook the leaves' gradient
        # accumulators from C++ (DistributedDataParallel): the direct call cannot see those hooks
        self.direct_backward = False

    @property
    def lazy_kg_adam(self) -> bool:
        """Opt-in (with ``fuse_kg_table_update``): the KG step's table Adam on the batch rows only, the
        other rows' zero-gradient steps replayed when they are next read (_LazyKGAdam; same bits)."""
        return self._lazy_kg.enabled

    @lazy_kg_adam.setter
    def lazy_kg_adam(self, on: bool) -> None:
        if not on:
            self.flush_kg_table()
            self._lazy_kg.last = None  # every row current: dense steps from here on
        self._lazy_kg.enabled = bool(on)

    def flush_kg_table(self) -> None:
        """Bring every table row and the KG optimiser's moments up to the current KG step (lazy_kg_adam)."""
        if self._lazy_kg.last is not None and getattr(self, "_kg_optimizer", None) is not None:
            self._lazy_kg.catch_up(self._kg_optimizer)

    def state_dict(self, *args, **kwargs):
        self.flush_kg_table()
        return super().state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        self.flush_kg_table()
        out = super().load_state_dict(state_dict, strict=strict, assign=assign)
        self._lazy_kg.last = None  # every row is current: restart the lazy state at the next KG step
        return out

    @property
    def fuse_table_update(self) -> bool:
        """Opt-in: leave the CF step's table gradient to ``update_cf_weights``, which computes it
        fused with the table's Adam step (_TableUpdate); ``table.grad`` is None in between."""
        return self._table_update.enabled

    @fuse_table_update.setter
    def fuse_table_update(self, on: bool) -> None:
        if not on:
            self._table_update.materialize()
        self._table_update.enabled = bool(on)

    @property
    def fuse_kg_table_update(self) -> bool:
        """Opt-in: the KG step's table gradient stays compact and ``update_kg_weights`` steps the
        table from it (_KGTableUpdate); ``table.grad`` is None in between."""
        return self._kg_table_update.enabled

    @fuse_kg_table_update.setter
    def fuse_kg_table_update(self, on: bool) -> None:
        if not on:
            self._kg_table_update.materialize()
        self._kg_table_update.enabled = bool(on)

    def materialize_table_grad(self) -> None:
        """Write a deferred table gradient (CF or KG step) into ``_user_entity_embedding.weight.grad``."""
        self._table_update.materialize()
        self._kg_table_update.materialize()
        self._kg_graph.materialize()

    @property
    def capture_kg_step(self) -> bool:
        """Opt-in (with ``fuse_kg_table_update`` and ``lazy_kg_adam``): TRAIN_KG's forward, its backward and
        ``update_kg_weights`` each replay one captured HIP graph (_KGStepGraph; same bits)."""
        return self._kg_graph.enabled

    @capture_kg_step.setter
    def capture_kg_step(self, on: bool) -> None:
        if not on:
            self._kg_graph.materialize()
            self._kg_graph.g = self._kg_graph.buf = self._kg_graph.key = None
        self._kg_graph.enabled = bool(on)

    # ------------------------------------------------------------------ graph
    def graph(self) -> DeviceGraph:
        """The HBM-resident CSR view of ``attentive_matrix`` (built once per change)."""
        A = self.attentive_matrix.data
        dev = self._user_entity_embedding.weight.device
        if self._graph is None or self._graph_key != self._matrix_key():
            if dev.type != "cuda":
                raise RuntimeError("KGAT runs on the MI355X HIP path only: move the model to a GPU first")
            n = self._user_num + self._entity_num
            Ac = A.coalesce() if A.is_sparse else A.to_sparse().coalesce()
            idx = Ac.indices().cpu().numpy()
            rowptr, col, val = csr_from_coo(n, idx[0], idx[1], Ac.values().detach().cpu().numpy())
            layout = GraphLayout(n_nodes=n, rel_order=[], heads=np.zeros(0, np.int64), rels=np.zeros(0, np.int64),
                                 tails=np.zeros(0, np.int64), edge_vals=np.zeros(0, np.float32), rowptr=rowptr,
                                 col=col, val=val, slot=np.zeros(0, np.int64))
            self._graph = DeviceGraph(layout, dev)
            # the public COO parameter shares the device value buffer from now on
            rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rowptr))
            coo = torch.sparse_coo_tensor(torch.from_numpy(np.vstack([rows, col.astype(np.int64)])).to(dev),
                                          self._graph.A.val, (n, n), is_coalesced=True)
            self.attentive_matrix.data = coo
            self._graph_key = self._matrix_key()
        return self._graph

    def _matrix_key(self):
        """Identity of the attentive matrix storage (a new Python object per ``.data`` access)."""
        A = self.attentive_matrix.data
        vals = A._values() if A.is_sparse else A
        return (vals.data_ptr(), vals.numel(), A._version, str(A.device),
                str(self._user_entity_embedding.weight.device))

    def attach_graph(self, layout: GraphLayout, device: torch.device | str | None = None) -> DeviceGraph:
        """Move the model to ``device`` and make ``layout`` the attentive matrix directly.

        Equivalent to passing ``KGATArgs(attentive_matrix=...)`` with the
        layout's COO, without the host round trip through a torch sparse tensor
        (the path used for the 10^7-10^9-edge synthetic graphs).
        """
        if device is not None:
            self.to(device)
        dev = self._user_entity_embedding.weight.device
        n = self._user_num + self._entity_num
        if layout.n_nodes != n:
            raise ValueError(f"layout has {layout.n_nodes} nodes, model has {n}")
        self._graph = DeviceGraph(layout, dev)
        rows = torch.repeat_interleave(torch.arange(n, device=dev), torch.diff(self._graph.A.rowptr))
        coo = torch.sparse_coo_tensor(torch.stack([rows, self._graph.A.col.long()]), self._graph.A.val, (n, n),
                                      is_coalesced=True)
        self.attentive_matrix.data = coo
        self._graph_key = self._matrix_key()
        return self._graph

    def _cf_weights(self) -> list[torch.Tensor]:
        return [w for agg in self._aggregator_layers for w in agg.weights()]

    def _dropouts(self) -> tuple[list[float], list[int]]:
        drops = [agg.dropout if self.training else 0.0 for agg in self._aggregator_layers]
        seeds = [int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0 for p in drops]
        return drops, seeds

    # ------------------------------------------------------------ propagation
    def _propagate(self) -> list[torch.Tensor]:
        """[X0, H1, ..., HL] without building autograd state (model.py:124-140)."""
        g = self.graph()
        drops, seeds = self._dropouts()
        with torch.no_grad():
            x = self._user_entity_embedding.weight.detach()
            tables = [x]
            for l, agg in enumerate(self._aggregator_layers):
                _, x = kernels.propagate_layer(g, x, *[w.detach() for w in agg.weights()], drops[l], seeds[l])
                tables.append(x)
        return tables

    def propagate(self) -> list[torch.Tensor]:
        """The propagated tables [X0, H1, ..., HL] (no autograd state): PREDICT's first half,
        computed once per evaluation by evaluation.evaluate / recommend_topk."""
        self.flush_kg_table()
        return self._propagate()

    def _build_cf_embeddings(self) -> torch.Tensor:
        return torch.cat(self._propagate(), dim=1)

    # ------------------------------------------------------------------ modes
    def _calc_cf_loss(self, user_ids, positive_item_ids, negative_item_ids) -> torch.Tensor:
        g = self.graph()
        drops, seeds = self._dropouts()
        # the data-parallel hook only where a backward follows (a no_grad loss evaluation has none: it must
        # not open the replicas' exchange of a step)
        hook = getattr(self, "_table_grad_hook", None) if torch.is_grad_enabled() else None
        # the frontier forward only where a backward follows: its batch-row map is released by the backward
        frontier = self.frontier_forward and torch.is_grad_enabled()
        marks = None
        if torch.is_grad_enabled():
            # ids checked and numbered as the batch frontier, the batch's first hop marked in the spare bitmap
            # pair and the pair the last step used zeroed, in one launch (kgat_cf_begin_ex); the marks go to
            # this step's backward (and frontier forward / DP hop exchange)
            _release_marks(g)
            mark, clear = kernels.hop_bitmaps_next(g)
            # the marking only where a consumer will list the first hop (C3's dense graph: every slot's row
            # holds thousands of entries and the hop path is off there -- 291 us of atomics for nothing);
            # otherwise the current pair is zeroed and a backward that does take the hop path marks it itself
            premark = self._first_hop_wanted(g, drops, frontier or hook is not None)
            r = self._ids.check_cf("TRAIN_CF ids", (user_ids, positive_item_ids, negative_item_ids), g.n_nodes,
                                   g.device, g.node_map, clear, mark=(g, mark) if premark else None)
            if r is not None:
                if premark:
                    kernels.hop_bitmaps_commit(g)
                ids, rows, fcount = r
                g._marked = tok = _MarkedBatch(rows, fcount,
                                               cleared=kernels.PREMARKED if premark else kernels.PRECLEARED)
                marks = (rows, fcount, tok)
        if marks is None:
            ids = self._ids.check("TRAIN_CF ids", (user_ids, positive_item_ids, negative_item_ids), g.n_nodes,
                                  g.device)
        cfg = (g, drops, seeds, float(self._regularization_params[0]), hook, self._table_update, frontier, marks)
        loss = _CFLoss.apply(*ids, cfg, self._user_entity_embedding.weight, *self._cf_weights())
        if not self.direct_backward and loss.grad_fn is not None:
            loss.grad_fn.fast_backward = None  # the autograd engine (the default; _StepLoss)
        return loss

    def _first_hop_wanted(self, g, drops, forward_sets: bool) -> bool:
        """Whether this step's first hop F + N(F) is likely listed: the hop path is on, layer L-2's hop set
        was small at the last step (or is unknown), and a consumer exists -- the frontier forward or the
        replicas' hop exchange (``forward_sets``), or the backward's hop chain, which needs layer L-2's fused
        saved state.  A wrong guess costs time only: unmarked, the backward marks the hop itself."""
        L = len(drops)
        if HOP_DENSE_FRACTION <= 0 or (L >= 2 and not _hop_small(g, L - 2, g.n_nodes)):
            return False
        if forward_sets or L < 2:
            return True
        W1 = self._cf_weights()[4 * (L - 2)]
        return kernels.saved_state_supported(W1.shape[1], W1.shape[0])

    def _calc_kg_loss(self, heads, relations, positive_tails, negative_tails) -> torch.Tensor:
        dev = self._user_entity_embedding.weight.device
        if dev.type != "cuda":
            raise RuntimeError("KGAT runs on the MI355X HIP path only: move the model to a GPU first")
        n = self._user_num + self._entity_num
        step, opt = self._kg_graph, getattr(self, "_kg_optimizer", None)
        if step.enabled and torch.is_grad_enabled():
            step.release()  # a dropped captured forward's batch-row marks
            ids = tuple(torch.as_tensor(t) for t in (heads, relations, positive_tails, negative_tails))
            states = step.usable(ids, opt)
            if states is not None:
                return _KGGraphLoss.apply(step, ids, opt, states, self._user_entity_embedding.weight,
                                          self._relation_embedding.weight, self._trans_matrix)
        h, p, q, r = self._ids.check("TRAIN_KG ids", (heads, positive_tails, negative_tails), n, dev,
                                     more=[((relations,), self._relation_num)])
        ids = [h, r, p, q]
        ktu = self._kg_table_update if torch.is_grad_enabled() else None
        lazy = self._lazy_kg
        if ktu is not None and ktu.wants(h.numel()):
            rows = ktu.mark(h, p, q)  # the batch rows, numbered once for the backward's compact gradient
            if lazy.enabled and getattr(self, "_kg_optimizer", None) is not None:
                # the rows TransR reads, brought up to the last KG step (their skipped steps replayed)
                lazy.ensure(self._kg_optimizer)
                lazy.catch_up(self._kg_optimizer, rows)
        elif lazy.enabled and lazy.last is not None:
            self.flush_kg_table()  # an unfused KG step (no compact rows) reads and updates every row
        return _KGLoss.apply(*ids, float(self._regularization_params[1]), ktu, self._user_entity_embedding.weight,
                             self._relation_embedding.weight, self._trans_matrix)

    def _update_attention(self, heads, relations, tails, relation_indices) -> None:
        """Refresh attentive_matrix in HBM (model.py:318-366): no host round trip."""
        g = self.graph()
        plan = g.refresh_plan(heads, relations, tails)
        if plan is None:  # edge set differs from the current structure: rebuild it from the edges
            h = torch.as_tensor(heads).cpu().numpy().astype(np.int64)
            t = torch.as_tensor(tails).cpu().numpy().astype(np.int64)
            n = self._user_num + self._entity_num
            rowptr, col, val = csr_from_coo(n, h, t, np.zeros(h.size, np.float32))
            layout = GraphLayout(n_nodes=n, rel_order=[int(x) for x in torch.as_tensor(relation_indices).tolist()],
                                 heads=np.zeros(0, np.int64), rels=np.zeros(0, np.int64), tails=np.zeros(0, np.int64),
                                 edge_vals=np.zeros(0, np.float32), rowptr=rowptr, col=col, val=val,
                                 slot=np.zeros(0, np.int64))
            g = self.attach_graph(layout)
            plan = g.refresh_plan(heads, relations, tails)
        mha = self._multi_head_attention
        p = mha.dropout if self.training else 0.0
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
        with torch.no_grad():
            logits = kernels.edge_logits(g, plan, self._user_entity_embedding.weight.detach(),
                                         self._trans_matrix.detach(), mha._value_weight.weight.detach(),
                                         mha._value_weight.bias.detach(), mha._output.weight.detach(),
                                         mha._output.bias.detach(), mha._layer_norm.weight.detach(),
                                         mha._layer_norm.bias.detach(), p, seed)
            kernels.row_softmax(g, logits)

    def _calc_score(self, user_ids, item_ids) -> torch.Tensor:
        """Full propagation, then the fused gather + MFMA score GEMM (model.py:368-391)."""
        u, i = self._ids.check("PREDICT ids", (user_ids, item_ids), self._user_num + self._entity_num,
                               self._user_entity_embedding.weight.device)
        tables = self._propagate()
        return kernels.scores(tables, u, i)

    # ------------------------------------------------------------- optimizers
    def build_optimizer(self, cf_lr: float, kg_lr: float) -> None:
        # lazy KG Adam: the replays still owed are the old optimiser's steps -- apply them, then restart
        # the per-row step record at the new optimiser's t = 0 (a stale last[r] would skip its steps)
        self.flush_kg_table()
        self._lazy_kg.last = None
        self._lazy_kg.dirty = False
        self._cf_optimizer = FusedAdam(self.parameters(), lr=cf_lr)
        self._kg_optimizer = FusedAdam(self.parameters(), lr=kg_lr)

    def raise_pending(self, block: bool = True) -> None:
        """Raise the IndexError of a device-side id check that has not been reported yet."""
        self._ids.raise_pending(block)

    def _raise_or_abandon(self, opt) -> None:
        """Report a device-side id error before an optimiser step.  The step it interrupts is
        abandoned as a whole, as the reference's raising forward leaves no gradient behind: its
        gradients and deferred table updates are dropped, so no later step sums them in."""
        try:
            self._ids.raise_pending()
        except IndexError:
            self._table_update.discard()
            self._kg_table_update.discard()
            self._kg_graph.release()
            hook = getattr(self, "_table_grad_hook", None)
            if hook is not None and opt is getattr(self, "_cf_optimizer", None):
                hook.abandon_step()  # a pipelined owner step's counter goes back (replicas.ShardedGradSync)
            opt.zero_grad()
            raise

    def update_cf_weights(self, row_ranges: dict | None = None) -> None:
        """``row_ranges``: the rows this rank steps (replicas.ShardedGradSync); None = all.
        A deferred table gradient (fuse_table_update) is stepped by the fused product + Adam."""
        # an earlier step's device-side id error surfaces here; this step's own is caught on the
        # device: its optimiser kernels read the check's flag and leave every parameter as it is
        self._raise_or_abandon(self._cf_optimizer)
        self.flush_kg_table()
        tu = self._table_update
        fused = None
        if tu.pending is not None:
            # another term of the loss may have written the table's .grad after the deferral (autograd
            # order, an extra regulariser on the table): the fused launch never reads .grad, so such a
            # gradient is summed with the deferred product first (materialize adds into .grad)
            if (row_ranges and id(tu.param) in row_ranges) or tu.param.grad is not None:
                tu.materialize()
            else:
                fused = {id(tu.param): tu.launch()}
        self._cf_optimizer.step(row_ranges, fused=fused, skip=self._ids.skip_flag())
        self._cf_optimizer.zero_grad()

    def update_kg_weights(self, row_ranges: dict | None = None) -> None:
        """A compact KG table gradient (fuse_kg_table_update) is stepped by kgat_adam_rows_f32."""
        self._raise_or_abandon(self._kg_optimizer)
        self._table_update.materialize()
        step = self._kg_graph
        if step.pending == "bwd":
            ps, _ = step._states(self._kg_optimizer)
            if row_ranges or any(p.grad is not None for p in ps):
                step.materialize()  # another gradient joined this step's: the eager update sums them
            else:
                step.update(self._kg_optimizer)
                self._kg_optimizer.zero_grad()
                return
        step.release()
        ktu, lazy, opt = self._kg_table_update, self._lazy_kg, self._kg_optimizer
        fused = None
        if ktu.pending is not None:
            if (row_ranges and id(ktu.param) in row_ranges) or ktu.param.grad is not None:
                ktu.materialize()
            elif lazy.enabled:
                lazy.ensure(opt)
                if lazy._t(opt) + 1 - lazy.flushed_at >= lazy.CAP:
                    lazy.catch_up(opt)  # no row may fall a whole history behind
                fused = {id(ktu.param): ktu.launch(lazy, opt)}
            else:
                fused = {id(ktu.param): ktu.launch()}
        dense_lazy = lazy.last is not None and fused is None and ktu.param.grad is not None
        if dense_lazy:
            lazy.catch_up(opt)  # a dense table step follows: every row current first (no-op when clean)
        opt.step(row_ranges, fused=fused, skip=self._ids.skip_flag())
        if dense_lazy:
            lazy.dense_step_done(opt)
        opt.zero_grad()

    def forward(self, *args: Any, mode: KGATMode) -> torch.Tensor | None:
        if mode != KGATMode.TRAIN_KG:
            self.flush_kg_table()  # lazy KG Adam: these modes read the whole table
        if mode != KGATMode.PREDICT:
            # a deferred table gradient refers to this step's hop buffers and A's values (CF) or
            # holds the batch-row map (KG): a new backward or an attention refresh would change them
            self._table_update.materialize()
            self._kg_table_update.materialize()
            self._kg_graph.materialize()
        if mode == KGATMode.TRAIN_CF:
            return self._calc_cf_loss(*args)
        if mode == KGATMode.TRAIN_KG:
            return self._calc_kg_loss(*args)
        if mode == KGATMode.UPDATE_ATTENTION:
            self._update_attention(*args)
            return None
        if mode == KGATMode.PREDICT:
            return self._calc_score(*args)
        raise ValueError(f"unknown mode {mode}")
