"""Row-sharded KGAT across GPUs -- SURVEY §8(e) mode 2 (the C5 configuration).

A table of 50M x 256 fp32 rows plus two Adam states does not fit one GPU, so
rank k owns a contiguous row range [lo_k, hi_k) of every node table (X0, H1,
..., HL, the side S_l).  It holds the same rows of the attentive matrix A
(``A_loc``: its rows, global column ids) and of its transpose (``AT_loc``:
rows [lo_k, hi_k) of A^T -- the in-edges of its nodes, global column ids).

Forward, per layer (aggregator.py:54-65):
    Xg   = every rank's rows of X_l   all-peer gather (one P2P send + receive per peer,
                                      all in flight together: on a fully connected xGMI
                                      node each peer pair has its own link); optionally in
                                      column chunks, chunk c+1 on the wire while chunk c's
                                      product runs (GATHER_CHUNK)
    S_k  = A_loc . Xg                 the single-GPU SpMM on the local rows: per row the
                                      same edges in the same order as one GPU -- bit for bit
    H_k  = biinter(X_k, S_k)          row-local
Backward ("pull": the transpose of the forward, no reduce-scatter):
    last layer: dS is nonzero on the global batch rows only.  Each rank computes the
      bi-interaction backward of the batch rows it owns; one exact all-reduce (one owner per
      row, zeros elsewhere) gives every rank the compact [dS | dXd] rows of the whole batch;
      dX_k = AT_loc . dS (masked to the batch rows) + dXd -- kgat_spmm_csr_masked_ex_f32
    lower layers: dSg = all-peer gather of dS_l; dX_k = dXd_k + AT_loc . dSg
  Per output row the single-GPU backward's edges in its order, so the propagated tables and the
  table gradient are the single GPU's bit for bit at every world size (whole-width gathers);
  only the aggregator weight gradients (per-rank partial sums, all-reduced) are summed in
  another order.
The BPR loss is taken over the GLOBAL batch (every rank's pairs, as data-parallel
training would): the batch rows are assembled on every rank by one exact all-reduce,
every rank evaluates the same loss, and each keeps the row gradients of the rows it
owns.  Relation / trans gradients of the KG step are already identical on every rank.
Adam runs on the local shard + replicas.

Wire bytes per rank and layer: (G-1)/G of the layer input table forward and of the
layer's dS backward (DESIGN.md §6 has the per-step budget at G = 8).

Transport: ``Comm`` (torch.distributed; RCCL point-to-point on device buffers, or gloo
staged through host memory to run several ranks on one test GPU) or comm.RcclComm (the
library's own kgat_comm_allgatherv / kgat_comm_alltoallv).  All arithmetic is the HIP
kernels of libkgat_hip.so.

Attention refresh (UPDATE_ATTENTION, model.py:318-366): the X0 shards are gathered, rank k
scores the edges of its rows, soft-maxes them over its local CSR rows (A_loc's values), and
an all-to-all moves each refreshed value to the owner of its A^T row (AT_loc's values).
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch
import torch.distributed as dist
from torch import nn

from . import kernels
from . import _lib
from .comm import count_all_gather, count_all_reduce, count_gather, wire
from .graph import GraphLayout, RefreshPlan, _CSRRowView, _DeviceCSR, degree_weights, stream_ptr
from . import model as _model
from .model import Aggregator, KGATArgs, KGATMode, MultiHeadAttention
from .optim import FusedAdam

# Columns per gathered chunk (0 = the whole width in one gather): chunk c+1 travels while chunk c's
# SpMM runs.  Off by default: the SpMM kernel of a narrower width walks a long (hub) row's
# 512-edge segments in a different interleave (spmm.hip: lane groups of d/4 lanes), so a chunked
# gather changes the summation order of hub rows -- within tolerance, but no longer the single
# GPU's bits, which the whole-width gather keeps for every world size (tests/sharded_worker.py).
# KGAT_SHARD_CHUNK=64 trades that for hiding each layer's SpMM under the next chunk's transfer.
GATHER_CHUNK = int(os.environ.get("KGAT_SHARD_CHUNK", "0"))


# ---------------------------------------------------------------- transport
class _Pending:
    def __init__(self, works, copies=()):
        self._works, self._copies = works, copies

    def wait(self) -> None:
        for w in self._works:
            w.wait()
        for dst, src in self._copies:
            dst.copy_(src)


class Comm:
    """Collectives over a torch.distributed group for the row-sharded model."""

    def __init__(self, group=None, host_staged: bool | None = None, force: bool = False):
        """``force``: collectives run even on a world of one rank (tests: RCCL at world 1)."""
        self.force = bool(force)
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        backend = dist.get_backend(group)
        self.host = (backend != "nccl") if host_staged is None else host_staged
        self._glob = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
        self.next = self._glob((self.rank + 1) % self.world)
        self.prev = self._glob((self.rank - 1) % self.world)

    @property
    def active(self) -> bool:
        """Collectives move data (more than one rank, or forced at world 1)."""
        return self.world > 1 or self.force

    def exchange(self, send: torch.Tensor, recv: torch.Tensor) -> _Pending:
        """Start: send -> next rank, prev rank -> recv.  wait() completes both."""
        wire(self).add(send.numel() * send.element_size())
        if self.host:
            s, r = send.detach().cpu(), torch.empty(recv.shape, dtype=recv.dtype)
            ops = [dist.P2POp(dist.isend, s, self.next, self.group), dist.P2POp(dist.irecv, r, self.prev, self.group)]
            return _Pending(dist.batch_isend_irecv(ops), [(recv, r)])
        ops = [dist.P2POp(dist.isend, send, self.next, self.group),
               dist.P2POp(dist.irecv, recv, self.prev, self.group)]
        return _Pending(dist.batch_isend_irecv(ops))

    def gather_v(self, send: torch.Tensor, out: torch.Tensor, bounds) -> _Pending:
        """Start the all-peer gather: rank r's rows land in out[bounds[r]:bounds[r+1]] on every rank
        (send = this rank's rows; it may be that slice of ``out`` itself).  One send and one receive
        per peer, all in one batch."""
        b = [int(x) for x in bounds]
        return self.gather_at(send, out, b[:-1], [hi - lo for lo, hi in zip(b[:-1], b[1:])])

    def gather_at(self, send: torch.Tensor, out: torch.Tensor, starts, sizes) -> _Pending:
        """Start an all-peer gather of blocks placed anywhere: rank r's ``sizes[r]`` rows land in
        out[starts[r]:starts[r] + sizes[r]] on every rank (send = this rank's rows; it may be its own
        slice of ``out``).  The pipelined forward posts each finished row block of a layer with it."""
        k = self.rank
        lo, n_own = int(starts[k]), int(sizes[k])
        own = out[lo:lo + n_own]
        if n_own and send.data_ptr() != own.data_ptr():
            own.copy_(send)
        if not self.active or self.world == 1:
            return _Pending([])
        count_gather(self, out, n_own)
        peers = [r for r in range(self.world) if r != k]
        if self.host:
            s = own.detach().cpu() if n_own else None
            bufs = {r: torch.empty((int(sizes[r]), *out.shape[1:]), dtype=out.dtype) for r in peers}
            ops = []
            for r in peers:
                if n_own:
                    ops.append(dist.P2POp(dist.isend, s, self._glob(r), self.group))
                if bufs[r].shape[0]:
                    ops.append(dist.P2POp(dist.irecv, bufs[r], self._glob(r), self.group))
            works = dist.batch_isend_irecv(ops) if ops else []
            return _Pending(works, [(out[int(starts[r]):int(starts[r]) + int(sizes[r])], bufs[r]) for r in peers
                                    if bufs[r].shape[0]])
        ops = []
        for r in peers:
            if n_own:
                ops.append(dist.P2POp(dist.isend, own, self._glob(r), self.group))
            a, z = int(starts[r]), int(sizes[r])
            if z:
                ops.append(dist.P2POp(dist.irecv, out[a:a + z], self._glob(r), self.group))
        return _Pending(dist.batch_isend_irecv(ops) if ops else [])

    def all_to_all_v(self, send: torch.Tensor, send_off, recv: torch.Tensor, recv_off) -> None:
        """send[send_off[p]:send_off[p+1]] -> rank p; rank p's block -> recv[recv_off[p]:recv_off[p+1]]
        (1-D tensors, element offsets); completes before returning."""
        k = self.rank
        recv[int(recv_off[k]):int(recv_off[k + 1])].copy_(send[int(send_off[k]):int(send_off[k + 1])])
        if not self.active or self.world == 1:
            return
        peers = [r for r in range(self.world) if r != k]
        wire(self).add(send.element_size() * (int(send_off[-1]) - int(send_off[0]) - (int(send_off[k + 1]) -
                                                                                       int(send_off[k]))))
        src = send.detach().cpu() if self.host else send
        dst = torch.empty(recv.shape, dtype=recv.dtype) if self.host else recv
        ops = []
        for r in peers:
            a, b = int(send_off[r]), int(send_off[r + 1])
            if b > a:
                ops.append(dist.P2POp(dist.isend, src[a:b], self._glob(r), self.group))
            a, b = int(recv_off[r]), int(recv_off[r + 1])
            if b > a:
                ops.append(dist.P2POp(dist.irecv, dst[a:b], self._glob(r), self.group))
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        if self.host:
            for r in peers:
                a, b = int(recv_off[r]), int(recv_off[r + 1])
                if b > a:
                    recv[a:b].copy_(dst[a:b])

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if not self.active:
            return t
        count_all_reduce(self, t)
        if self.host:
            c = t.detach().cpu()
            dist.all_reduce(c, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, group=self.group)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape], rank order."""
        if not self.active:
            return t.unsqueeze(0)
        count_all_gather(self, t)
        if self.host:
            c = t.detach().cpu().contiguous()
            parts = [torch.empty_like(c) for _ in range(self.world)]
            dist.all_gather(parts, c, group=self.group)
            return torch.stack(parts).to(t.device)
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out


# ---------------------------------------------------------------- the plan
# shard_bounds' cost model of a rank's CF step, fitted in round 6 to four full-size C5 rank shares (bench.py
# --rank-share 8 --share-rank ...; profiles/r06_c5_rank_share_0_5.log, r06_c5_rank_share_w48.log):
#   t ~ c_r R + c_e E + c_i E_item,  c_r = 10.3 ms per M rows (the bi-interaction GEMMs + epilogues, the table
#   update, the gathered-buffer copies), c_e = 0.21 ms per M entries (user / entity rows: their gathers hit the
#   Zipf-popular item rows in the caches), c_i = 0.47 ms per M entries of item rows (hub rows whose entries
#   gather uniformly random 1 KB user rows: HBM-bound).  Measured: rank 0 of the mean-degree bounds (users,
#   200M entries / 2.5M rows) 68.1 ms, rank 5 (entities, 27.5M / 11.1M) 120.0 ms; with the row weight alone,
#   rank 4 (entities, 20.8M / 8.4M) 87.6 ms, rank 2 (items, 292M / 2.8M) 166.6 ms.
# SHARD_ROW_WEIGHT = c_r / c_e in entries (None: the graph's mean degree); HUB_EDGE_SCALE = c_i / c_e.
SHARD_ROW_WEIGHT: float | None = 48.0
HUB_EDGE_SCALE = 2.2


def shard_bounds(rowptr: np.ndarray, world: int, row_weight: float | None = None,
                 edge_scale: list | None = None) -> np.ndarray:
    """Contiguous row ranges balancing the cost model above: a row weighs its entries plus ``row_weight``
    entries (default SHARD_ROW_WEIGHT; None = the mean degree); ``edge_scale`` = [(lo, hi, factor)]: the
    entries of rows [lo, hi) weigh ``factor`` each (the C5 bench passes the item rows with HUB_EDGE_SCALE)."""
    n = rowptr.size - 1
    if row_weight is None:
        row_weight = SHARD_ROW_WEIGHT
    mean = rowptr[-1] / max(n, 1) if row_weight is None else float(row_weight)
    cum = rowptr.astype(np.float64) + mean * np.arange(n + 1)
    for lo, hi, factor in edge_scale or ():
        lo, hi = max(0, int(lo)), min(n, int(hi))
        if hi > lo:
            idx = np.clip(np.arange(n + 1), lo, hi)
            cum += (float(factor) - 1.0) * (rowptr[idx] - rowptr[lo]).astype(np.float64)
    targets = cum[-1] * np.arange(1, world) / world
    cuts = np.searchsorted(cum, targets)
    b = np.concatenate([[0], np.clip(cuts, 0, n), [n]]).astype(np.int64)
    return np.maximum.accumulate(b)


def _transpose_rows(rowptr: np.ndarray, col: np.ndarray, val: np.ndarray, lo: int, hi: int):
    """Rows [lo, hi) of the transpose of a whole CSR: (rowptr from 0, col int32, val fp32) with the
    columns of each row ascending (graph.DeviceGraph's CSR(A^T) order)."""
    n = rowptr.size - 1
    col = np.asarray(col)
    sel = np.flatnonzero((col >= lo) & (col < hi))
    rows = np.searchsorted(rowptr, sel, side="right") - 1          # source row of each kept entry
    order = np.lexsort((rows, col[sel]))
    tr = col[sel][order].astype(np.int64) - lo
    rp = np.zeros(hi - lo + 1, np.int64)
    np.cumsum(np.bincount(tr, minlength=hi - lo), out=rp[1:])
    del n
    return rp, rows[order].astype(np.int32), np.asarray(val, np.float32)[sel][order]


class _PeerIdGuard:
    """The hop backward's check of the row ids other ranks sent.  The all-peer gather of
    every rank's hop rows (``_hop_layer``) hands this rank ids no local code produced; they index its node
    map.  ``kgat_map_build_checked`` maps only ids inside [0, N), overwrites any other with -1 (so nothing
    downstream -- the masked A^T product, which looks rows up through the map, and the map reset -- reads
    or writes out of range) and raises a flag in pinned host memory and one on the device.  The flag is
    read before the optimiser step (``RowShardedKGAT.update_cf_weights``) and before a deferred table
    gradient is materialised: the step is abandoned -- no parameter or Adam moment moves, its gradients and
    deferred update are dropped -- and IndexError is raised, instead of a GPU fault.  Every rank receives
    the same gathered ids, so every rank abandons the same step."""

    def __init__(self, device):
        self.host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.dev = torch.zeros(1, dtype=torch.int32, device=device)
        self.event = torch.cuda.Event()
        self.pending = False

    def map_build(self, ids: torch.Tensor, total: int, node_map: torch.Tensor, n_nodes: int) -> None:
        _lib.call("kgat_map_build_checked", ids.data_ptr(), total, node_map.data_ptr(), n_nodes,
                  self.host.data_ptr(), self.dev.data_ptr(), stream_ptr(ids.device))
        self.event.record()
        self.pending = True

    def sanitize(self, ids: torch.Tensor, total: int, n_nodes: int) -> None:
        """Gathered ids outside [-1, N) become -1 (nothing indexes with them) and raise the flags."""
        _lib.call("kgat_ids_sanitize_i32", ids.data_ptr(), total, n_nodes, self.host.data_ptr(), self.dev.data_ptr(),
                  stream_ptr(ids.device))
        self.event.record()
        self.pending = True

    def take(self) -> bool:
        """True (and the flags cleared) if a gathered id since the last call was out of range."""
        if not self.pending:
            return False
        self.event.synchronize()
        self.pending = False
        if not int(self.host[0]):
            return False
        self.host.zero_()
        self.dev.zero_()
        return True


class RowShard:
    """Rank k's rows of A (``A``: local rows, global columns) and of A^T (``AT``).

    ``local=False``: rowptr / col / val are the whole CSR (every rank holds the graph; the
    transpose rows are cut from it).  ``local=True``: they are this rank's rows only (rowptr
    [hi-lo+1] from 0, global column ids) and ``transpose`` = (rowptr, col, val) of its rows of A^T
    (graph.HashedCKG.shard(lo, hi, transpose=True): the C4/C5 sizes, where no rank holds the
    whole graph)."""

    def __init__(self, rowptr: np.ndarray, col: np.ndarray, val: np.ndarray, bounds: np.ndarray, rank: int, device,
                 local: bool = False, transpose=None):
        self.bounds = np.asarray(bounds, np.int64)
        self.rank, self.world = rank, self.bounds.size - 1
        lo, hi = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.lo, self.hi, self.n = lo, hi, hi - lo
        self.n_nodes = int(self.bounds[-1])
        self.sizes = np.diff(self.bounds)
        self.device = torch.device(device)
        if local:
            if rowptr.size != self.n + 1:
                raise ValueError(f"local rowptr has {rowptr.size - 1} rows, shard {rank} has {self.n}")
            if transpose is None:
                raise ValueError("local rows need their rows of A^T too (transpose=)")
            lrp = np.asarray(rowptr, np.int64) - int(rowptr[0])
            e0, e1 = int(rowptr[0]), int(rowptr[-1])
            trp, tcol, tval = transpose
            trp = np.asarray(trp, np.int64) - int(trp[0])
        else:
            lrp = np.asarray(rowptr[lo:hi + 1], np.int64) - int(rowptr[lo])
            e0, e1 = int(rowptr[lo]), int(rowptr[hi])
            trp, tcol, tval = _transpose_rows(rowptr, col, val, lo, hi)
        lcol = np.ascontiguousarray(col[e0:e1], np.int32)
        lval = np.asarray(val[e0:e1], np.float32)
        self._lrp, self._lcol = lrp, lcol
        self._trp, self._tcol = trp, np.ascontiguousarray(tcol, np.int32)
        self.A = _DeviceCSR(lrp, lcol, torch.from_numpy(lval.copy()).to(self.device), self.device)
        self.AT = _DeviceCSR(trp, self._tcol, torch.from_numpy(np.asarray(tval, np.float32).copy()).to(self.device),
                             self.device, col_cuts=False)
        self.nnz = int(lcol.size)
        # the local CSR's row pointers / values under the names the attention refresh uses
        self.local_rowptr = self.A.rowptr
        self.local_val = self.A.val
        # node -> compact batch row of the last layer's masked backward (-1 between steps)
        self.node_map = torch.full((self.n_nodes,), -1, dtype=torch.int32, device=self.device)
        self._ident = None

    def peer_ids(self) -> _PeerIdGuard:
        """The check of the hop rows gathered from the peers (allocated once)."""
        g = self.__dict__.get("_peer_ids")
        if g is None:
            g = self._peer_ids = _PeerIdGuard(self.device)
        return g

    def hop_buffers(self, slot: int = 0):
        """Scratch of the hop backward (allocated once): local row flags, local row -> hop position,
        the hop rows (local ids), device count, kgat_hop_compact's scan work.  ``slot`` 1: a second set
        (the frontier forward's second hop, listed while the first hop's list is still in use)."""
        key = "_hop" if slot == 0 else f"_hop{slot}"
        hb = self.__dict__.get(key)
        if hb is None:
            n, dev = self.n, self.device
            work = int(_lib.lib().kgat_hop_compact_work_bytes(n))
            if work < 0:
                raise ValueError("shard too large for the hop compaction")
            hb = (torch.zeros(max(n, 1), dtype=torch.int32, device=dev),
                  torch.full((max(n, 1),), -1, dtype=torch.int32, device=dev),
                  torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                  torch.zeros(1, dtype=torch.int32, device=dev),
                  torch.empty(max(work, 1), dtype=torch.uint8, device=dev))
            self.__dict__[key] = hb
        return hb

    def ident(self, n: int) -> torch.Tensor:
        """int32 [0, n) on the device (row list of the pack copies)."""
        if self._ident is None or self._ident.numel() < n:
            self._ident = torch.arange(max(n, self.n, 1), dtype=torch.int32, device=self.device)
        return self._ident[:n]

    @property
    def local_keys(self) -> np.ndarray:
        """row * n_nodes + col of the local CSR entries (row-major sorted; attention refresh only)."""
        k = self.__dict__.get("_keys")
        if k is None:
            lrow = np.repeat(np.arange(self.n, dtype=np.int64), np.diff(self._lrp))
            k = self._keys = lrow * self.n_nodes + self._lcol.astype(np.int64)
        return k

    def value_plan(self):
        """The refresh's value exchange (built once): A_loc entries whose column lies in shard j, in
        (column, row) order, go to rank j, where they are exactly its AT rows' entries from shard k in
        CSR order.  Returns (send_pos int32 [nnz], send_off [G+1], recv_inv int32 [nnz], recv_off [G+1])
        with AT.val = recv[recv_inv]."""
        plan = self.__dict__.get("_vplan")
        if plan is not None:
            return plan
        lrow = np.repeat(np.arange(self.n, dtype=np.int64), np.diff(self._lrp))
        order = np.lexsort((lrow, self._lcol))                        # by column, then row
        sid = np.searchsorted(self.bounds, self._lcol[order], side="right") - 1
        send_off = np.zeros(self.world + 1, np.int64)
        np.cumsum(np.bincount(sid, minlength=self.world), out=send_off[1:])
        tsid = np.searchsorted(self.bounds, self._tcol, side="right") - 1
        recv_order = np.argsort(tsid, kind="stable")                   # grouped by source shard, CSR order
        recv_off = np.zeros(self.world + 1, np.int64)
        np.cumsum(np.bincount(tsid, minlength=self.world), out=recv_off[1:])
        recv_inv = np.empty(recv_order.size, np.int64)
        recv_inv[recv_order] = np.arange(recv_order.size)
        dev = self.device
        plan = (torch.from_numpy(order.astype(np.int32)).to(dev), send_off,
                torch.from_numpy(recv_inv.astype(np.int32)).to(dev), recv_off)
        self._vplan = plan
        return plan


# The frontier forward's layer inputs travel as row sets (_RowSet: only the rows the next product reads)
# when those rows are at most this fraction of the nodes; beyond it the whole-table gather moves about as
# many bytes without the ids and the placement pass.  KGAT_ROW_SET_GATHERS=0: whole-table gathers only.
COMPACT_FRACTION = 0.6
ROW_SET_GATHERS = os.environ.get("KGAT_ROW_SET_GATHERS", "1") != "0"
ROW_SET_STATS: dict = {}  # the last frontier forward's global set sizes (bench.py reports them)


class _RowSet:
    """The rows of a layer input that the next product reads, per rank -- the frontier forward's row-set
    gathers (model.py:124-140 reads layer L-1's input on N(F) only, layer L-2's on N(hop1)).
    Holds this rank's rows (local ids, ascending: the first ``m`` of ``rows``), every rank's count, the
    global ids of every rank's rows in rank order (one int32 all-peer gather, range-checked: _PeerIdGuard)
    and, for a pipelined producer, every rank's per-block counts.  Only these rows travel; the receiver
    places them at their global rows of the [N, d] buffer the single-GPU SpMM reads, so every row the
    product reads holds the bits the whole-table gather would have put there (the others are never read)."""

    def __init__(self, shard: RowShard, comm, rows: torch.Tensor, m: int, counts, block_counts=None):
        dev = shard.device
        self.m = int(m)
        self.counts = np.asarray(counts, np.int64).reshape(-1)
        self.off = np.concatenate([[0], np.cumsum(self.counts)]).astype(np.int64)
        self.total = int(self.off[-1])
        self.k = comm.rank if comm.active else 0
        self.rows = rows[:self.m] if self.m else torch.full((1,), -1, dtype=torch.int32, device=dev)
        ids = torch.empty(max(self.total, 1), dtype=torch.int32, device=dev)
        own = ids[int(self.off[self.k]):int(self.off[self.k + 1])]
        if self.m:
            kernels.map_compose(self.rows, None, shard.lo, out=own)
        comm.gather_v(own, ids, self.off).wait()
        if self.total:
            shard.peer_ids().sanitize(ids, self.total, shard.n_nodes)
        self.ids = ids
        self.block_counts = self.block_off = None
        if block_counts is not None:
            bc = np.asarray(block_counts, np.int64)  # [G, K]
            self.block_counts = bc
            self.block_off = np.concatenate([np.zeros((bc.shape[0], 1), np.int64), np.cumsum(bc, 1)], 1)

    def buffer(self, d: int, dev) -> torch.Tensor:
        """The compact receive buffer: every rank's rows, rank order (= ``ids`` order)."""
        return torch.empty(max(self.total, 1), d, dtype=torch.float32, device=dev)

    def post_block(self, comm, h: torch.Tensor, Pc: torch.Tensor, b: int):
        """Post block b's rows of the set (rows of h, a pipelined layer's output) to every peer, compact."""
        k, G = self.k, self.counts.size
        a, z = int(self.block_off[k][b]), int(self.block_off[k][b + 1])
        own = Pc[int(self.off[k]) + a:int(self.off[k]) + z]
        if z > a:
            kernels.gather_rows(h, self.rows[a:z], out=own)
        starts = [int(self.off[r] + self.block_off[r][b]) for r in range(G)]
        sizes = [int(self.block_counts[r][b]) for r in range(G)]
        return comm.gather_at(own, Pc, starts, sizes)

    def place(self, buf: torch.Tensor, Pc: torch.Tensor) -> None:
        """Every rank's compact rows into their global rows of ``buf``."""
        if self.total:
            kernels.scatter_rows(buf, self.ids[:self.total], Pc[:self.total], accumulate=False)

    def gather(self, shard: RowShard, comm, X: torch.Tensor) -> torch.Tensor:
        """[N, d]: every rank's rows of this set of X at their global rows (the rest never written)."""
        d = X.shape[1]
        Pc = self.buffer(d, X.device)
        own = Pc[int(self.off[self.k]):int(self.off[self.k + 1])]
        if self.m:
            kernels.gather_rows(X, self.rows, out=own)
        comm.gather_v(own, Pc, self.off).wait()
        buf = torch.empty(shard.n_nodes, d, dtype=torch.float32, device=X.device)
        self.place(buf, Pc)
        return buf


def _ids_bitmap(shard: RowShard, ids: torch.Tensor, total: int) -> torch.Tensor:
    """int32 bitmap over the N nodes with the bits of ``ids`` (global, distinct, checked) set: through
    the node map (kgat_map_build, kgat_map_bits, then the map reset)."""
    N = shard.n_nodes
    bits = torch.empty(2 * ((N + 63) // 64) + 2, dtype=torch.int32, device=shard.device)
    if total:
        _lib.call("kgat_map_build", ids.data_ptr(), total, shard.node_map.data_ptr(), stream_ptr(shard.device))
    kernels.map_bits(shard.node_map, bits)
    if total:
        kernels.frontier_reset(ids[:total], shard.node_map)
    return bits


def gathered_spmm(shard: RowShard, comm, csr, X: torch.Tensor, out: torch.Tensor, accumulate: bool = False,
                  transpose: bool = False, rows=None, pre=None, need: "_RowSet | None" = None) -> torch.Tensor:
    """out (+)= csr . Xg, Xg = [N, d] every rank's rows of X (all-peer gather), csr = shard.A (forward)
    or shard.AT (backward).  Column chunks of GATHER_CHUNK: chunk c+1 is on the wire while chunk c's
    product runs; each product is the single-GPU kernel on the local rows.  ``rows`` = (list, device
    count, bitmap) of local output rows: only those rows are produced (kgat_spmm_csr_rows_f32).
    ``need``: the rows of X the product reads, per rank (_RowSet) -- only those travel (compact), the rest
    of Xg is never read."""
    n, d = X.shape

    def product(src, dst):
        if rows is not None:
            return kernels.spmm_rows_block(csr, src, dst, *rows)
        return kernels.spmm_block(csr, src, dst, accumulate=accumulate, transpose=transpose)

    if not comm.active:  # one rank: X is the whole table
        return product(X, out)
    if pre is not None:  # gathered by the previous (pipelined) layer's block posts
        return product(_gathered(shard, comm, X, pre), out)
    if need is not None:  # only the rows the product reads travel
        return product(need.gather(shard, comm, X), out)
    w = min(d, GATHER_CHUNK) if GATHER_CHUNK > 0 else d
    chunks = [(c, min(c + w, d)) for c in range(0, d, w)]
    N, lo, hi = shard.n_nodes, shard.lo, shard.hi

    def start(c0, c1):
        buf = torch.empty(N, c1 - c0, dtype=torch.float32, device=X.device)
        own = buf[lo:hi]
        if hi > lo:
            kernels.gather_rows(X[:, c0:c1], shard.ident(n), out=own)  # pack this rank's columns
        return buf, comm.gather_v(own, buf, shard.bounds)

    nxt = start(*chunks[0])
    for i, (c0, c1) in enumerate(chunks):
        buf, pend = nxt
        if i + 1 < len(chunks):
            nxt = start(*chunks[i + 1])
        pend.wait()
        product(buf, out[:, c0:c1])
    return out


class _RowBlocks:
    """The pipelined forward's row blocks: every rank's shard cut into K blocks at 16-row boundaries (the
    bi-interaction's sub-tiles), from the shard sizes alone -- every rank knows every rank's blocks, so
    block b's all-peer post pairs up on every rank.  This rank's blocks carry a row view of A (its own
    long-row plan: a row never spans two blocks, so each row's edges are summed exactly as in the whole
    launch), the row list and the tile bitmap of the block."""

    def __init__(self, shard: RowShard, K: int):
        dev = shard.device
        self.K = K
        cuts = []
        for n in (int(z) for z in shard.sizes):
            c = [min(n, (n * b // K) // 16 * 16) for b in range(K)] + [n]
            cuts.append(list(np.maximum.accumulate(c)))
        self.cuts = cuts
        mine = cuts[shard.rank]
        self.mine = mine
        self.views, self.rows, self.bits = [], [], []
        for a, b in zip(mine[:-1], mine[1:]):
            self.views.append(_CSRRowView(shard.A, a, b, dev) if b > a else None)
            self.rows.append(torch.arange(a, b, dtype=torch.int32, device=dev) if b > a else None)
            w = np.zeros((shard.n + 31) // 32 + 1, np.uint32)
            for t in range(a // 16, (b + 15) // 16):  # the block's 16-row tiles: half-words of the bitmap
                w[t >> 1] |= np.uint32(0xFFFF) << np.uint32(16 * (t & 1))
            self.bits.append(torch.from_numpy(w.view(np.int32)).to(dev) if b > a else None)
        bounds = shard.bounds
        self.starts = [[int(bounds[r]) + cuts[r][b] for r in range(shard.world)] for b in range(K)]
        self.sizes = [[cuts[r][b + 1] - cuts[r][b] for r in range(shard.world)] for b in range(K)]


# Optional record of one step's pipelined forward (bench.py --timeline): when set to a list, the
# pipelined layers append (what, GPU event, host seconds) at each block's compute start / end, its post
# to the peers and each post's landing -- a rehearsal's evidence that block b travels while block b+1
# computes.
TIMELINE: list | None = None


def _mark(what: str) -> None:
    if TIMELINE is not None:
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        TIMELINE.append((what, e, time.perf_counter()))


def _gathered(shard: RowShard, comm, X: torch.Tensor, pre) -> torch.Tensor:
    """[N, d] every rank's rows of X: the blocks a pipelined layer already posted (``pre`` = (buffer,
    pending posts)), else one whole-width all-peer gather."""
    if pre is not None:
        buf, pends = pre[:2]
        for i, pd in enumerate(pends):
            pd.wait()
            _mark(f"width {buf.shape[1]}: block {i} post landed")
        if len(pre) == 4:  # compact block posts (a _RowSet): every rank's rows into place
            rs, Pc = pre[2], pre[3]
            rs.place(buf, Pc)
        return buf
    return gather_table(shard, comm, X)


def _layer_pipelined(shard: RowShard, comm, blocks: _RowBlocks, Xg: torch.Tensor, x: torch.Tensor, W1, b1, W2, b2,
                     drop: float, seed: int, st, s: torch.Tensor, need_next: "_RowSet | None" = None):
    """One whole-shard layer forward computed in row blocks, each block's output rows posted to every peer
    (the next layer's gathered input) as soon as they exist: the next layer's gather travels under this
    layer's remaining blocks instead of after the layer.  Per row: the SpMM of its edges in order (a row
    view of A), the bi-interaction with its own dropout draws and state (the tile-list / row-list kernels)
    -- the whole launch's bits.  Returns (this rank's output rows, (next gathered buffer, pending posts)).
    ``need_next`` (a _RowSet with per-block counts): only the block's rows the next layer reads are posted
    (compact; placed into the gathered buffer once every post has landed)."""
    dout = W1.shape[0]
    nxt = torch.empty(shard.n_nodes, dout, dtype=torch.float32, device=x.device)
    # the layer's output rows live in their own slot of the next layer's gathered buffer: no pack copy before
    # the posts (a row-heavy C5 rank copied ~11 GB per step), no separate [rows, d] allocation
    h = nxt[shard.lo:shard.hi]
    Pc = need_next.buffer(dout, x.device) if need_next is not None else None
    pends = []
    for b in range(blocks.K):
        a0, a1 = blocks.mine[b], blocks.mine[b + 1]
        _mark(f"width {dout}: block {b} compute start")
        if a1 > a0:
            kernels.spmm_block(blocks.views[b], Xg, s[a0:a1])
            if st.kind == "gemm":
                kernels.biinter_fwd_gemm_rows(x, s, blocks.rows[b], a1 - a0, W1, b1, W2, b2, drop, seed, h, st)
            else:
                kernels.biinter_fwd_tiles(x, s, W1, b1, W2, b2, drop, seed, h, blocks.bits[b], state=st)
        _mark(f"width {dout}: block {b} computed")
        if need_next is None:
            pends.append(comm.gather_at(h[a0:a1], nxt, blocks.starts[b], blocks.sizes[b]))
        else:
            pends.append(need_next.post_block(comm, h, Pc, b))
        _mark(f"width {dout}: block {b} posted")
    return h, ((nxt, pends) if need_next is None else (nxt, pends, need_next, Pc))


def gather_table(shard: RowShard, comm, X: torch.Tensor) -> torch.Tensor:
    """[N, d]: every rank's rows of X (the refresh's edge scorer reads whole rows)."""
    if not comm.active:
        return X
    buf = torch.empty(shard.n_nodes, X.shape[1], dtype=torch.float32, device=X.device)
    comm.gather_v(X.contiguous(), buf, shard.bounds).wait()
    return buf


# ---------------------------------------------------------------- batch rows
class _BatchRows:
    """The distinct rows a global batch touches: compact index <-> global id <-> local row."""

    def __init__(self, ids: np.ndarray, lo: int, hi: int, device):
        uniq, inv = np.unique(ids, return_inverse=True)
        self.n = uniq.size
        self.inv = inv.astype(np.int64)
        self.uniq_np = uniq
        self.uniq = torch.from_numpy(uniq.astype(np.int32)).to(device)   # compact -> global id
        owned = (uniq >= lo) & (uniq < hi)
        self.local_np = np.where(owned, uniq - lo, -1).astype(np.int32)
        self.local = torch.from_numpy(self.local_np).to(device)          # compact -> local row or -1
        self.frontier_np = self.local_np[owned]                           # owned local rows, compact order
        self.n_frontier = int(self.frontier_np.size)
        # never empty: a -1 row is padding every kernel reads as zero and writes nowhere
        fr = self.frontier_np if self.n_frontier else np.full(1, -1, np.int32)
        self.frontier = torch.from_numpy(fr.copy()).to(device)
        oc = np.flatnonzero(owned).astype(np.int32)
        self.owned_compact = torch.from_numpy(oc if oc.size else np.full(1, -1, np.int32)).to(device)
        pos = np.full(self.n, -1, np.int32)
        pos[owned] = np.arange(int(owned.sum()), dtype=np.int32)
        self.pos = torch.from_numpy(pos).to(device)                       # compact -> frontier position or -1

    def gather(self, tables: list[torch.Tensor], comm) -> list[torch.Tensor]:
        """Every rank gets the compact rows of every table (exact: one owner per row)."""
        widths = [t.shape[1] for t in tables]
        R = torch.empty(self.n, sum(widths), dtype=torch.float32, device=tables[0].device)
        off = 0
        for t, w in zip(tables, widths):
            kernels.gather_rows(t, self.local, out=R[:, off:off + w])
            off += w
        comm.all_reduce_(R)
        out, off = [], 0
        for w in widths:
            out.append(R[:, off:off + w])
            off += w
        return out


def _host_bits(ids: np.ndarray, n: int, device) -> torch.Tensor:
    """int32 device bitmap of n nodes with the bits of ``ids`` set (host-built: the ids are host data)."""
    b = np.zeros((n + 31) // 32 + 1, np.uint32)
    ids = np.asarray(ids, np.int64)
    ids = ids[ids >= 0]
    np.bitwise_or.at(b, ids >> 5, (np.uint32(1) << (ids & 31).astype(np.uint32)))
    return torch.from_numpy(b.view(np.int32)).to(device, non_blocking=True)


def _frontier_sets(shard: RowShard, comm, rows, L: int, blocks: _RowBlocks | None = None):
    """The row sets the CF loss reaches, per layer (this rank's part).  The last layer's output is read on
    the batch rows F only (model.py:189-191), so the last layer runs on F; it reads its input on N_A(F),
    inside the first hop h1 = F + N_A(F), so layer L-2 need only run on h1; that one reads its input on
    h2 = h1 + N_A(h1), and so on down the layers.  h_j is marked on the device by each owner from its rows
    of A^T and the global bitmap of h_(j-1) (row j is in it iff j is in h_(j-1) or A^T[j, h] != 0 for an h
    of it: kgat_csr_mark_rows); the counts are all-gathered (one host sync per hop) and layer L-1-j runs
    on h_j while the global h_j holds at most model.HOP_DENSE_FRACTION of the nodes -- the backward then
    runs that layer on the same set (its hop chain flags the same rows).  The chain stops at the first
    layer that runs whole (its input is then read on every row).  Returns (sets, needs):

    ``sets[l]``: None (layer l runs on the whole shard) or (rows int32 -- the first count valid --, count
    int32 [1] on the device, int32 bitmap, count).

    ``needs[l]``: None (layer l's input is gathered whole) or the _RowSet of input rows its product reads
    (VERDICT r5 #3): h_(L-l) -- every rank's rows of it travel, compact, when the global set holds at most
    COMPACT_FRACTION of the nodes (posted block by block when a pipelined whole layer produces them).  At
    full C5 (G = 8: 5.5k batch rows) h1 holds 0.25 % of the nodes and h2 14 % (every user is in it), so layer
    0 runs on h2 too and X0 travels on h3 (tools/c5_hop_fractions.py, profiles/r06_c5_hop_fractions.json)."""
    dev = shard.device
    N = shard.n_nodes
    sets = [None] * L
    needs = [None] * L
    m = rows.n_frontier
    sets[L - 1] = (rows.frontier, torch.tensor([m], dtype=torch.int32).to(dev, non_blocking=True),
                   _host_bits(rows.frontier_np, shard.n, dev), m)
    ROW_SET_STATS.update(nodes=int(N), hops=[], restricted=[L - 1], compact=[])
    if L < 2 or _model.HOP_DENSE_FRACTION <= 0:
        return sets, needs
    k = comm.rank if comm.active else 0
    prev_bits = _host_bits(rows.uniq_np, N, dev)  # the global bitmap of h0 = F (host data)
    for j in range(1, L + 1):
        l = L - 1 - j  # the layer that may run on h_j (-1: none -- h_L only sizes the gather of X0)
        hit, hmap, hrows, count, work = shard.hop_buffers(j - 1)
        kernels.csr_mark_rows(shard.AT, prev_bits, N, shard.lo, hit)
        kernels.hop_list(hit[:shard.n], hmap, hrows, count, work)
        # a whole layer l posts its output block by block when pipelined: every rank's per-block counts too
        piped = l >= 0 and blocks is not None and comm.active
        parts = [count.long()]
        if piped:
            parts += [hit[a:b].sum().reshape(1) for a, b in zip(blocks.mine[:-1], blocks.mine[1:])]
        g = comm.all_gather(torch.cat(parts)).reshape(-1, len(parts)).cpu().numpy().astype(np.int64)
        counts, total = g[:, 0], int(g[:, 0].sum())
        ROW_SET_STATS["hops"].append(total)
        restrict = l >= 0 and total <= _model.HOP_DENSE_FRACTION * N
        if restrict:
            bits = torch.empty(2 * ((shard.n + 63) // 64) + 2, dtype=torch.int32, device=dev)
            kernels.map_bits(hmap[:shard.n], bits)
            sets[l] = (hrows, count.clone(), bits, int(counts[k]))
            ROW_SET_STATS["restricted"].append(l)
        rs = None
        if comm.active and ROW_SET_GATHERS and total <= COMPACT_FRACTION * N:
            rs = needs[L - j] = _RowSet(shard, comm, hrows, int(counts[k]), counts,
                                        g[:, 1:] if piped and not restrict else None)
            ROW_SET_STATS["compact"].append(L - j)
        if not restrict or j == L:
            break
        # the global bitmap of h_j, the next hop's seed: from every rank's ids (gathered by the row set), or,
        # on one rank, from the local list itself
        if rs is not None:
            prev_bits = _ids_bitmap(shard, rs.ids, rs.total)
        elif not comm.active:
            prev_bits = _ids_bitmap(shard, kernels.map_compose(hrows[:max(int(counts[k]), 1)], None, shard.lo),
                                    int(counts[k]))
        else:  # (unreachable: a set small enough to run a layer on is small enough to travel compact)
            break
    return sets, needs


class _ShardTableUpdate:
    """The row-sharded CF step's table gradient left as its last product until ``update_cf_weights``
    (``RowShardedKGAT.fuse_table_update``; the single-GPU model._TableUpdate's idea): with the hop
    backward, layer 0's table gradient is the masked product AT_loc . dS (+ dXd) of the gathered compact
    [dS | dXd] hop rows; deferred, the update runs it fused with the shard's Adam step
    (kgat_spmm_csr_masked_adam_block_f32): each product row is the gradient of its table row and goes
    straight into that row's Adam -- no [rows, d] gradient written and read back.  Same bits as the
    product + Adam.  Anything that needs the gradient first (a forward, a KG update) materialises it."""

    def __init__(self):
        self.pending = None

    def defer(self, shard: RowShard, Pg: torch.Tensor, ids: torch.Tensor, total: int, din: int) -> None:
        self.pending = (shard, Pg, ids, total, din)  # shard.node_map keeps the gathered ids' map

    def _release(self, shard, ids, total) -> None:
        if total:
            kernels.frontier_reset(ids[:total], shard.node_map)

    @torch.no_grad()
    def materialize(self, param: torch.Tensor) -> None:
        if self.pending is None:
            return
        shard, Pg, ids, total, din = self.pending
        self.pending = None
        g = torch.empty(shard.n, din, dtype=torch.float32, device=Pg.device)
        kernels.spmm_block_masked(shard.AT, shard.node_map, Pg[:, :din], g, Yc_init=Pg[:, din:], row0=shard.lo)
        self._release(shard, ids, total)
        if param.grad is None:
            param.grad = g
        else:
            kernels.add_(param.grad, g)

    def launch(self, param: torch.Tensor):
        shard, Pg, ids, total, din = self.pending
        self.pending = None

        def run(m, v, step_size, bc2s, b1, b2, eps, skip=None):
            kernels.spmm_masked_adam_block(shard.AT, shard.node_map, Pg[:, :din], Pg[:, din:], shard.lo, param.data, m,
                                           v, step_size, b1, b2, bc2s, eps, skip)
            self._release(shard, ids, total)
        return run


def _hop_layer(shard: RowShard, comm, l: int, tables, sides, states, ws, drops, seeds, dX, rows, bpr, reduce_w,
               force: bool = False, defer: _ShardTableUpdate | None = None):
    """Layer l's backward on the global hop set flagged in shard.hop_buffers()'s row flags, if the set
    is small (every rank decides alike from the all-gathered local counts: one host sync) or ``force``
    (the frontier forward computed layer l on that set only).
    Returns (dX_{l}, True) -- dense local rows, the next hop's rows flagged -- or (dX, False): the
    set is large, the caller runs the layer densely (nothing was computed)."""
    hit, hmap, hrows, count, work = shard.hop_buffers()
    dev = dX.device
    kernels.hop_list(hit[:shard.n], hmap, hrows, count, work)
    counts = comm.all_gather(count).reshape(-1).cpu().numpy().astype(np.int64)
    total = int(counts.sum())
    if not force and total > _model.HOP_DENSE_FRACTION * shard.n_nodes:
        return dX, False
    Tc, cu, cp, cn, reg, coef, gout = bpr
    W1, b1, W2, b2 = ws[4 * l: 4 * l + 4]
    din = W1.shape[1]
    k = comm.rank if comm.active else 0
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    mine = int(counts[k])
    # every rank's compact [dS | dXd] hop rows, rank order (= ascending global ids); this rank's
    # bi-interaction backward writes its own block in place
    Pg = torch.empty(max(total, 1), 2 * din, dtype=torch.float32, device=dev)
    ids = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    own = Pg[int(off[k]):int(off[k + 1])]
    hr = hrows[:mine] if mine else torch.full((1,), -1, dtype=torch.int32, device=dev)
    dS_out = own[:, :din] if mine else torch.empty(1, din, dtype=torch.float32, device=dev)
    dXd_out = own[:, din:] if mine else torch.empty(1, din, dtype=torch.float32, device=dev)
    # dX is indexed by local row: the wide kinds read it (and X, S, H, the state) through the hop list.
    # The dXd / dS half first: the rows go to the peers while the weight-gradient GEMMs (which nothing
    # downstream waits for) run under the transfer
    _, _, wgrads = kernels.biinter_bwd(tables[l], sides[l], dX, W1, b1, W2, b2, drops[l], seeds[l], dXd=dXd_out,
                                       dS=dS_out, rows=hr, dh_full=True, split=True,
                                       **({} if states[l] is None else {"H": tables[l + 1], "state": states[l]}))
    if mine:
        # the BPR terms of layer l on the batch rows this rank owns (each is in the hop set)
        kernels.bpr_bwd(Tc, l, cu, cp, cn, reg, coef, gout, dXd_out, row_map=kernels.map_compose(rows.local, hmap))
        kernels.map_compose(hr, None, shard.lo, out=ids[int(off[k]):int(off[k + 1])])
    pend = [comm.gather_v(own, Pg, off), comm.gather_v(ids[int(off[k]):int(off[k + 1])], ids, off)] \
        if comm.active else []
    reduce_w(l, list(wgrads()))
    for p in pend:
        p.wait()
    if total:
        # the peers' blocks were never validated here: ids outside [0, N) are dropped, not indexed
        shard.peer_ids().map_build(ids, total, shard.node_map, shard.n_nodes)
    if l == 0 and defer is not None:
        defer.defer(shard, Pg, ids, total, din)  # the table's product runs fused with its Adam step
        return None, True
    out = torch.empty(shard.n, din, dtype=torch.float32, device=dev)
    kernels.spmm_block_masked(shard.AT, shard.node_map, Pg[:, :din], out, Yc_init=Pg[:, din:], row0=shard.lo,
                              row_hit=hit if l > 0 else None)
    if total:
        kernels.frontier_reset(ids[:total], shard.node_map)
    return out, True


class _ShardedCFLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cu, cp, cn, cfg, X0, *ws):
        shard, comm, drops, seeds, reg, rows, frontier, _tu, blocks = cfg
        L = len(drops)
        tables, sides, states = [X0], [], []
        # frontier forward: layers whose output the loss reads on a row set only run on that set (the
        # rest of their tables is never read: the next layer's A rows, the BPR rows and the backward
        # all stay inside it); per row the whole-shard call's bits
        wire(comm).phase = "forward"
        sets, needs = _frontier_sets(shard, comm, rows, L, blocks) if frontier else ([None] * L, [None] * L)
        x = X0
        pre = None  # the next layer's gathered input, posted block by block by a pipelined layer
        for l in range(L):
            W1, b1, W2, b2 = ws[4 * l: 4 * l + 4]
            s = torch.empty(shard.n, x.shape[1], dtype=torch.float32, device=x.device)
            st = kernels.make_state(x.shape[0], W1.shape[1], W1.shape[0], x.device)
            if sets[l] is None and blocks is not None and l + 1 < L and comm.active:
                x, pre = _layer_pipelined(shard, comm, blocks, _gathered(shard, comm, x, pre), x, W1, b1, W2, b2,
                                          drops[l], seeds[l], st, s, need_next=needs[l + 1])
            elif sets[l] is None:
                gathered_spmm(shard, comm, shard.A, x, s, pre=pre, need=needs[l])
                pre = None
                x = kernels.biinter_fwd(x, s, W1, b1, W2, b2, drops[l], seeds[l], state=st)
            else:
                rws, cnt, bits, m = sets[l]
                gathered_spmm(shard, comm, shard.A, x, s, rows=(rws, cnt, bits), pre=pre, need=needs[l])
                pre = None
                h = torch.empty(shard.n, W1.shape[0], dtype=torch.float32, device=x.device)
                if st.kind == "gemm":
                    x = kernels.biinter_fwd_gemm_rows(x, s, rws, m, W1, b1, W2, b2, drops[l], seeds[l], h, st)
                else:  # the set's 4-row quads (kgat_biinter_fwd_list_f32), as the single-GPU frontier forward
                    x = kernels.biinter_fwd_list(x, s, W1, b1, W2, b2, drops[l], seeds[l], h, rws, cnt, state=st)
            sides.append(s)
            states.append(st)
            tables.append(x)
        Tc = rows.gather(tables, comm)
        loss, coef = kernels.bpr_fwd(Tc, cu, cp, cn, reg)
        ctx.cfg, ctx.saved = cfg, (tables, sides, states, Tc, coef, ws)
        ctx.ids = (cu, cp, cn)
        ctx.forced = {l for l in range(L - 1) if sets[l] is not None}
        wire(comm).phase = "other"
        return loss.view(())

    @staticmethod
    def backward(ctx, gout):
        shard, comm, drops, seeds, reg, rows, _frontier, tu, _blocks = ctx.cfg
        wire(comm).phase = "backward"
        tables, sides, states, Tc, coef, ws = ctx.saved
        cu, cp, cn = ctx.ids
        gout = gout.reshape(1).to(torch.float32).contiguous()
        L = len(drops)
        dev = tables[0].device
        wgrads: list[torch.Tensor | None] = [None] * (4 * L)

        def saved(l):
            return {} if states[l] is None else {"H": tables[l + 1], "state": states[l]}

        def reduce_w(l, grads):
            flat = torch.cat([g.reshape(-1) for g in grads])
            comm.all_reduce_(flat)
            out, off = [], 0
            for g in grads:
                out.append(flat[off:off + g.numel()].view_as(g))
                off += g.numel()
            wgrads[4 * l: 4 * l + 4] = out

        # ---- last layer: the bi-interaction backward on the batch rows this rank owns
        l = L - 1
        din = tables[l].shape[1]
        dHc = kernels.zeros((rows.frontier.numel(), tables[L].shape[1]), dev)
        kernels.bpr_bwd(Tc, L, cu, cp, cn, reg, coef, gout, dHc, row_map=rows.pos)
        dXdc, dSc, *g = kernels.biinter_bwd(tables[l], sides[l], dHc, *ws[4 * l: 4 * l + 4], drops[l], seeds[l],
                                            rows=rows.frontier, **saved(l))
        reduce_w(l, g)
        # every rank's [dS | dXd] batch rows, compact (one exact all-reduce: one owner per row)
        P = kernels.zeros((rows.n, 2 * din), dev)
        if rows.n_frontier:
            kernels.scatter_rows(P[:, :din], rows.owned_compact, dSc[:rows.n_frontier], accumulate=False)
            kernels.scatter_rows(P[:, din:], rows.owned_compact, dXdc[:rows.n_frontier], accumulate=False)
        comm.all_reduce_(P)
        _lib.call("kgat_map_build", rows.uniq.data_ptr(), rows.n, shard.node_map.data_ptr(), stream_ptr(dev))
        dX = torch.empty(shard.n, din, dtype=torch.float32, device=dev)
        sparse = L > 1 and _model.HOP_DENSE_FRACTION > 0
        hit = shard.hop_buffers()[0] if sparse else None
        kernels.spmm_block_masked(shard.AT, shard.node_map, P[:, :din], dX, Yc_init=P[:, din:], row0=shard.lo,
                                  row_hit=hit)
        kernels.frontier_reset(rows.uniq, shard.node_map)
        kernels.bpr_bwd(Tc, l, cu, cp, cn, reg, coef, gout, dX, row_map=rows.local)
        # ---- lower layers: dX_l is zero outside the hop set the last product flagged (the batch rows
        # and their A^T neighbours, one hop more per layer).  While the global set holds at most
        # model.HOP_DENSE_FRACTION of the nodes the layer runs on it (as KGAT's backward does): the
        # bi-interaction backward on this rank's hop rows, one all-peer gather of every rank's compact
        # [dS | dXd] hop rows (not the whole dS table), and the A^T product masked to them.  Then densely.
        for l in range(L - 2, -1, -1):
            W1, b1, W2, b2 = ws[4 * l: 4 * l + 4]
            if sparse or l in ctx.forced:
                dX, sparse = _hop_layer(shard, comm, l, tables, sides, states, ws, drops, seeds, dX, rows,
                                        (Tc, cu, cp, cn, reg, coef, gout), reduce_w, force=l in ctx.forced,
                                        defer=tu)
                if sparse:
                    continue
            dXd, dS, *g = kernels.biinter_bwd(tables[l], sides[l], dX, W1, b1, W2, b2, drops[l], seeds[l], **saved(l))
            reduce_w(l, g)
            kernels.bpr_bwd(Tc, l, cu, cp, cn, reg, coef, gout, dXd, row_map=rows.local)
            gathered_spmm(shard, comm, shard.AT, dS, dXd, accumulate=True, transpose=True)
            dX = dXd
        ctx.saved = None
        wire(comm).phase = "other"
        return (None, None, None, None, dX, *wgrads)


class _ShardedKGLoss(torch.autograd.Function):
    """TransR over the global KG batch on compact rows; the table gradient lands in owned rows."""

    @staticmethod
    def forward(ctx, heads, rels, pos, neg, cfg, emb_shard, rel_emb, trans):
        comm, rows, reg = cfg
        Ec = rows.gather([emb_shard], comm)[0].contiguous()
        loss, work = kernels.transr_fwd(Ec, rel_emb, trans, heads, rels, pos, neg, reg)
        ctx.save_for_backward(heads, rels, pos, neg, work, Ec)
        ctx.rows, ctx.n_shard = rows, emb_shard.shape[0]
        ctx.shape = (rel_emb.shape[0], rel_emb.shape[1])
        return loss.view(())

    @staticmethod
    def backward(ctx, gout):
        heads, rels, pos, neg, work, Ec = ctx.saved_tensors
        n_rel, k = ctx.shape
        gout = gout.reshape(1).to(torch.float32).contiguous()
        d_c, d_rel, d_trans = kernels.transr_bwd(Ec, n_rel, k, heads, rels, pos, neg, work, gout)
        d_emb = kernels.zeros((ctx.n_shard, Ec.shape[1]), Ec.device)
        kernels.scatter_rows(d_emb, ctx.rows.local, d_c, accumulate=False)
        return None, None, None, None, None, d_emb, d_rel, d_trans


class RowShardedKGAT(nn.Module):
    """KGAT with the node tables row-sharded over the ranks of ``comm``.

    Same modes as KGAT (model.py:421-431) for TRAIN_CF, TRAIN_KG, UPDATE_ATTENTION and
    PREDICT; each rank passes ITS OWN batch and the loss is the mean over the global batch.
    """

    def __init__(self, args: KGATArgs, layout: GraphLayout | None, comm, device,
                 bounds: np.ndarray | None = None, shard: RowShard | None = None):
        """``layout``: the whole graph (every rank slices its rows); or ``shard``: this rank's
        rows already built (graph.HashedCKG at C5 size, where no rank holds the whole graph)."""
        super().__init__()
        device = torch.device(device)
        n = args.user_num + args.entity_num
        if device.type != "cuda":
            raise RuntimeError("RowShardedKGAT runs on the MI355X HIP path only")
        self.comm = comm
        if shard is not None:
            if shard.n_nodes != n or shard.world != comm.world or shard.rank != comm.rank:
                raise ValueError(f"shard ({shard.n_nodes} nodes, rank {shard.rank}/{shard.world}) does not match "
                                 f"the model ({n} nodes) / communicator ({comm.rank}/{comm.world})")
            self.bounds, self.shard = shard.bounds, shard
        else:
            if layout.n_nodes != n:
                raise ValueError(f"layout has {layout.n_nodes} nodes, model has {n}")
            self.bounds = shard_bounds(layout.rowptr, comm.world) if bounds is None else np.asarray(bounds, np.int64)
            self.shard = RowShard(layout.rowptr, layout.col, layout.val, self.bounds, comm.rank, device)
        self.lo, self.hi = self.shard.lo, self.shard.hi
        self._n_nodes = n
        self._user_num = args.user_num
        self._regularization_params = list(args.regularization_params)
        d = args.cf_embedding_dim
        # local rows of the reference's xavier-uniform table (same bound as the full [n, d] init)
        bound = math.sqrt(6.0 / (n + d))
        self._user_entity_embedding_shard = nn.Parameter(torch.empty(self.shard.n, d).uniform_(-bound, bound))
        self._relation_embedding = nn.Embedding(args.relation_num, args.kg_embedding_dim)
        self._trans_matrix = nn.Parameter(torch.Tensor(args.relation_num, d, args.kg_embedding_dim))
        nn.init.xavier_uniform_(self._relation_embedding.weight)
        nn.init.xavier_uniform_(self._trans_matrix)
        self._aggregator_layers = nn.ModuleList()
        dims = [d, *args.layer_size]
        for l in range(len(args.layer_size)):
            self._aggregator_layers.append(Aggregator(dims[l], dims[l + 1], args.message_dropout[l]))
        self._multi_head_attention = MultiHeadAttention(d, args.kg_embedding_dim)
        self._step = 0
        # TRAIN_CF's forward on the row sets the loss reads (see _frontier_sets); the driver's
        # training step turns it on, off = the whole-shard propagation of every layer
        self.frontier_forward = False
        # layer 0's table product fused with the shard's Adam step (_ShardTableUpdate); off = the
        # product in the backward, the table gradient in .grad
        self.fuse_table_update = False
        self._table_update = _ShardTableUpdate()
        # row blocks of the pipelined forward (each finished block's output posted to the peers while the
        # next block computes; same bits); 0 = whole-shard launches, the next layer gathered after them
        self.pipeline_blocks = 4
        self.to(device)

    def _blocks(self) -> _RowBlocks | None:
        K = int(self.pipeline_blocks)
        if K <= 1 or GATHER_CHUNK > 0:
            return None
        cached = self.__dict__.get("_row_blocks")
        if cached is None or cached.K != K:
            cached = self._row_blocks = _RowBlocks(self.shard, K)
        return cached

    # ------------------------------------------------------------------ state
    @torch.no_grad()
    def load_full_state(self, state_dict: dict) -> None:
        """Take this rank's rows of a full (single-GPU / reference) state_dict."""
        own = self.state_dict()
        for k, v in state_dict.items():
            if k == "_user_entity_embedding.weight":
                self._user_entity_embedding_shard.copy_(v[self.lo:self.hi])
            elif k in own and not v.is_sparse:
                own[k].copy_(v)

    def _cf_weights(self) -> list[torch.Tensor]:
        return [w for agg in self._aggregator_layers for w in agg.weights()]

    def _dropouts(self) -> tuple[list[float], list[int]]:
        drops = [agg.dropout if self.training else 0.0 for agg in self._aggregator_layers]
        self._step += 1
        # same on every rank (no RNG traffic), different per step, layer and shard
        seeds = [(self._step * 0x9E3779B1 + 7919 * (l + 1) + 104729 * self.comm.rank) & ((1 << 62) - 1) if p > 0
                 else 0 for l, p in enumerate(drops)]
        return drops, seeds

    def _global_ids(self, *ids: torch.Tensor) -> list[np.ndarray]:
        dev = self._user_entity_embedding_shard.device
        stacked = torch.stack([t.to(dev).long().reshape(-1) for t in ids])
        out = [a.reshape(-1) for a in self.comm.all_gather(stacked).transpose(0, 1).cpu().numpy()]
        return out

    def _check(self, what: str, ids: list[np.ndarray], n: int) -> None:
        """IndexError unless every id is in [0, n) (as the reference's embedding gathers)."""
        for a in ids:
            if a.size and (a.min() < 0 or a.max() >= n):
                raise IndexError(f"{what}: id out of range [0, {n}) (min {a.min()}, max {a.max()})")

    # ------------------------------------------------------------------ modes
    def propagate(self) -> list[torch.Tensor]:
        """This rank's rows of [X0, H1, ..., HL] (no autograd state)."""
        drops, seeds = self._dropouts()
        blocks = self._blocks()
        L = len(self._aggregator_layers)
        with torch.no_grad():
            x = self._user_entity_embedding_shard.detach()
            tables = [x]
            pre = None
            for l, agg in enumerate(self._aggregator_layers):
                ws = [w.detach() for w in agg.weights()]
                s = torch.empty(self.shard.n, x.shape[1], dtype=torch.float32, device=x.device)
                if blocks is not None and l + 1 < L and self.comm.active:
                    st = kernels.make_state(x.shape[0], ws[0].shape[1], ws[0].shape[0], x.device)
                    x, pre = _layer_pipelined(self.shard, self.comm, blocks, _gathered(self.shard, self.comm, x, pre),
                                              x, *ws, drops[l], seeds[l], st, s)
                else:
                    gathered_spmm(self.shard, self.comm, self.shard.A, x, s, pre=pre)
                    pre = None
                    x = kernels.biinter_fwd(x, s, *ws, drops[l], seeds[l])
                tables.append(x)
        return tables

    def _calc_cf_loss(self, users, pos, neg) -> torch.Tensor:
        dev = self._user_entity_embedding_shard.device
        u, p, q = self._global_ids(users, pos, neg)
        self._check("TRAIN_CF ids", [u, p, q], self._n_nodes)
        B = u.size
        rows = _BatchRows(np.concatenate([u, p, q]), self.lo, self.hi, dev)
        cu, cp, cn = (torch.from_numpy(rows.inv[i * B:(i + 1) * B]).to(dev) for i in range(3))
        drops, seeds = self._dropouts()
        tu = self._table_update if self.fuse_table_update and torch.is_grad_enabled() else None
        cfg = (self.shard, self.comm, drops, seeds, float(self._regularization_params[0]), rows,
               self.frontier_forward and torch.is_grad_enabled(), tu, self._blocks())
        return _ShardedCFLoss.apply(cu, cp, cn, cfg, self._user_entity_embedding_shard, *self._cf_weights())

    def _calc_kg_loss(self, heads, relations, pos_tails, neg_tails) -> torch.Tensor:
        dev = self._user_entity_embedding_shard.device
        h, r, p, q = self._global_ids(heads, relations, pos_tails, neg_tails)
        self._check("TRAIN_KG heads/tails", [h, p, q], self._n_nodes)
        self._check("TRAIN_KG relations", [r], self._relation_embedding.weight.shape[0])
        B = h.size
        rows = _BatchRows(np.concatenate([h, p, q]), self.lo, self.hi, dev)
        ch, cp, cn = (torch.from_numpy(rows.inv[i * B:(i + 1) * B]).to(dev) for i in range(3))
        cfg = (self.comm, rows, float(self._regularization_params[1]))
        return _ShardedKGLoss.apply(ch, torch.from_numpy(r).to(dev), cp, cn, cfg, self._user_entity_embedding_shard,
                                    self._relation_embedding.weight, self._trans_matrix)

    def _refresh_plan(self, h: np.ndarray, r: np.ndarray, t: np.ndarray):
        """One scoring plan over this rank's edges (tails: global rows of the gathered X0), logits
        landing by local edge id; slot sums onto the local CSR."""
        key = (h.size, h.tobytes()[:64], r.tobytes()[:64], t.tobytes()[:64], int(h.sum()), int(t.sum()))
        cached = getattr(self, "_att_plan", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        sh, n, dev = self.shard, self._n_nodes, self._user_entity_embedding_shard.device
        w = degree_weights(h, t, r, n)  # per-relation degrees over the whole graph (model.py:309-314)
        sel = (h >= sh.lo) & (h < sh.hi)
        hl, rl, tl, wl = h[sel] - sh.lo, r[sel], t[sel], w[sel]
        keys = hl * n + tl
        slot = np.searchsorted(sh.local_keys, keys)
        ok = slot < sh.local_keys.size
        ok[ok] &= sh.local_keys[slot[ok]] == keys[ok]
        covered = np.zeros(sh.local_keys.size, bool)
        covered[slot[ok]] = True
        if not ok.all() or not covered.all():
            raise NotImplementedError("row-sharded attention refresh needs the edge list of the sharded graph")
        eid = np.arange(hl.size, dtype=np.int64)
        plan = RefreshPlan.for_edges(tl, rl, wl, eid, dev) if hl.size else None
        so = np.argsort(slot, kind="stable")
        slot_order = torch.from_numpy(so.astype(np.int32)).to(dev)
        slot_ptr = torch.from_numpy(np.searchsorted(slot[so], np.arange(sh.local_keys.size + 1)).astype(np.int64)).to(dev)
        out = (plan, slot_ptr, slot_order, int(hl.size))
        self._att_plan = (key, out)
        return out

    @torch.no_grad()
    def _update_attention(self, heads, relations, tails, relation_indices) -> None:
        """UPDATE_ATTENTION (model.py:318-366) on this rank's rows: the X0 shards are gathered, the local
        edges scored and soft-maxed over the local rows (A_loc's values); an all-to-all hands every
        refreshed value to the owner of its A^T row (AT_loc's values)."""
        h, r, t = (torch.as_tensor(x).cpu().numpy().astype(np.int64) for x in (heads, relations, tails))
        plan, slot_ptr, slot_order, n_edges = self._refresh_plan(h, r, t)
        sh, dev = self.shard, self._user_entity_embedding_shard.device
        mha = self._multi_head_attention
        p = mha.dropout if self.training else 0.0
        self._step += 1
        seed = (self._step * 0x632BE5AB + 31 * self.comm.rank + 1) & ((1 << 62) - 1) if p > 0 else 0
        W = [x.detach().contiguous() for x in (self._trans_matrix, mha._value_weight.weight, mha._value_weight.bias,
                                                mha._output.weight, mha._output.bias, mha._layer_norm.weight,
                                                mha._layer_norm.bias)]
        logits = torch.empty(max(n_edges, 1), dtype=torch.float32, device=dev)
        Xg = gather_table(sh, self.comm, self._user_entity_embedding_shard.detach())
        if plan is not None:
            kernels.score_edges(plan, Xg, *W, logits, p, seed)
        del Xg
        nnz = sh.nnz
        slot_logits = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
        st = stream_ptr(dev)
        _lib.call("kgat_slot_sum_f32", slot_ptr.data_ptr(), slot_order.data_ptr(), nnz, logits.data_ptr(),
                  slot_logits.data_ptr(), st)
        A = sh.A
        kernels.row_softmax_csr(A, slot_logits, A.val)
        # A^T's rows live with the owners of A's columns: move the refreshed values there
        send_pos, send_off, recv_inv, recv_off = sh.value_plan()
        send = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
        if nnz:
            _lib.call("kgat_gather_f32", A.val.data_ptr(), send_pos.data_ptr(), nnz, send.data_ptr(), st)
        nt = int(recv_off[-1])
        recv = torch.empty(max(nt, 1), dtype=torch.float32, device=dev)
        self.comm.all_to_all_v(send, send_off, recv, recv_off)
        if nt:
            _lib.call("kgat_gather_f32", recv.data_ptr(), recv_inv.data_ptr(), nt, sh.AT.val.data_ptr(), st)

    @torch.no_grad()
    def _calc_score(self, user_ids, item_ids) -> torch.Tensor:
        """[len(users), len(items)] -- identical on every rank (item ids index the table raw)."""
        dev = self._user_entity_embedding_shard.device
        tables = self.propagate()
        u = torch.as_tensor(user_ids).long().reshape(-1).cpu().numpy()
        i = torch.as_tensor(item_ids).long().reshape(-1).cpu().numpy()
        self._check("PREDICT ids", [u, i], self._n_nodes)
        rows = _BatchRows(np.concatenate([u, i]), self.lo, self.hi, dev)
        Tc = rows.gather(tables, self.comm)
        cu = torch.from_numpy(rows.inv[:u.size]).to(dev)
        ci = torch.from_numpy(rows.inv[u.size:]).to(dev)
        return kernels.scores(Tc, cu, ci)

    def build_optimizer(self, cf_lr: float, kg_lr: float) -> None:
        self._cf_optimizer = FusedAdam(self.parameters(), lr=cf_lr)
        self._kg_optimizer = FusedAdam(self.parameters(), lr=kg_lr)

    def _raise_on_bad_peer_ids(self) -> None:
        """IndexError (the step abandoned: gradients and the deferred table update dropped, nothing
        stepped) if the last hop backward received an out-of-range row id from a peer (_PeerIdGuard)."""
        if self.shard.peer_ids().take():
            tu = self._table_update
            if tu.pending is not None:
                shard, _, ids, total, _ = tu.pending
                tu.pending = None
                tu._release(shard, ids, total)
            for p in self.parameters():
                p.grad = None
            raise IndexError("row-sharded CF backward: a peer's gathered hop row id is out of range "
                             f"[0, {self.shard.n_nodes}); the step was abandoned (no parameter moved)")

    def materialize_table_grad(self) -> None:
        """Write a deferred table gradient (fuse_table_update) into the shard's .grad."""
        if self._table_update.pending is not None:
            self._raise_on_bad_peer_ids()
        self._table_update.materialize(self._user_entity_embedding_shard)

    def update_cf_weights(self) -> None:
        self._raise_on_bad_peer_ids()
        tu, param = self._table_update, self._user_entity_embedding_shard
        fused = None
        if tu.pending is not None:
            if param.grad is not None:  # another term wrote .grad: the fused launch never reads it
                tu.materialize(param)
            else:
                fused = {id(param): tu.launch(param)}
        self._cf_optimizer.step(fused=fused)
        self._cf_optimizer.zero_grad()

    def update_kg_weights(self) -> None:
        self.materialize_table_grad()
        self._kg_optimizer.step()
        self._kg_optimizer.zero_grad()

    def forward(self, *args, mode: KGATMode):
        # a deferred table product refers to this step's gathered rows and A^T's values
        self.materialize_table_grad()
        if mode == KGATMode.TRAIN_CF:
            return self._calc_cf_loss(*args)
        if mode == KGATMode.TRAIN_KG:
            return self._calc_kg_loss(*args)
        if mode == KGATMode.PREDICT:
            return self._calc_score(*args)
        if mode == KGATMode.UPDATE_ATTENTION:
            self._update_attention(*args)
            return None
        raise ValueError(f"unknown mode {mode}")
