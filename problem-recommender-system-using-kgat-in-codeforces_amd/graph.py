"""Collaborative knowledge graph (CKG) layout: host construction + HBM residency.

Host side (numpy, vectorised) restates the reference's input-layout producer
(src/model/KGAT/preprocess.py:157-246, 268-326, 628-634):

* adjacency blocks in the reference order ``[0, R+1, 1, R+2, ...]`` -- the
  interaction block user -> U+problem, its inverse, then every KG relation and
  its inverse (preprocess.py:177-222);
* each block normalised to ``(D^-1/2 A)^T D^-1/2 = A^T D^-1`` -- entry (t, h)
  = count(h, t) / outdeg(h) (preprocess.py:224-246);
* the per-edge arrays sorted by head then tail (preprocess.py:268-326) and the
  summed attentive matrix (preprocess.py:628-634).

Device side (:class:`DeviceGraph`) keeps, resident in HBM:

* CSR of A (int64 rowptr, int32 col, fp32 val) + its long-row plan;
* CSR of A^T with ``perm_t`` (CSR(A^T) position -> CSR(A) position) so that
  refreshed values are re-permuted with one gather instead of a re-sort;
* the refresh edge list (head, tail, relation, CSR slot, static degree weight).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

LONG_THRESHOLD = 256   # rows with more edges are split across waves (see csrc/spmm.hip)
SEG_LEN = 512          # edges per long-row segment


@dataclass
class GraphLayout:
    """Host arrays of the attentive matrix and the refresh edge list."""

    n_nodes: int
    rel_order: list[int]          # adjacency_relations, reference order
    heads: np.ndarray             # int64 [E], sorted by (head, tail)
    rels: np.ndarray              # int64 [E]
    tails: np.ndarray             # int64 [E]
    edge_vals: np.ndarray         # fp32 [E] per-relation normalised value
    rowptr: np.ndarray            # int64 [N+1]  CSR of the coalesced sum
    col: np.ndarray               # int32 [nnz]
    val: np.ndarray               # fp32 [nnz]
    slot: np.ndarray              # int64 [E] CSR position of each edge

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])

    def coo(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        rows = np.repeat(np.arange(self.n_nodes, dtype=np.int64), np.diff(self.rowptr))
        return rows, self.col.astype(np.int64), self.val


def adjacency_blocks(user_num: int, interactions: np.ndarray, triplets: np.ndarray,
                     kg_relation_ids=(0, 1, 2, 3)):
    """(relation id, heads, tails) per adjacency block, preprocess.py:177-222."""
    R = len(kg_relation_ids)
    ui = np.asarray(interactions, dtype=np.int64).reshape(-1, 2)
    tr = np.asarray(triplets, dtype=np.int64).reshape(-1, 3)
    users, items = ui[:, 0], ui[:, 1] + user_num
    out = [(0, users, items), (R + 1, items, users)]
    for r in kg_relation_ids:
        sel = tr[:, 1] == r
        h, t = tr[sel, 0] + user_num, tr[sel, 2] + user_num
        out += [(r + 1, h, t), (r + 2 + R, t, h)]
    return out


def _normalised(n: int, h: np.ndarray, t: np.ndarray):
    """Unique (row=t, col=h) entries with value count(h,t)/outdeg(h) (fp64)."""
    if h.size == 0:
        e = np.zeros(0, np.int64)
        return e, e, np.zeros(0, np.float64)
    key = h * n + t
    uk, cnt = np.unique(key, return_counts=True)
    hh, tt = uk // n, uk % n
    outdeg = np.bincount(h, minlength=n).astype(np.float64)
    return tt, hh, cnt / outdeg[hh]


def layout_from_blocks(n_nodes: int, blocks) -> GraphLayout:
    rows, cols, rels, vals, order = [], [], [], [], []
    for bi, (rel, h, t) in enumerate(blocks):
        r, c, v = _normalised(n_nodes, np.asarray(h, np.int64), np.asarray(t, np.int64))
        rows.append(r)
        cols.append(c)
        vals.append(v)
        rels.append(np.full(r.size, rel, np.int64))
        order.append(np.full(r.size, bi, np.int64))
    rows, cols, rels = np.concatenate(rows), np.concatenate(cols), np.concatenate(rels)
    vals64, order = np.concatenate(vals), np.concatenate(order)
    perm = np.lexsort((order, cols, rows))      # head, then tail, then block order
    rows, cols, rels, vals64 = rows[perm], cols[perm], rels[perm], vals64[perm]
    # coalesce duplicates (same (row, col) in two relations): values summed in fp64
    key = rows * n_nodes + cols
    first = np.ones(key.size, bool)
    first[1:] = key[1:] != key[:-1]
    slot = np.cumsum(first) - 1
    csr_val = np.zeros(int(first.sum()), np.float64)
    np.add.at(csr_val, slot, vals64)
    csr_rows, csr_col = rows[first], cols[first]
    rowptr = np.zeros(n_nodes + 1, np.int64)
    np.cumsum(np.bincount(csr_rows, minlength=n_nodes), out=rowptr[1:])
    return GraphLayout(n_nodes=n_nodes, rel_order=[b[0] for b in blocks], heads=rows, rels=rels, tails=cols,
                       edge_vals=vals64.astype(np.float32), rowptr=rowptr, col=csr_col.astype(np.int32),
                       val=csr_val.astype(np.float32), slot=slot.astype(np.int64))


def build_layout(user_num: int, entity_num: int, interactions: np.ndarray, triplets: np.ndarray,
                 kg_relation_ids=(0, 1, 2, 3)) -> GraphLayout:
    """The reference preprocess graph (preprocess.py:617-634) from raw ids."""
    return layout_from_blocks(user_num + entity_num,
                              adjacency_blocks(user_num, interactions, triplets, kg_relation_ids))


def csr_from_coo(n: int, rows: np.ndarray, cols: np.ndarray, vals: np.ndarray):
    """Coalesced CSR (duplicates summed) of a COO matrix."""
    rows, cols = np.asarray(rows, np.int64), np.asarray(cols, np.int64)
    key = rows * n + cols
    uk, inv = np.unique(key, return_inverse=True)
    v = np.zeros(uk.size, np.float64)
    np.add.at(v, inv, np.asarray(vals, np.float64))
    r = uk // n
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=n), out=rowptr[1:])
    return rowptr, (uk % n).astype(np.int32), v.astype(np.float32)


def long_row_plan(rowptr: np.ndarray, long_threshold: int = LONG_THRESHOLD, seg_len: int = SEG_LEN):
    """numpy twin of kgat_csr_plan(): long rows and their edge segments."""
    deg = np.diff(rowptr)
    long_rows = np.nonzero(deg > long_threshold)[0]
    nseg = (deg[long_rows] + seg_len - 1) // seg_len
    off = np.zeros(long_rows.size + 1, np.int64)
    np.cumsum(nseg, out=off[1:])
    seg_row = np.repeat(long_rows, nseg)
    local = np.arange(seg_row.size, dtype=np.int64) - np.repeat(off[:-1], nseg)
    seg_beg = rowptr[seg_row] + local * seg_len
    return (long_rows.astype(np.int32), off.astype(np.int32), seg_row.astype(np.int32), seg_beg.astype(np.int64))


N_XCDS = 8  # blocks b, b + 8, ... share an XCD (round-robin dispatch)


def seg_launch_order(col: np.ndarray, seg_beg: np.ndarray) -> np.ndarray:
    """numpy twin of kgat_csr_seg_order(): the SpMM's launch slot -> segment map.

    Segments stable-sorted by first column, dealt so that the long-row blocks sharing an XCD take
    one contiguous run of that list (each XCD's L2 then serves one slice of the column range).
    Scheduling only: results are bit-identical for any order.
    """
    n_seg = int(seg_beg.size)
    by_col = np.argsort(np.asarray(col)[seg_beg], kind="stable").astype(np.int32)
    nb = (n_seg + 3) // 4
    cnt = np.array([(nb - x + N_XCDS - 1) // N_XCDS if nb > x else 0 for x in range(N_XCDS)], np.int64)
    start = np.concatenate([[0], np.cumsum(cnt)])
    b = np.arange(nb, dtype=np.int64)
    pos = ((start[b % N_XCDS] + b // N_XCDS)[:, None] * 4 + np.arange(4)).ravel()
    out = np.full(4 * nb, n_seg, np.int32)
    ok = pos < n_seg
    out[ok] = by_col[pos[ok]]
    return out


SEG_COL_BLOCK = 8192   # SpMM plan: hub-row segments also cut at multiples of this column (csrc kgat_csr_plan_cols)
SEG_MIN_PIECE = 32     # ... once they hold this many entries


def long_row_plan_cols(rowptr: np.ndarray, col: np.ndarray, long_threshold: int = LONG_THRESHOLD,
                       seg_len: int = SEG_LEN, col_block: int | None = None, min_piece: int = SEG_MIN_PIECE):
    """The SpMM's long-row plan with column-aware cuts (kgat_csr_plan_cols, host C): like
    :func:`long_row_plan`, but a segment also ends where its column crosses a multiple of
    ``col_block`` (default :data:`SEG_COL_BLOCK`) once it holds ``min_piece`` entries."""
    if col_block is None:
        col_block = SEG_COL_BLOCK
    rp = np.ascontiguousarray(rowptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    n = rp.size - 1
    lib = _lib.lib()
    nl, ns = ctypes.c_int32(), ctypes.c_int32()
    args = (rp.ctypes.data, cl.ctypes.data, n, long_threshold, seg_len, col_block, min_piece)
    _lib.check(lib.kgat_csr_plan_cols(*args, ctypes.byref(nl), ctypes.byref(ns), None, None, None, None),
               "kgat_csr_plan_cols")
    lr, off = np.zeros(nl.value, np.int32), np.zeros(nl.value + 1, np.int32)
    sr, sb = np.zeros(ns.value, np.int32), np.zeros(ns.value, np.int64)
    _lib.check(lib.kgat_csr_plan_cols(*args, ctypes.byref(nl), ctypes.byref(ns), lr.ctypes.data, off.ctypes.data,
                                      sr.ctypes.data, sb.ctypes.data), "kgat_csr_plan_cols")
    return lr, off, sr, sb


def _ptr(t) -> int:
    return t.data_ptr() if t is not None else 0


def _seg_order_device(col: np.ndarray, seg_beg: np.ndarray, device):
    if seg_beg.size == 0:
        return None
    return torch.from_numpy(seg_launch_order(col, seg_beg)).to(device)


def degree_weights(heads: np.ndarray, tails: np.ndarray, rels: np.ndarray, n: int) -> np.ndarray:
    """1 / (log1p(deg_h) + log1p(deg_t)), degrees counted within each relation (model.py:309-314)."""
    w = np.empty(heads.size, np.float32)
    for r in np.unique(rels):
        sel = np.nonzero(rels == r)[0]
        dh = np.bincount(heads[sel], minlength=n)[heads[sel]].astype(np.float32)
        dt = np.bincount(tails[sel], minlength=n)[tails[sel]].astype(np.float32)
        w[sel] = np.float32(1.0) / (np.log1p(dh) + np.log1p(dt))
    return w


class _PlanArrays:
    """The two long-row plans of a CSR (or a row view of one), resident on the device: the SpMM's
    column-cut plan with its launch order (:meth:`descriptor`), and the fixed-length plan the row
    softmax's hub-segment arithmetic assumes (:meth:`softmax_descriptor`)."""

    def __init__(self, rowptr: np.ndarray, col_host: np.ndarray, device, col_cuts: bool = True, n_cols: int = 0):
        # Both only pay when the source table spans more than one column block per XCD: C3's 16k-node
        # table (L2-resident) measured 1.69 -> 1.75-1.77 ms per step with the cuts
        # (profiles/r05_seg_order_ab.md), C2's 1M-node one 1.88 -> 1.86 ms.
        wide = n_cols >= N_XCDS * SEG_COL_BLOCK
        self.col_cuts = col_cuts = col_cuts and wide
        self.long_threshold = LONG_THRESHOLD  # 128 for the column-cut plan measured 5-15 us slower per step
        lr, off, sr, sb = long_row_plan_cols(rowptr, col_host) if col_cuts else long_row_plan(rowptr)
        self.long_rows = torch.from_numpy(lr).to(device)
        self.long_seg_off = torch.from_numpy(off).to(device)
        self.seg_row = torch.from_numpy(sr).to(device)
        self.seg_beg = torch.from_numpy(sb).to(device)
        self.n_long, self.n_seg = int(lr.size), int(sr.size)
        self.seg_order = _seg_order_device(col_host, sb, device) if wide else None
        flr, foff, fsr, fsb = long_row_plan(rowptr)
        self._fixed = [torch.from_numpy(a).to(device) for a in (flr, foff, fsr, fsb)]
        self._fixed_n = (int(flr.size), int(fsr.size))

    def _desc(self, rowptr_ptr: int, val) -> _lib.CSR:
        b = getattr(self, "base", self)
        return _lib.CSR(rowptr_ptr, b.col.data_ptr(), val.data_ptr(), self.n_rows, b.col.numel(),
                        self.long_rows.data_ptr(), self.long_seg_off.data_ptr(), self.seg_row.data_ptr(),
                        self.seg_beg.data_ptr(), self.n_long, self.n_seg, 0 if self.col_cuts else SEG_LEN,
                        self.long_threshold, _ptr(self.seg_order))

    def softmax_descriptor(self) -> _lib.CSR:
        """The descriptor with the fixed-length plan (kgat_row_softmax_plan_f32)."""
        d = self.descriptor()
        lr, off, sr, sb = self._fixed
        d.long_rows, d.long_seg_off, d.seg_row, d.seg_beg = (lr.data_ptr(), off.data_ptr(), sr.data_ptr(),
                                                            sb.data_ptr())
        d.n_long, d.n_seg = self._fixed_n
        d.seg_len, d.long_threshold = SEG_LEN, LONG_THRESHOLD
        d.seg_order = None
        return d


class _DeviceCSR(_PlanArrays):
    """A CSR resident on the device plus its ctypes descriptor."""

    def __init__(self, rowptr: np.ndarray, col: np.ndarray, val: torch.Tensor, device, col_cuts: bool = True):
        self.n_rows = rowptr.size - 1
        self.rowptr_host = np.ascontiguousarray(rowptr, np.int64)
        self.rowptr = torch.from_numpy(self.rowptr_host).to(device)
        self.col = torch.from_numpy(np.ascontiguousarray(col, np.int32)).to(device)
        self.val = val
        self.max_deg = int(np.diff(rowptr).max()) if self.n_rows else 0
        self.col_host = np.ascontiguousarray(col, np.int32)
        self.n_cols = int(self.col_host.max()) + 1 if self.col_host.size else 0
        _PlanArrays.__init__(self, self.rowptr_host, self.col_host, device, col_cuts, self.n_cols)

    def descriptor(self) -> _lib.CSR:
        return self._desc(self.rowptr.data_ptr(), self.val)


class _CSRRowView(_PlanArrays):
    """Rows [r0, r1) of a _DeviceCSR, sharing its device arrays (values stay live across
    refreshes): the descriptor points at rowptr + r0 -- row pointers are absolute
    offsets into col / val -- with a long-row plan of its own rows."""

    def __init__(self, base: _DeviceCSR, r0: int, r1: int, device):
        self.base, self.r0, self.n_rows = base, int(r0), int(r1) - int(r0)
        self.nnz = int(base.rowptr_host[r1] - base.rowptr_host[r0])
        _PlanArrays.__init__(self, base.rowptr_host[r0:r1 + 1], base.col_host, device, base.col_cuts, base.n_cols)

    def descriptor(self) -> _lib.CSR:
        return self._desc(self.base.rowptr.data_ptr() + 8 * self.r0, self.base.val)


class DeviceGraph:
    """HBM-resident attentive matrix A, its transpose and the refresh edge list."""

    def __init__(self, layout: GraphLayout, device: torch.device | str):
        device = torch.device(device)
        self.device = device
        self.layout = layout
        self.n_nodes = layout.n_nodes
        rowptr, col = layout.rowptr, layout.col
        self.A = _DeviceCSR(rowptr, col, torch.from_numpy(layout.val.copy()).to(device), device)
        # transpose: CSR(A^T) positions sorted by (col, row) -> CSR(A) positions
        rows = np.repeat(np.arange(self.n_nodes, dtype=np.int64), np.diff(rowptr))
        perm_t = np.lexsort((rows, col.astype(np.int64)))
        rowptr_t = np.zeros(self.n_nodes + 1, np.int64)
        np.cumsum(np.bincount(col, minlength=self.n_nodes), out=rowptr_t[1:])
        self.perm_t = torch.from_numpy(perm_t.astype(np.int32)).to(device)
        self.AT = _DeviceCSR(rowptr_t, rows[perm_t].astype(np.int32),
                             torch.empty(col.size, dtype=torch.float32, device=device), device, col_cuts=False)
        # refresh edge list (model.py:318-366)
        self.edge_heads = torch.from_numpy(layout.heads.astype(np.int32)).to(device)
        self.edge_tails = torch.from_numpy(layout.tails.astype(np.int32)).to(device)
        self.edge_rels = torch.from_numpy(layout.rels.astype(np.int32)).to(device)
        self.edge_slot = torch.from_numpy(layout.slot.astype(np.int32)).to(device)
        self.edge_weight = torch.from_numpy(
            degree_weights(layout.heads, layout.tails, layout.rels, self.n_nodes)).to(device)
        self.rel_order = list(layout.rel_order)
        # node -> frontier position map for the last layer's sparse backward; -1 between steps
        self.node_map = torch.from_numpy(np.full(self.n_nodes, -1, np.int32)).to(device)
        self.refresh_transpose()

    @property
    def nnz(self) -> int:
        return int(self.A.col.numel())

    def hop_buffers(self):
        """Scratch of the backward's hop chain (kernels.hop_compact): row flags, node -> hop
        position map, hop rows, device count, scan work, pinned count, membership bitmap of the
        hop set, bitmap of the batch frontier, kgat_frontier_hop scratch, rank words of the hop
        set (allocated once)."""
        hb = getattr(self, "_hop", None)
        if hb is None:
            n = self.n_nodes
            work = int(_lib.lib().kgat_hop_compact_work_bytes(n))
            if work < 0:
                raise ValueError("graph too large for the hop compaction")
            hb = (torch.zeros(n, dtype=torch.int32, device=self.device),
                  torch.full((n,), -1, dtype=torch.int32, device=self.device),
                  torch.empty(max(n, 1), dtype=torch.int32, device=self.device),
                  torch.zeros(1, dtype=torch.int32, device=self.device),
                  torch.empty(work, dtype=torch.uint8, device=self.device),
                  torch.zeros(1, dtype=torch.int32, pin_memory=True),
                  torch.zeros(2 * ((n + 63) // 64) + 2, dtype=torch.int32, device=self.device),
                  torch.zeros(2 * ((n + 63) // 64) + 2, dtype=torch.int32, device=self.device),
                  # the single-pass scan's state: zero before the first kgat_frontier_hop / kgat_rows_union,
                  # left reusable by every call
                  torch.zeros(max(int(_lib.lib().kgat_frontier_hop_work_bytes(n)), 8), dtype=torch.uint8,
                              device=self.device),
                  torch.zeros((n + 31) // 32 + 1, dtype=torch.int64, device=self.device))
            self._hop = hb
        return hb

    def row_blocks(self, k: int) -> list[_CSRRowView]:
        """k row-block views of A with (about) equal edge counts, boundaries on multiples of 16
        rows (the bi-interaction's sub-tiles), cached per k."""
        cache = self.__dict__.setdefault("_a_blocks", {})
        if k not in cache:
            rp = self.A.rowptr_host
            n = self.n_nodes
            cuts = [0]
            for b in range(1, k):
                r = int(np.searchsorted(rp, rp[-1] * b // k)) // 16 * 16
                cuts.append(min(max(r, cuts[-1]), n))
            cuts.append(n)
            cache[k] = [_CSRRowView(self.A, a, b, self.device) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
        return cache[k]

    def side_stream(self):
        """The second stream of the pipelined layer forward (kernels.propagate_layer)."""
        s = self.__dict__.get("_side")
        if s is None:
            s = self._side = torch.cuda.Stream(device=self.device)
        return s

    def transpose_row_blocks(self, bounds) -> list[_CSRRowView]:
        """Row-block views of A^T for ``bounds`` [(r0, r1), ...] (cached per bounds)."""
        key = tuple((int(a), int(b)) for a, b in bounds)
        cache = getattr(self, "_at_blocks", {})
        if key not in cache:
            cache[key] = [_CSRRowView(self.AT, a, b, self.device) for a, b in key]
            self._at_blocks = cache
        return cache[key]

    def refresh_transpose(self) -> None:
        """valT = val[perm_t] after A's values changed (one gather kernel)."""
        if self.nnz:
            _lib.call("kgat_gather_f32", self.A.val.data_ptr(), self.perm_t.data_ptr(), self.nnz,
                      self.AT.val.data_ptr(), stream_ptr(self.device))

    def refresh_plan(self, heads, rels, tails) -> "RefreshPlan | None":
        """Edge-scoring plan for UPDATE_ATTENTION's edge list (model.py:318-366).

        Cached across calls with identical edge arrays (compared on device).
        Returns None when the (head, tail) set is not exactly this CSR's
        structure -- the caller then rebuilds the graph from the edges.
        """
        h = torch.as_tensor(heads).to(self.device).long()
        r = torch.as_tensor(rels).to(self.device).long()
        t = torch.as_tensor(tails).to(self.device).long()
        cached = getattr(self, "_plan", None)
        if cached is not None and cached.matches(h, r, t):
            return cached
        plan = RefreshPlan.build(self, h, r, t)
        self._plan = plan
        return plan

    def to_sparse_coo(self) -> torch.Tensor:
        """The attentive matrix as the reference's coalesced sparse COO (model.py:83-92)."""
        rows, cols, _ = self.layout.coo()
        idx = torch.from_numpy(np.vstack([rows, cols]))
        return torch.sparse_coo_tensor(idx, self.A.val.detach().cpu(), (self.n_nodes, self.n_nodes)).coalesce()


class RefreshPlan:
    """Device arrays that drive the edge scorer: relation-sorted 16-edge tiles,
    per-edge tails and static degree weights, and the edge -> CSR slot map."""

    TILE = 16

    def __init__(self):
        self.key: tuple[torch.Tensor, torch.Tensor, torch.Tensor] | None = None

    def matches(self, h, r, t) -> bool:
        if self.key is None:
            return False
        kh, kr, kt = self.key
        return (kh.shape == h.shape and torch.equal(kh, h) and torch.equal(kr, r) and torch.equal(kt, t))

    def set_tiles(self, r: np.ndarray, t: np.ndarray, dev) -> None:
        """Relation-sorted 16-edge tiles over this plan's edges (relation-major, then tail, so
        neighbouring tiles share rows), plus the host copy of the relation runs."""
        E = r.size
        order = np.lexsort((t, r))
        rs = r[order]
        starts = np.flatnonzero(np.r_[True, rs[1:] != rs[:-1]]) if E else np.zeros(0, np.int64)
        ends = np.r_[starts[1:], E]
        cnt = (ends - starts + self.TILE - 1) // self.TILE
        first_tile = np.zeros(cnt.size + 1, np.int64)
        np.cumsum(cnt, out=first_tile[1:])
        local = np.arange(first_tile[-1], dtype=np.int64) - np.repeat(first_tile[:-1], cnt)
        tile_beg = np.r_[np.repeat(starts, cnt) + self.TILE * local, E]
        self.rel_perm = torch.from_numpy(order.astype(np.int32)).to(dev)
        self.tile_rel = torch.from_numpy(np.repeat(rs[starts], cnt).astype(np.int32)).to(dev)
        self.tile_beg = torch.from_numpy(tile_beg.astype(np.int32)).to(dev)
        self.n_tiles = int(first_tile[-1])
        # host copy of the relation runs of rel_perm (the wide-embedding GEMM scorer walks them)
        self.seg_rel = np.ascontiguousarray(rs[starts], dtype=np.int32)
        self.seg_beg = np.ascontiguousarray(np.r_[starts, E], dtype=np.int64)

    @classmethod
    def for_edges(cls, tails: np.ndarray, rels: np.ndarray, weight: np.ndarray, out_pos: np.ndarray,
                  dev) -> "RefreshPlan":
        """A scoring plan over an arbitrary edge list: logit of edge i lands in out[out_pos[i]]."""
        p = cls()
        p.n_edges = int(tails.size)
        p.tails = torch.from_numpy(np.ascontiguousarray(tails, np.int32)).to(dev)
        p.weight = torch.from_numpy(np.ascontiguousarray(weight, np.float32)).to(dev)
        p.set_tiles(np.asarray(rels, np.int64), np.asarray(tails, np.int64), dev)
        p.out_pos = torch.from_numpy(np.ascontiguousarray(out_pos, np.int32)).to(dev)
        p.slot_ptr = p.slot_order = None
        return p

    @classmethod
    def build(cls, g: "DeviceGraph", h_d, r_d, t_d) -> "RefreshPlan | None":
        n = g.n_nodes
        h, r, t = h_d.cpu().numpy(), r_d.cpu().numpy(), t_d.cpu().numpy()
        E = h.size
        rowptr = g.layout.rowptr
        nnz = g.nnz
        csr_keys = np.repeat(np.arange(n, dtype=np.int64), np.diff(rowptr)) * n + g.layout.col.astype(np.int64)
        keys = h * n + t
        slot = np.searchsorted(csr_keys, keys)
        ok = slot < nnz
        ok[ok] &= csr_keys[slot[ok]] == keys[ok]
        if not ok.all():
            return None
        covered = np.zeros(nnz, bool)
        covered[slot] = True
        if not covered.all():
            return None
        p = cls()
        dev = g.device
        p.n_edges = E
        p.tails = torch.from_numpy(t.astype(np.int32)).to(dev)
        p.weight = torch.from_numpy(degree_weights(h, t, r, n)).to(dev)
        p.set_tiles(r, t, dev)
        if E == nnz:  # bijective: scores land directly in slot order
            p.out_pos = torch.from_numpy(slot.astype(np.int32)).to(dev)
            p.slot_ptr = p.slot_order = None
        else:         # duplicate (head, tail) pairs: summed per slot after scoring
            p.out_pos = None
            so = np.argsort(slot, kind="stable")
            p.slot_order = torch.from_numpy(so.astype(np.int32)).to(dev)
            p.slot_ptr = torch.from_numpy(np.searchsorted(slot[so], np.arange(nnz + 1)).astype(np.int64)).to(dev)
        p.key = (h_d.clone(), r_d.clone(), t_d.clone())
        return p


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device: torch.device) -> ctypes.c_void_p:
    """The current torch stream of ``device`` as a hipStream_t (the raw-handle query: ~1 us, where
    torch.cuda.current_stream(device) builds a Stream object through the device-index resolution,
    ~7 us -- 14 of them per CF step)."""
    if _raw_stream is not None and isinstance(device, torch.device) and device.type == "cuda":
        idx = device.index if device.index is not None else torch.cuda.current_device()
        return ctypes.c_void_p(_raw_stream(idx))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


# --------------------------------------------------------------------------
# Seeded synthetic CKG: the GPU configs C2/C4/C5
# --------------------------------------------------------------------------
def synthetic_ckg(n_nodes: int, n_triples: int, seed: int = 2024, user_frac: float = 0.1,
                  interaction_frac: float = 0.8, zipf_s: float = 1.1):
    """(user_num, entity_num, interactions [M,2], triplets [T,3]).

    First 10 % of nodes are users, the rest entities; items (problems) are the
    first 10 % of entities.  80 % of triples are user -> item interactions with
    Zipf(1.1) item popularity (item identity shuffled), 20 % are KG triples over
    the 4 reference relation types with uniform heads/tails inside type ranges.
    Duplicates are dropped (first occurrence in draw order wins).
    """
    rng = np.random.default_rng(seed)
    U = max(1, int(n_nodes * user_frac))
    E = n_nodes - U
    I = max(1, int(E * 0.1))
    m_target = int(n_triples * interaction_frac)
    k_target = n_triples - m_target
    ranks = np.arange(1, I + 1, dtype=np.float64)
    cdf = np.cumsum(ranks ** (-zipf_s))
    cdf /= cdf[-1]
    item_perm = rng.permutation(I)

    def draw_interactions(count):
        u = rng.integers(0, U, size=count, dtype=np.int64)
        it = item_perm[np.minimum(np.searchsorted(cdf, rng.random(count)), I - 1)]
        return u, it

    inter = np.zeros((0, 2), np.int64)
    need = m_target
    while need > 0:
        u, it = draw_interactions(int(need * 1.3) + 1024)
        cand = np.concatenate([inter, np.stack([u, it], 1)])
        key = cand[:, 0] * I + cand[:, 1]
        _, first = np.unique(key, return_index=True)
        inter = cand[np.sort(first)][:m_target]
        if inter.shape[0] >= m_target or inter.shape[0] >= U * I:
            break
        need = m_target - inter.shape[0]
    # KG: 4 relation types, tails from 4 disjoint ranges of the non-item entities
    rest = max(4, E - I)
    bounds = [I + (rest * k) // 4 for k in range(5)]
    rel = rng.integers(0, 4, size=k_target, dtype=np.int64)
    heads = rng.integers(0, I, size=k_target, dtype=np.int64)
    # HAS_CONTEST_DIVISION (3): contest (range of IN_CONTEST tails, 2) -> division range (3)
    c_lo, c_hi = bounds[2], bounds[3]
    sel3 = rel == 3
    heads[sel3] = rng.integers(c_lo, c_hi, size=int(sel3.sum()), dtype=np.int64)
    lo = np.array(bounds[:4])[rel]
    hi = np.array(bounds[1:])[rel]
    tails = lo + (rng.random(k_target) * (hi - lo)).astype(np.int64)
    trip = np.stack([heads, rel, np.minimum(tails, E - 1)], 1)
    key = (trip[:, 0] * 4 + trip[:, 1]) * E + trip[:, 2]
    _, first = np.unique(key, return_index=True)
    trip = trip[np.sort(first)]
    return U, E, inter, trip


class HashedCKG:
    """The seeded synthetic CKG of csrc/synth.cpp (C4/C5 sizes): every triple is a pure function
    of (seed, index), so each rank builds only its own rows of the attentive matrix.

    Same node layout and distributions as :func:`synthetic_ckg` (users first, items = first 10 %
    of entities, 80 % Zipf interactions, 20 % KG triples over 4 relations); repeated triples are
    dropped and redrawn, so the graph holds exactly ``n_triples`` distinct triples
    and E ~= 2 * n_triples attentive-matrix entries.  ``draws`` = the draws that took.
    """

    def __init__(self, n_nodes: int, n_triples: int, seed: int = 2024, zipf_s: float = 1.1, threads: int = 0):
        import os

        threads = threads or min(16, os.cpu_count() or 1)
        h = ctypes.c_void_p()
        _lib.call("kgat_synth_open", int(n_nodes), int(n_triples), int(seed) & ((1 << 64) - 1), float(zipf_s),
                  int(threads), ctypes.byref(h))
        self._h = h
        info = np.zeros(8, np.int64)
        _lib.call("kgat_synth_info", self._h, info.ctypes.data)
        self.n_nodes, self.n_triples, self.user_num, self.entity_num, self.item_num, self.n_interactions, \
            self.n_kg, self.draws = (int(x) for x in info[:8])

    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h is not None and h.value and _lib is not None:
            try:
                _lib.lib().kgat_synth_close(h)
            except (TypeError, AttributeError):  # interpreter shutdown: the module's globals are gone
                pass

    __del__ = close

    def row_offsets(self) -> np.ndarray:
        """[N+1] prefix sums of each row's pre-coalesce entry count (shard balance weights)."""
        off = np.empty(self.n_nodes + 1, np.int64)
        _lib.call("kgat_synth_row_offsets", self._h, off.ctypes.data)
        return off

    def triples(self, idx: np.ndarray):
        """Raw triples by index: (a, rel, b) -- rel -1: interaction (user a, item b), else (head, rel, tail)."""
        idx = np.ascontiguousarray(idx, np.int64)
        a, b = np.empty(idx.size, np.int64), np.empty(idx.size, np.int64)
        r = np.empty(idx.size, np.int32)
        _lib.call("kgat_synth_triples", self._h, idx.ctypes.data, idx.size, a.ctypes.data, r.ctypes.data,
                  b.ctypes.data)
        return a, r, b

    def raw(self):
        """(user_num, entity_num, interactions [M,2], triplets [T,3]) of the whole graph (small sizes only)."""
        a, r, b = self.triples(np.arange(self.n_triples, dtype=np.int64))
        m = r < 0
        inter = np.stack([a[m], b[m]], 1)
        trip = np.stack([a[~m], r[~m].astype(np.int64), b[~m]], 1)
        return self.user_num, self.entity_num, inter, trip

    def shard(self, lo: int, hi: int, transpose: bool = False):
        """Coalesced CSR of rows [lo, hi): (rowptr [hi-lo+1] from 0, col int32 global ids, val fp32); with
        ``transpose`` the rows of A^T (sharded.RowShard's AT_loc)."""
        nnz = ctypes.c_int64()
        _lib.call("kgat_synth_shard_build_ex", self._h, int(lo), int(hi), int(bool(transpose)), ctypes.byref(nnz))
        rowptr = np.empty(int(hi) - int(lo) + 1, np.int64)
        col = np.empty(nnz.value, np.int32)
        val = np.empty(nnz.value, np.float32)
        _lib.call("kgat_synth_shard_copy", self._h, rowptr.ctypes.data, col.ctypes.data, val.ctypes.data)
        return rowptr, col, val

    def sample_interactions(self, rng: np.random.Generator, count: int):
        """(users, items) of `count` uniformly drawn interaction triples (the bench's positives)."""
        idx = rng.integers(0, max(self.n_interactions, 1), count)
        a, _, b = self.triples(idx)
        return a, b
