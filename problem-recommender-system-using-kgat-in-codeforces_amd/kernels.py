"""Typed wrappers over the C-ABI: shape/dtype/device checks, then one HIP call.

Every wrapper launches on the current torch stream of the tensors' device and
returns without synchronising.  Tensors must be fp32 (ids int64), on the GPU,
with unit stride in the last dimension; violations raise ``ValueError`` before
anything is launched, HIP/launch errors raise ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from .graph import DeviceGraph, stream_ptr


def _req(t: torch.Tensor, name: str, dtype=torch.float32, dim: int | None = None) -> None:
    if not isinstance(t, torch.Tensor):
        raise ValueError(f"{name}: expected a tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name}: must live on the GPU (the HIP path has no CPU fallback)")
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    if dim is not None and t.dim() != dim:
        raise ValueError(f"{name}: expected {dim}-D, got {tuple(t.shape)}")
    if t.dim() >= 1 and t.numel() and t.shape[-1] > 1 and t.stride(-1) != 1:  # a size-1 dim may keep any stride
        raise ValueError(f"{name}: last dimension must be contiguous")


def _ld(t: torch.Tensor) -> int:
    return t.stride(0) if t.dim() == 2 else t.shape[-1]


# Optional launch timer for the dominant kernel (bench.py): when set to a list,
# every spmm() appends (start_event, end_event, d, transpose, accumulate) recorded
# on the launch stream around its kernels.
SPMM_EVENTS: list | None = None

# Optional per-kernel launch timer (bench.py's KG-step and refresh legs): when set to a dict,
# the wrappers below that take part append (start_event, end_event) recorded on the launch stream
# around their launches under their kernel's name.
KERNEL_EVENTS: dict | None = None


def _ev_begin(name: str):
    if KERNEL_EVENTS is None:
        return None
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    return name, e0


def _ev_end(tok) -> None:
    if tok is None or KERNEL_EVENTS is None:
        return
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record()
    KERNEL_EVENTS.setdefault(tok[0], []).append((tok[1], e1))


# Edges per chunk of the wide-embedding GEMM edge scorer (scratch = 2 * chunk * d floats).
EDGE_GEMM_CHUNK = 1 << 20


def spmm(graph: DeviceGraph, X: torch.Tensor, out: torch.Tensor | None = None, transpose: bool = False,
         accumulate: bool = False) -> torch.Tensor:
    """Y = A . X (or A^T . X); with accumulate, Y += ..."""
    _req(X, "X", dim=2)
    n, d = X.shape
    if n != graph.n_nodes:
        raise ValueError(f"X has {n} rows, graph has {graph.n_nodes} nodes")
    if out is None:
        if accumulate:
            raise ValueError("accumulate needs an output tensor")
        out = torch.empty(n, d, dtype=torch.float32, device=X.device)
    _req(out, "out", dim=2)
    if tuple(out.shape) != (n, d):
        raise ValueError("out shape mismatch")
    csr = graph.AT if transpose else graph.A
    desc = csr.descriptor()
    ws = torch.empty(max(1, csr.n_seg * d), dtype=torch.float32, device=X.device)
    ev = SPMM_EVENTS
    if ev is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.call("kgat_spmm_csr_f32", ctypes.byref(desc), X.data_ptr(), _ld(X), out.data_ptr(), _ld(out), d,
              int(accumulate), ws.data_ptr(), ws.numel(), stream_ptr(X.device))
    if ev is not None:
        e1.record()
        ev.append((e0, e1, d, transpose, accumulate))
    return out


def spmm_block(csr, X: torch.Tensor, out: torch.Tensor, accumulate: bool = False,
               transpose: bool = False) -> torch.Tensor:
    """Y (+)= B . X for a rectangular device CSR block B [out rows x X rows] (graph._DeviceCSR).
    ``transpose`` only labels the launch for SPMM_EVENTS (B is a transposed block)."""
    _req(X, "X", dim=2)
    _req(out, "out", dim=2)
    d = X.shape[1]
    if out.shape[0] != csr.n_rows or out.shape[1] != d:
        raise ValueError("out shape mismatch")
    if csr.n_rows == 0:
        return out
    desc = csr.descriptor()
    ws = torch.empty(max(1, csr.n_seg * d), dtype=torch.float32, device=X.device)
    ev = SPMM_EVENTS
    if ev is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.call("kgat_spmm_csr_f32", ctypes.byref(desc), X.data_ptr(), _ld(X), out.data_ptr(), _ld(out), d,
              int(accumulate), ws.data_ptr(), ws.numel(), stream_ptr(X.device))
    if ev is not None:
        e1.record()
        nnz = csr.nnz if hasattr(csr, "nnz") else csr.col.numel()  # a row view (_CSRRowView) or a whole CSR
        ev.append((e0, e1, d, transpose, ("block", int(csr.n_rows), int(nnz), bool(accumulate))))
    return out


def spmm_block_masked(csr, src_map: torch.Tensor, Xc: torch.Tensor, out: torch.Tensor,
                      Yc_init: torch.Tensor | None = None, row0: int = 0,
                      src_bits: torch.Tensor | None = None, src_rank: torch.Tensor | None = None,
                      row_hit: torch.Tensor | None = None) -> torch.Tensor:
    """Y = B . X for a rectangular block where X[c] = Xc[src_map[c]] (-1 => zero row); with Yc_init,
    local row r also gets Yc_init[src_map[row0 + r]] (B = rows [row0, ...) of a square matrix).
    ``row_hit`` (int32 [rows of B]): zeroed, then set for every row that gathered an edge or has a
    Yc row -- the next hop set of the backward chain (kgat_hop_compact lists it)."""
    _req(src_map, "src_map", dtype=torch.int32, dim=1)
    _req(Xc, "Xc", dim=2)
    _req(out, "out", dim=2)
    d = Xc.shape[1]
    if out.shape[0] != csr.n_rows or out.shape[1] != d:
        raise ValueError("out shape mismatch")
    if Yc_init is not None:
        _req(Yc_init, "Yc_init", dim=2)
        if Yc_init.shape[1] != d or row0 < 0 or row0 + csr.n_rows > src_map.numel():
            raise ValueError("Yc_init width / row0 mismatch")
    if csr.n_rows == 0:
        return out
    desc = csr.descriptor()
    ws = torch.empty(max(1, csr.n_seg * d), dtype=torch.float32, device=Xc.device)
    if row_hit is not None:
        _req(row_hit, "row_hit", dtype=torch.int32, dim=1)
        if row_hit.numel() < csr.n_rows:
            raise ValueError("row_hit shorter than the block")
    _lib.call("kgat_spmm_csr_masked_ex_f32", ctypes.byref(desc), src_map.data_ptr(), Xc.data_ptr(), _ld(Xc),
              Yc_init.data_ptr() if Yc_init is not None else None, _ld(Yc_init) if Yc_init is not None else 0,
              int(row0), out.data_ptr(), _ld(out), d, row_hit.data_ptr() if row_hit is not None else None,
              _bits_ptr(src_bits, src_map), _rank_ptr(src_rank, src_map),
              src_map.numel(), ws.data_ptr(), ws.numel(), stream_ptr(Xc.device))
    return out


def map_compose(a: torch.Tensor, b: torch.Tensor | None = None, offset: int = 0,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """out[i] = a[i] < 0 ? -1 : (b[a[i]] if b is given else a[i]) + offset (-1 stays -1), int32."""
    _req(a, "a", dtype=torch.int32, dim=1)
    if b is not None:
        _req(b, "b", dtype=torch.int32, dim=1)
    out = torch.empty_like(a) if out is None else out
    _req(out, "out", dtype=torch.int32, dim=1)
    if out.numel() != a.numel():
        raise ValueError("map_compose: out size")
    _lib.call("kgat_map_compose", a.data_ptr(), a.numel(), b.data_ptr() if b is not None else None, int(offset),
              out.data_ptr(), stream_ptr(a.device))
    return out


def gather_rows(src: torch.Tensor, rows: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[i] = src[rows[i]] (rows int32, -1 => zeros)."""
    _req(src, "src", dim=2)
    _req(rows, "rows", dtype=torch.int32, dim=1)
    n, d = rows.numel(), src.shape[1]
    if out is None:
        out = torch.empty(n, d, dtype=torch.float32, device=src.device)
    _req(out, "out", dim=2)
    _lib.call("kgat_gather_rows_f32", src.data_ptr(), _ld(src), rows.data_ptr(), n, d, out.data_ptr(), _ld(out),
              stream_ptr(src.device))
    return out


def scatter_rows(dst: torch.Tensor, rows: torch.Tensor, src: torch.Tensor, accumulate: bool = True) -> None:
    """dst[rows[i]] (+)= src[i] (rows int32 distinct, -1 skipped)."""
    _req(dst, "dst", dim=2)
    _req(src, "src", dim=2)
    _req(rows, "rows", dtype=torch.int32, dim=1)
    if src.shape[0] != rows.numel() or src.shape[1] != dst.shape[1]:
        raise ValueError("scatter_rows shape mismatch")
    _lib.call("kgat_scatter_rows_f32", dst.data_ptr(), _ld(dst), rows.data_ptr(), rows.numel(), dst.shape[1],
              src.data_ptr(), _ld(src), int(accumulate), stream_ptr(dst.device))


def add_(y: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """y += x (same shape, contiguous)."""
    _req(y, "y")
    _req(x, "x")
    if y.shape != x.shape or not (y.is_contiguous() and x.is_contiguous()):
        raise ValueError("add_: contiguous tensors of one shape")
    _lib.call("kgat_add_f32", y.data_ptr(), x.data_ptr(), y.numel(), stream_ptr(y.device))
    return y


def _bits_ptr(src_bits: torch.Tensor | None, src_map: torch.Tensor):
    if src_bits is None:
        return None
    _req(src_bits, "src_bits", dtype=torch.int32, dim=1)
    if src_bits.numel() < 2 * ((src_map.numel() + 63) // 64) or src_bits.data_ptr() % 8:
        raise ValueError("src_bits must be map_bits(src_map)")
    return src_bits.data_ptr()


def _rank_ptr(src_rank: torch.Tensor | None, src_map: torch.Tensor):
    if src_rank is None:
        return None
    _req(src_rank, "src_rank", dtype=torch.int64, dim=1)
    if src_rank.numel() < (src_map.numel() + 31) // 32:
        raise ValueError("src_rank must be map_rank(src_map)")
    return src_rank.data_ptr()


def map_rank(node_map: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out (int64 [ceil(N/32)]): rank words of the set of an ascending-order node map (kgat_map_rank)."""
    _req(node_map, "node_map", dtype=torch.int32, dim=1)
    _rank_ptr(out, node_map)
    _lib.call("kgat_map_rank", node_map.data_ptr(), node_map.numel(), out.data_ptr(), stream_ptr(node_map.device))
    return out


def map_bits(node_map: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out (int32 [2*ceil(N/64)], 8-byte aligned): bit i set <=> node_map[i] >= 0 (kgat_map_bits)."""
    _req(node_map, "node_map", dtype=torch.int32, dim=1)
    _bits_ptr(out, node_map)
    _lib.call("kgat_map_bits", node_map.data_ptr(), node_map.numel(), out.data_ptr(), stream_ptr(node_map.device))
    return out


def spmm_masked(graph: DeviceGraph, src_map: torch.Tensor, Xc: torch.Tensor, Yc_init: torch.Tensor | None = None,
                transpose: bool = False, row_hit: torch.Tensor | None = None,
                src_bits: torch.Tensor | None = None, src_rank: torch.Tensor | None = None) -> torch.Tensor:
    """Dense Y = A . X where X is zero outside a frontier: X[node] = Xc[src_map[node]] (src_map -1 => 0),
    plus Yc_init[src_map[r]] on frontier rows.  Returns a new dense [N, d] tensor.  With ``row_hit``
    (int32 [N]) the rows of Y that can be nonzero are flagged 1 (the next hop set, see hop_compact)."""
    _req(src_map, "src_map", dtype=torch.int32, dim=1)
    _req(Xc, "Xc", dim=2)
    if src_map.numel() != graph.n_nodes:
        raise ValueError("src_map must cover every node")
    d = Xc.shape[1]
    if Yc_init is not None:
        _req(Yc_init, "Yc_init", dim=2)
        if Yc_init.shape[1] != d:
            raise ValueError("Yc_init width mismatch")
    if row_hit is not None:
        _req(row_hit, "row_hit", dtype=torch.int32, dim=1)
        if row_hit.numel() != graph.n_nodes:
            raise ValueError("row_hit must cover every node")
    out = torch.empty(graph.n_nodes, d, dtype=torch.float32, device=Xc.device)
    csr = graph.AT if transpose else graph.A
    desc = csr.descriptor()
    ws = torch.empty(max(1, csr.n_seg * d), dtype=torch.float32, device=Xc.device)
    ev = SPMM_EVENTS
    if ev is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.call("kgat_spmm_csr_masked_ex_f32", ctypes.byref(desc), src_map.data_ptr(), Xc.data_ptr(), _ld(Xc),
              Yc_init.data_ptr() if Yc_init is not None else None, _ld(Yc_init) if Yc_init is not None else 0, 0,
              out.data_ptr(), _ld(out), d, row_hit.data_ptr() if row_hit is not None else None,
              _bits_ptr(src_bits, src_map), _rank_ptr(src_rank, src_map), src_map.numel(), ws.data_ptr(), ws.numel(),
              stream_ptr(Xc.device))
    if ev is not None:
        e1.record()
        ev.append((e0, e1, d, transpose, "masked"))
    return out


def spmm_masked_adam_block(csr, src_map: torch.Tensor, Xc: torch.Tensor, Yc_init: torch.Tensor | None, row0: int,
                           p: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step_size: float, beta1: float,
                           beta2: float, bc2_sqrt: float, eps: float, skip: torch.Tensor | None = None) -> None:
    """spmm_masked_adam on a row block of the transposed graph (a shard's rows of A^T, global columns):
    block row r is global row row0 + r (its Yc row: Yc_init[src_map[row0 + r]]); p / m / v are the
    block's rows (kgat_spmm_csr_masked_adam_block_f32)."""
    _req(src_map, "src_map", dtype=torch.int32, dim=1)
    _req(Xc, "Xc", dim=2)
    n, d = csr.n_rows, Xc.shape[1]
    for t, nm in ((p, "param"), (m, "exp_avg"), (v, "exp_avg_sq")):
        _req(t, nm, dim=2)
        if tuple(t.shape) != (n, d) or not t.is_contiguous():
            raise ValueError(f"{nm}: contiguous [{n}, {d}] expected, got {tuple(t.shape)}")
    if Yc_init is not None:
        _req(Yc_init, "Yc_init", dim=2)
        if Yc_init.shape[1] != d or row0 < 0 or row0 + n > src_map.numel():
            raise ValueError("Yc_init width / row0 mismatch")
    if n == 0:
        return
    desc = csr.descriptor()
    ws = torch.empty(max(1, csr.n_seg * d), dtype=torch.float32, device=Xc.device)
    ev = SPMM_EVENTS
    if ev is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.call("kgat_spmm_csr_masked_adam_block_f32", ctypes.byref(desc), src_map.data_ptr(), Xc.data_ptr(), _ld(Xc),
              Yc_init.data_ptr() if Yc_init is not None else None, _ld(Yc_init) if Yc_init is not None else 0,
              int(row0), None, p.data_ptr(), m.data_ptr(), v.data_ptr(), d, d, step_size, beta1, beta2, bc2_sqrt, eps,
              _skip_ptr(skip), ws.data_ptr(), ws.numel(), stream_ptr(Xc.device))
    if ev is not None:
        e1.record()
        ev.append((e0, e1, d, True, "fused_adam"))


def _skip_ptr(skip: torch.Tensor | None):
    """The optimiser skip flag (device int32 [1], kgat_ids_check_ex's bad_dev) or None."""
    if skip is None:
        return None
    _req(skip, "skip", dtype=torch.int32, dim=1)
    return skip.data_ptr()


def spmm_masked_adam(graph: DeviceGraph, src_map: torch.Tensor, Xc: torch.Tensor, Yc_init: torch.Tensor | None,
                     src_rank: torch.Tensor | None, p: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                     step_size: float, beta1: float, beta2: float, bc2_sqrt: float, eps: float,
                     skip: torch.Tensor | None = None, extra=None) -> None:
    """The table's Adam step fused into its gradient's last product: row r of the masked A^T product
    (spmm_masked(..., transpose=True)) is the gradient of table row r and goes straight into r's Adam
    update of p / m / v (adam_multi's arithmetic: the same bits as spmm_masked + adam_multi).  ``extra``:
    <= KGAT_ADAM_MAX_TENSORS adam_multi items [(p, g, m, v, step_size, bc2_sqrt), ...] stepped in the
    launch pair's fix-up launch (kgat_spmm_csr_masked_adam_multi_f32: the same bits as adam_multi)."""
    _req(src_map, "src_map", dtype=torch.int32, dim=1)
    _req(Xc, "Xc", dim=2)
    n, d = graph.n_nodes, Xc.shape[1]
    if src_map.numel() != n:
        raise ValueError("src_map must cover every node")
    for t, nm in ((p, "param"), (m, "exp_avg"), (v, "exp_avg_sq")):
        _req(t, nm, dim=2)
        if tuple(t.shape) != (n, d) or not t.is_contiguous():
            raise ValueError(f"{nm}: contiguous [{n}, {d}] expected, got {tuple(t.shape)}")
    if Yc_init is not None:
        _req(Yc_init, "Yc_init", dim=2)
        if Yc_init.shape[1] != d:
            raise ValueError("Yc_init width mismatch")
    csr = graph.AT
    desc = csr.descriptor()
    ws = torch.empty(max(1, csr.n_seg * d), dtype=torch.float32, device=Xc.device)
    ev = SPMM_EVENTS
    if ev is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    yc = (Yc_init.data_ptr() if Yc_init is not None else None, _ld(Yc_init) if Yc_init is not None else 0)
    rank = _rank_ptr(src_rank, src_map)

    if extra:
        if len(extra) > _lib.KGAT_ADAM_MAX_TENSORS:
            raise ValueError("spmm_masked_adam: at most KGAT_ADAM_MAX_TENSORS extra tensors")
        arr = _adam_array(extra)
        _lib.call("kgat_spmm_csr_masked_adam_multi_f32", ctypes.byref(desc), src_map.data_ptr(), Xc.data_ptr(),
                  _ld(Xc), yc[0], yc[1], rank, p.data_ptr(), m.data_ptr(), v.data_ptr(), d, d, step_size, beta1,
                  beta2, bc2_sqrt, eps, _skip_ptr(skip), ws.data_ptr(), ws.numel(), arr, len(extra),
                  stream_ptr(Xc.device))
    else:
        _lib.call("kgat_spmm_csr_masked_adam_block_f32", ctypes.byref(desc), src_map.data_ptr(), Xc.data_ptr(),
                  _ld(Xc), yc[0], yc[1], 0, rank, p.data_ptr(), m.data_ptr(), v.data_ptr(), d, d, step_size, beta1,
                  beta2, bc2_sqrt, eps, _skip_ptr(skip), ws.data_ptr(), ws.numel(), stream_ptr(Xc.device))
    if ev is not None:
        e1.record()
        ev.append((e0, e1, d, True, "fused_adam"))


def _host_ptr(t: torch.Tensor | None):
    """A pinned int32 host tensor the kernels write directly (host-mapped memory), or None."""
    if t is None:
        return None
    if t.device.type != "cpu" or not t.is_pinned() or t.dtype != torch.int32 or t.numel() < 1:
        raise ValueError("count_host: a pinned int32 host tensor")
    return t.data_ptr()


def hop_compact(graph: DeviceGraph, sync: bool = False, count_host: torch.Tensor | None = None):
    """The hop set flagged in graph.hop_buffers()'s row_hit by the last spmm_masked.

    Returns (rows int32 [N] -- the first n entries are the hop set, ascending --, node_map
    int32 [N] node -> position or -1, count int32 [1] on the device, n); the hop set's rank
    words are left in graph.hop_buffers()[9] (kgat_map_rank).  With ``sync`` the
    count is read back (one stream sync) and rows is cut to n; otherwise n is None and
    consumers read the count on the device (biinter_bwd_hop).  ``count_host`` (pinned int32): the
    kernel also writes the count there (the next step's hop-size estimate, model._hop_record)."""
    hb = graph.hop_buffers()
    hit, node_map, rows, count, work, host = hb[:6]
    dev = hit.device
    if sync and count_host is None:
        count_host = host
    hop_list(hit, node_map, rows, count, work, count_host)
    map_rank(node_map, hb[9])
    if not sync:
        return rows, node_map, count, None
    torch.cuda.current_stream(dev).synchronize()  # the kernel wrote count_host
    n = int(count_host[0])
    return rows[:n], node_map, count, n


def hop_list(hit: torch.Tensor, node_map: torch.Tensor, rows: torch.Tensor, count: torch.Tensor, work: torch.Tensor,
             count_host: torch.Tensor | None = None) -> None:
    """kgat_hop_compact on explicit buffers: the rows flagged in ``hit`` listed ascending in ``rows``
    (first count entries), ``node_map`` row -> position or -1, the count on the device (and in the
    pinned ``count_host``)."""
    n = hit.numel()
    if node_map.numel() < n or rows.numel() < max(n, 1) or work.numel() < int(_lib.lib().kgat_hop_compact_work_bytes(n)):
        raise ValueError("hop_list buffers too small")
    _lib.call("kgat_hop_compact", hit.data_ptr(), n, node_map.data_ptr(), rows.data_ptr(), count.data_ptr(),
              _host_ptr(count_host), work.data_ptr(), work.numel(), stream_ptr(hit.device))


def hop_bitmaps(graph: DeviceGraph):
    """(bits0, bits1, words): the two bitmaps kgat_frontier_hop marks (frontier, hop set) and their size in
    uint32 words -- what kgat_cf_begin zeroes for a following frontier_hop(precleared=True)."""
    hb = graph.hop_buffers()
    return hb[7], hb[6], (graph.n_nodes + 31) // 32


def hop_bitmaps_next(graph: DeviceGraph):
    """The TRAIN_CF prologue's bitmap plan (kgat_cf_begin_ex marks the batch's first hop itself): the
    graph keeps a second (frontier, hop set) pair that is all zero between steps; the step marks that
    one and zeroes the pair the previous step used, in the same launch.  Returns (mark = (bits0, bits1)
    of the next pair, clear = the current pair (bits0, bits1, words)); hop_bitmaps_commit makes the
    marked pair current once the launch is queued."""
    hb = graph.hop_buffers()
    alt = graph.__dict__.get("_hop_alt")
    if alt is None:  # the spare pair, zero (the invariant every commit keeps)
        alt = graph._hop_alt = (torch.zeros_like(hb[7]), torch.zeros_like(hb[6]))
    return alt, (hb[7], hb[6], (graph.n_nodes + 31) // 32)


def hop_bitmaps_commit(graph: DeviceGraph) -> None:
    """Swap the pairs after a kgat_cf_begin_ex launch that marked the spare one and zeroed the current
    one: the marked pair is the hop buffers' (hb[7], hb[6]) now, the zeroed one the spare."""
    hb = graph.hop_buffers()
    b0, b1 = graph._hop_alt
    graph._hop = hb[:6] + (b1, b0) + hb[8:]
    graph._hop_alt = (hb[7], hb[6])


PRECLEARED, PREMARKED = 1, 2  # frontier_hop's ``precleared`` states (_MarkedBatch.take_cleared)


def frontier_hop(graph: DeviceGraph, rows0: torch.Tensor, count_host: torch.Tensor | None = None,
                 precleared: int = 0):
    """The first hop set of the backward chain from the batch frontier rows0 (frontier_build's
    rows, -1 padded): (hop rows int32 [N] ascending -- first count valid --, node_map, count int32 [1]
    on the device, hop-set bitmap, frontier bitmap).  No graph scan: the frontier rows' A edges are
    marked (kgat_frontier_hop_ex); ``precleared``: PRECLEARED -- kgat_cf_begin zeroed the bitmaps already,
    PREMARKED -- kgat_cf_begin_ex marked the first hop in them too (only the listing runs)."""
    _req(rows0, "rows0", dtype=torch.int32, dim=1)
    hb = graph.hop_buffers()
    _, node_map, rows, count, _, _, bits1, bits0, work = hb[:9]
    desc = graph.A.descriptor()
    n0 = 0 if precleared == PREMARKED else rows0.numel()
    _lib.call("kgat_frontier_hop_ex", ctypes.byref(desc), rows0.data_ptr(), n0, bits0.data_ptr(),
              bits1.data_ptr(), node_map.data_ptr(), rows.data_ptr(), count.data_ptr(), _host_ptr(count_host),
              hb[9].data_ptr(), work.data_ptr(), work.numel(), _lib.KGAT_HOP_PRECLEARED if precleared else 0,
              stream_ptr(rows0.device))
    return rows, node_map, count, bits1, bits0


def rows_union(graph: DeviceGraph, lists: torch.Tensor, counts: torch.Tensor, cap: int):
    """Union of G ascending row lists (list g = lists[g*cap : g*cap + counts[g]], counts int32 [G] on
    the device) into graph.hop_buffers(): (rows int32 [N] ascending -- first count valid --, node_map,
    count int32 [1] on the device, rank words) (kgat_rows_union)."""
    _req(lists, "lists", dtype=torch.int32, dim=1)
    _req(counts, "counts", dtype=torch.int32, dim=1)
    G = counts.numel()
    if lists.numel() < G * cap:
        raise ValueError("lists must hold G * cap entries")
    hb = graph.hop_buffers()
    _, node_map, rows, count, _, _, bits, _, work = hb[:9]
    _lib.call("kgat_rows_union", lists.data_ptr(), counts.data_ptr(), G, cap, graph.n_nodes, bits.data_ptr(),
              node_map.data_ptr(), rows.data_ptr(), count.data_ptr(), hb[9].data_ptr(), work.data_ptr(), work.numel(),
              stream_ptr(lists.device))
    return rows, node_map, count, hb[9]


def rows_merge(lists: torch.Tensor, counts: torch.Tensor, cap: int, vals: torch.Tensor, rows: torch.Tensor,
               count: torch.Tensor, max_rows: int, scale: float) -> torch.Tensor:
    """out[k] = scale * sum over the lists holding rows[k] (in list order) of their vals rows, for k <
    count (device), out [max_rows, w] (kgat_rows_merge_f32)."""
    _req(lists, "lists", dtype=torch.int32, dim=1)
    _req(counts, "counts", dtype=torch.int32, dim=1)
    _req(vals, "vals", dim=2)
    _req(rows, "rows", dtype=torch.int32, dim=1)
    _req(count, "count", dtype=torch.int32, dim=1)
    G, w = counts.numel(), vals.shape[1]
    if vals.shape[0] < G * cap or lists.numel() < G * cap:
        raise ValueError("lists / vals must hold G * cap rows")
    out = torch.empty(max(max_rows, 1), w, dtype=torch.float32, device=vals.device)
    _lib.call("kgat_rows_merge_f32", lists.data_ptr(), counts.data_ptr(), G, cap, vals.data_ptr(), _ld(vals), w,
              rows.data_ptr(), count.data_ptr(), max_rows, out.data_ptr(), _ld(out), float(scale),
              stream_ptr(vals.device))
    return out


def spmm_masked_rows(graph: DeviceGraph, src_map, src_bits, Xc, Yc_init, out_rows, out_map, out_count, out_bits,
                     transpose: bool = True, Gc: torch.Tensor | None = None,
                     out_src: torch.Tensor | None = None) -> torch.Tensor:
    """The masked product (see spmm_masked) on the output rows of a hop set only, written compactly:
    Y[k] = row out_rows[k] for k < out_count (kgat_spmm_csr_masked_rows_ex_f32); returns Y [N, d]
    (capacity; the first count rows are valid).  ``Gc``: compact rows (src_map's numbering) added after
    the Yc_init term -- the BPR loss's batch-row gradient of this table (bpr_bwd_multi).  ``out_src`` (int32
    [N]): gets src_map[out_rows[k]] for the valid k (biinter_bwd_hop's gidx)."""
    _req(src_map, "src_map", dtype=torch.int32, dim=1)
    _req(Xc, "Xc", dim=2)
    d = Xc.shape[1]
    if Yc_init is not None:
        _req(Yc_init, "Yc_init", dim=2)
        if Yc_init.shape[1] != d:
            raise ValueError("Yc_init width mismatch")
    for t, nm in ((out_rows, "out_rows"), (out_map, "out_map"), (out_count, "out_count")):
        _req(t, nm, dtype=torch.int32, dim=1)
    _bits_ptr(out_bits, out_map)
    n = graph.n_nodes
    if src_map.numel() != n or out_map.numel() != n or out_rows.numel() < n:
        raise ValueError("maps must cover every node")
    out = torch.empty(n, d, dtype=torch.float32, device=Xc.device)
    csr = graph.AT if transpose else graph.A
    desc = csr.descriptor()
    ws = torch.empty(max(1, csr.n_seg * d), dtype=torch.float32, device=Xc.device)
    ev = SPMM_EVENTS
    if ev is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    if Gc is not None:
        _req(Gc, "Gc", dim=2)
        if Gc.shape[1] != d:
            raise ValueError("Gc width mismatch")
    if out_src is not None:
        _req(out_src, "out_src", dtype=torch.int32, dim=1)
        if out_src.numel() < n:
            raise ValueError("out_src must cover every node")
    _lib.call("kgat_spmm_csr_masked_rows_ex_f32", ctypes.byref(desc), src_map.data_ptr(),
              _bits_ptr(src_bits, src_map), Xc.data_ptr(), _ld(Xc), Yc_init.data_ptr() if Yc_init is not None else None,
              _ld(Yc_init) if Yc_init is not None else 0, Gc.data_ptr() if Gc is not None else None,
              _ld(Gc) if Gc is not None else 0, out_bits.data_ptr(), out_map.data_ptr(),
              out_rows.data_ptr(), out_count.data_ptr(), out.data_ptr(), _ld(out),
              out_src.data_ptr() if out_src is not None else None, d, ws.data_ptr(), ws.numel(),
              stream_ptr(Xc.device))
    if ev is not None:
        e1.record()
        ev.append((e0, e1, d, transpose, "masked"))
    return out


def spmm_rows(graph: DeviceGraph, X: torch.Tensor, out: torch.Tensor, out_rows: torch.Tensor,
              out_count: torch.Tensor, out_bits: torch.Tensor) -> torch.Tensor:
    """out[r] = (A . X)[r] for the rows r = out_rows[k], k < out_count (device), only; the other
    rows of ``out`` are left as they are (kgat_spmm_csr_rows_f32: same bits per row as spmm)."""
    _req(X, "X", dim=2)
    _req(out, "out", dim=2)
    n, d = X.shape
    if n != graph.n_nodes or tuple(out.shape) != (n, d):
        raise ValueError("X / out must be [n_nodes, d]")
    for t, nm in ((out_rows, "out_rows"), (out_count, "out_count")):
        _req(t, nm, dtype=torch.int32, dim=1)
    if out_bits.dtype != torch.int32 or out_bits.numel() * 32 < n:
        raise ValueError("out_bits must be an int32 bitmap covering every node")
    csr = graph.A
    desc = csr.descriptor()
    ws = torch.empty(max(1, csr.n_seg * d), dtype=torch.float32, device=X.device)
    ev = SPMM_EVENTS
    if ev is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.call("kgat_spmm_csr_rows_f32", ctypes.byref(desc), X.data_ptr(), _ld(X), out_bits.data_ptr(),
              out_rows.data_ptr(), out_count.data_ptr(), out.data_ptr(), _ld(out), d, ws.data_ptr(), ws.numel(),
              stream_ptr(X.device))
    if ev is not None:
        e1.record()
        ev.append((e0, e1, d, False, "rows"))
    return out


def spmm_rows_block(csr, X: torch.Tensor, out: torch.Tensor, out_rows: torch.Tensor, out_count: torch.Tensor,
                    out_bits: torch.Tensor) -> torch.Tensor:
    """spmm_rows on a rectangular CSR block (a shard's rows of A, global columns): out[r] = (B . X)[r]
    for r = out_rows[k], k < out_count; other rows of ``out`` untouched."""
    _req(X, "X", dim=2)
    _req(out, "out", dim=2)
    d = X.shape[1]
    if out.shape[0] != csr.n_rows or out.shape[1] != d:
        raise ValueError("out shape mismatch")
    for t, nm in ((out_rows, "out_rows"), (out_count, "out_count")):
        _req(t, nm, dtype=torch.int32, dim=1)
    if out_bits.dtype != torch.int32 or out_bits.numel() * 32 < csr.n_rows:
        raise ValueError("out_bits must be an int32 bitmap covering every row")
    if csr.n_rows == 0:
        return out
    desc = csr.descriptor()
    ws = torch.empty(max(1, csr.n_seg * d), dtype=torch.float32, device=X.device)
    ev = SPMM_EVENTS
    if ev is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    _lib.call("kgat_spmm_csr_rows_f32", ctypes.byref(desc), X.data_ptr(), _ld(X), out_bits.data_ptr(),
              out_rows.data_ptr(), out_count.data_ptr(), out.data_ptr(), _ld(out), d, ws.data_ptr(), ws.numel(),
              stream_ptr(X.device))
    if ev is not None:
        e1.record()
        ev.append((e0, e1, d, False, "rows"))
    return out


def csr_mark_rows(csr, bits: torch.Tensor, n_bits: int, row0: int, hit: torch.Tensor) -> torch.Tensor:
    """hit[r] = 1 iff row r of the block is in the node set ``bits`` (bit row0 + r) or has an edge into
    it, else 0 (kgat_csr_mark_rows)."""
    _req(hit, "hit", dtype=torch.int32, dim=1)
    if bits.dtype != torch.int32 or bits.numel() * 32 < n_bits or hit.numel() < csr.n_rows:
        raise ValueError("csr_mark_rows: bitmap / flags too small")
    desc = csr.descriptor()
    _lib.call("kgat_csr_mark_rows", ctypes.byref(desc), bits.data_ptr(), int(n_bits), int(row0), hit.data_ptr(),
              stream_ptr(hit.device))
    return hit


def biinter_fwd_gemm_rows(X, S, rows: torch.Tensor, m: int, W1, b1, W2, b2, dropout_p: float, seed: int,
                          out: torch.Tensor, state: "BiState") -> torch.Tensor:
    """The wide (GEMM) bi-interaction forward on rows[0..m) of X / S only (kgat_biinter_fwd_gemm_rows_f32):
    each listed row's H row, pre-activation state and norm land at its own index with the whole-table
    call's bits (same dropout draws); other rows of ``out`` and the state are untouched."""
    n, din = X.shape
    dout = W1.shape[0]
    _req(rows, "rows", dtype=torch.int32, dim=1)
    if S.shape != X.shape or tuple(out.shape) != (n, dout) or rows.numel() < m:
        raise ValueError("bi-interaction rows shape mismatch")
    if state.kind != "gemm" or state.n != n:
        raise ValueError("bi-interaction state does not match the layer")
    if m == 0:
        return out
    w = int(_lib.lib().kgat_biinter_gemm_rows_work_floats(m, din, dout))
    if w < 0:
        raise ValueError(f"unsupported bi-interaction shape {din}->{dout}")
    work = torch.empty(max(w, 1), dtype=torch.float32, device=X.device)
    _lib.call("kgat_biinter_fwd_gemm_rows_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S), rows.data_ptr(), int(m),
              W1.data_ptr(), b1.data_ptr(), W2.data_ptr(), b2.data_ptr(), out.data_ptr(), _ld(out), n, din, dout,
              float(dropout_p), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), state.P.data_ptr(), work.data_ptr(),
              work.numel(), stream_ptr(X.device))
    return out


def biinter_fwd_tiles(X, S, W1, b1, W2, b2, dropout_p: float, seed: int, out: torch.Tensor,
                      row_bits: torch.Tensor, state: BiState | None = None) -> torch.Tensor:
    """biinter_fwd on the 16-row tiles holding a member of the node set ``row_bits`` (int32 bitmap)
    only (kgat_biinter_fwd_tiles_f32): H / state rows of those tiles get the whole-table call's bits,
    the rest of ``out`` and the state are left as they are."""
    for t, nm in ((X, "X"), (S, "S"), (W1, "W1"), (W2, "W2"), (out, "out")):
        _req(t, nm, dim=2)
    n, din = X.shape
    dout = W1.shape[0]
    if row_bits.dtype != torch.int32 or row_bits.numel() * 32 < n or not row_bits.is_cuda:
        raise ValueError("row_bits must be an int32 device bitmap covering every row")
    if S.shape != X.shape or W1.shape != (dout, din) or W2.shape != (dout, din) or tuple(out.shape) != (n, dout):
        raise ValueError("bi-interaction shape mismatch")
    if not fused_supported(din, dout) or dout > 128:
        raise ValueError(f"no fused forward for {din}->{dout}")
    if not (W1.is_contiguous() and W2.is_contiguous()):
        raise ValueError("W must be contiguous")
    words = (dout + 63) // 64
    if state is not None and (state.kind not in ("fused", "bits") or state.norm.numel() < n
                              or state.mask.numel() < (n + 15) // 16 * 64 * words):
        raise ValueError("bi-interaction state too small")
    _lib.call("kgat_biinter_fwd_tiles_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S), W1.data_ptr(), b1.data_ptr(),
              W2.data_ptr(), b2.data_ptr(), out.data_ptr(), _ld(out), n, row_bits.data_ptr(), din, dout,
              float(dropout_p), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
              state.norm.data_ptr() if state is not None else None,
              state.mask.data_ptr() if state is not None else None, stream_ptr(X.device))
    return out


def biinter_fwd_list(X, S, W1, b1, W2, b2, dropout_p: float, seed: int, out: torch.Tensor,
                     rows: torch.Tensor, count: torch.Tensor, state: BiState | None = None) -> torch.Tensor:
    """biinter_fwd on the 4-row quads holding a listed node only (kgat_biinter_fwd_list_f32): rows[0..*count)
    (int32, count a device int32; -1 = padding).  H / state rows of those quads get the whole-table call's
    bits, the rest of ``out`` and the state are left as they are."""
    for t, nm in ((X, "X"), (S, "S"), (W1, "W1"), (W2, "W2"), (out, "out")):
        _req(t, nm, dim=2)
    n, din = X.shape
    dout = W1.shape[0]
    _req(rows, "rows", dtype=torch.int32, dim=1)
    if count.dtype != torch.int32 or count.numel() < 1 or not count.is_cuda or not rows.is_contiguous():
        raise ValueError("rows / count must be contiguous int32 device tensors")
    if S.shape != X.shape or W1.shape != (dout, din) or W2.shape != (dout, din) or tuple(out.shape) != (n, dout):
        raise ValueError("bi-interaction shape mismatch")
    if not fused_supported(din, dout) or dout > 128:
        raise ValueError(f"no fused forward for {din}->{dout}")
    if not (W1.is_contiguous() and W2.is_contiguous()):
        raise ValueError("W must be contiguous")
    words = (dout + 63) // 64
    if state is not None and (state.kind not in ("fused", "bits") or state.norm.numel() < n
                              or state.mask.numel() < (n + 15) // 16 * 64 * words):
        raise ValueError("bi-interaction state too small")
    _lib.call("kgat_biinter_fwd_list_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S), W1.data_ptr(), b1.data_ptr(),
              W2.data_ptr(), b2.data_ptr(), out.data_ptr(), _ld(out), n, rows.data_ptr(), count.data_ptr(),
              rows.numel(), din, dout, float(dropout_p), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
              state.norm.data_ptr() if state is not None else None,
              state.mask.data_ptr() if state is not None else None, stream_ptr(X.device))
    return out


def biinter_bwd_hop(X, S, dH, W1, W2, dropout_p: float, rows, count, H, state: BiState, out_rows: int,
                    dh_compact: bool = False, out=None, G: torch.Tensor | None = None,
                    gidx: torch.Tensor | None = None, gmap: torch.Tensor | None = None):
    """Saved-state bi-interaction backward on a hop set whose size is only known on the device:
    rows / count from hop_compact or frontier_hop, dH indexed by node ([N, d_out], the previous
    masked product's output) or, with ``dh_compact``, by hop position (spmm_masked_rows' output).
    Returns compact (dXd, dS) with ``out_rows`` rows allocated (the first count are valid) and
    (dW1, db1, dW2, db2).  ``out`` = (dXd, dS): caller-owned [>= out_rows, d_in] views to write
    (e.g. the two halves of one [cap, 2*d_in] exchange buffer).  ``G`` / ``gidx``: the BPR loss's
    batch-row gradient of this table (compact, bpr_bwd_multi) and, per hop position, its G row or -1
    (spmm_masked_rows' out_src) -- added to dXd in the same launch; ``gmap`` (optional): the batch-row
    node map numbering G, its entries of those rows reset to -1 (kgat_biinter_bwd_hop_ex_f32)."""
    src_rows, din = X.shape
    dout = W1.shape[0]
    for t, nm in ((X, "X"), (S, "S"), (dH, "dH"), (H, "H")):
        _req(t, nm, dim=2)
    if dH.shape[1] != dout or (not dh_compact and dH.shape[0] != src_rows) or (dh_compact and dH.shape[0] < out_rows) \
            or H.shape != (src_rows, dout) or S.shape != X.shape:
        raise ValueError("hop backward shape mismatch")
    if state is None or state.kind != "fused" or not saved_state_supported(din, dout):
        raise ValueError("hop backward needs the fused saved state")
    if out_rows < 1 or rows.numel() < out_rows:
        raise ValueError("hop rows buffer too small")
    dev = X.device
    if out is not None:
        dXd, dS = out
        for t, nm in ((dXd, "out dXd"), (dS, "out dS")):
            _req(t, nm, dim=2)
            if t.shape[0] < out_rows or t.shape[1] != din:
                raise ValueError(f"{nm}: [>= {out_rows}, {din}] expected, got {tuple(t.shape)}")
    else:
        dXd = torch.empty(out_rows, din, dtype=torch.float32, device=dev)
        dS = torch.empty(out_rows, din, dtype=torch.float32, device=dev)
    dW1, dW2 = torch.empty_like(W1), torch.empty_like(W2)
    db1 = torch.empty(dout, dtype=torch.float32, device=dev)
    db2 = torch.empty(dout, dtype=torch.float32, device=dev)
    ws_n = int(_lib.lib().kgat_biinter_bwd_workspace(out_rows, din, dout))
    ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=dev)
    if (G is None) != (gidx is None):
        raise ValueError("G and gidx go together")
    if G is not None:
        _req(G, "G", dim=2)
        _req(gidx, "gidx", dtype=torch.int32, dim=1)
        if G.shape[1] != din or gidx.numel() < out_rows:
            raise ValueError("G / gidx shape mismatch")
    if gmap is not None:
        _req(gmap, "gmap", dtype=torch.int32, dim=1)
        if gmap.numel() < src_rows:
            raise ValueError("gmap must cover every node")
    _lib.call("kgat_biinter_bwd_hop_ex_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S), H.data_ptr(), _ld(H),
              state.norm.data_ptr(), state.mask.data_ptr(), dH.data_ptr(), _ld(dH), W1.data_ptr(), W2.data_ptr(),
              dXd.data_ptr(), _ld(dXd), dS.data_ptr(), _ld(dS), dW1.data_ptr(), db1.data_ptr(), dW2.data_ptr(),
              db2.data_ptr(), rows.data_ptr(), count.data_ptr(), out_rows, src_rows, int(dh_compact), din, dout,
              float(dropout_p), G.data_ptr() if G is not None else None, _ld(G) if G is not None else 0,
              gidx.data_ptr() if gidx is not None else None, gmap.data_ptr() if gmap is not None else None,
              ws.data_ptr(), ws.numel(), stream_ptr(dev))
    return dXd, dS, dW1, db1, dW2, db2


def frontier_build(users, pos, neg, node_map: torch.Tensor):
    """(rows int32 [3B] -- distinct batch ids in first-occurrence order, -1 padded -- , count int32 [1])."""
    B = users.numel()
    rows = torch.empty(3 * B, dtype=torch.int32, device=users.device)
    count = torch.empty(1, dtype=torch.int32, device=users.device)
    _lib.call("kgat_frontier_build", users.data_ptr(), pos.data_ptr(), neg.data_ptr(), B, node_map.data_ptr(),
              rows.data_ptr(), count.data_ptr(), stream_ptr(users.device))
    return rows, count


def frontier_reset(rows: torch.Tensor, node_map: torch.Tensor) -> None:
    _lib.call("kgat_frontier_reset", rows.data_ptr(), rows.numel(), node_map.data_ptr(), stream_ptr(rows.device))


# (d_in, d_out) pairs the fused kernels of csrc/biinter.hip dispatch; others run the
# GEMM (csrc/gemm.hip) + epilogue path of csrc/biinter_gemm.hip (kgat_biinter_*_gemm_f32).
FUSED_SHAPES = {(16, 16), (32, 16), (32, 32), (64, 16), (64, 32), (64, 64), (128, 32), (128, 64), (128, 128),
                (32, 64), (16, 32), (64, 128)}


def fused_supported(d_in: int, d_out: int) -> bool:
    return (d_in, d_out) in FUSED_SHAPES


# C4's wide fused shapes (d_out > 64 or d_in * d_out > 4096: no saved-state fused backward) run the
# fused MFMA forward keeping its norm + sign/keep bits and the GEMM backward from those bits
# (kgat_biinter_bwd_gemm_bits_f32) -- instead of the rocBLAS forward with its [n, 2*d_out]
# pre-activation state.


def bits_supported(d_in: int, d_out: int) -> bool:
    return fused_supported(d_in, d_out) and d_out <= 128 and not saved_state_supported(d_in, d_out)


class BiState:
    """The forward's saved state for the backward, indexed by node.
    fused shapes (kgat_biinter_fwd_f32 norm_out / mask_out): row norms + per-lane sign/keep words;
    "bits": the same state for wide fused shapes (ceil(d_out/64) words per lane), consumed by the
    GEMM backward; wide shapes (kgat_biinter_fwd_gemm_f32): pre-activations P1+b1, P2+b2 and row norms."""

    def __init__(self, n: int, device, d_in: int = 64, d_out: int = 64, kind: str | None = None):
        self.n, self.d_in, self.d_out = n, d_in, d_out
        if kind is None:
            kind = "fused" if saved_state_supported(d_in, d_out) else ("bits" if bits_supported(d_in, d_out)
                                                                      else "gemm")
        if kind == "fused" and not saved_state_supported(d_in, d_out):
            raise ValueError(f"no fused saved state for {d_in}->{d_out}")
        if kind == "bits" and not (fused_supported(d_in, d_out) and d_out <= 128):
            raise ValueError(f"no fused forward for {d_in}->{d_out}")
        self.kind = kind
        if self.kind in ("fused", "bits"):
            words = (d_out + 63) // 64
            self.norm = torch.empty(max((n + 15) // 16 * 16, 16), dtype=torch.float32, device=device)
            self.mask = torch.empty(max((n + 15) // 16, 1) * 64 * words, dtype=torch.int64, device=device)
        else:
            m = int(_lib.lib().kgat_biinter_gemm_state_floats(n, d_in, d_out))
            if m < 0:
                raise ValueError(f"unsupported bi-interaction shape {d_in}->{d_out}")
            self.P = torch.empty(max(m, 1), dtype=torch.float32, device=device)

    def gemm_views(self):
        n, o = self.n, self.d_out
        return self.P[:n * o].view(n, o), self.P[n * o:2 * n * o].view(n, o), self.P[2 * n * o:2 * n * o + n]


def saved_state_supported(d_in: int, d_out: int) -> bool:
    """Fused shapes whose backward runs from the saved state (see kgat_biinter_bwd_f32)."""
    return d_out <= 64 and d_in * d_out <= 4096


def make_state(n: int, d_in: int, d_out: int, device) -> BiState:
    """The state a training forward keeps for this layer's backward: the fused kernels' norm + sign
    words where the saved-state backward exists (d_out <= 64, d_in*d_out <= 4096), else the GEMM
    path's pre-activations -- e.g. C4's 128->128 layer, whose recomputing fused backward is 6x slower
    than GEMMs on MI355X at 10M rows."""
    return BiState(n, device, d_in, d_out)


def _gemm_work(n: int, d_in: int, d_out: int, device) -> torch.Tensor:
    m = int(_lib.lib().kgat_biinter_gemm_work_floats(n, d_in, d_out))
    if m < 0:
        raise ValueError(f"unsupported bi-interaction shape {d_in}->{d_out}")
    return torch.empty(max(m, 1), dtype=torch.float32, device=device)


def biinter_fwd(X, S, W1, b1, W2, b2, dropout_p: float = 0.0, seed: int = 0, out=None,
                state: BiState | None = None) -> torch.Tensor:
    for t, nm in ((X, "X"), (S, "S"), (W1, "W1"), (W2, "W2")):
        _req(t, nm, dim=2)
    _req(b1, "b1", dim=1)
    _req(b2, "b2", dim=1)
    n, din = X.shape
    dout = W1.shape[0]
    if S.shape != X.shape or W1.shape != (dout, din) or W2.shape != (dout, din) or b1.numel() != dout:
        raise ValueError("bi-interaction shape mismatch")
    if not (W1.is_contiguous() and W2.is_contiguous()):
        raise ValueError("W must be contiguous")
    if out is None:
        out = torch.empty(n, dout, dtype=torch.float32, device=X.device)
    if not fused_supported(din, dout) or (state is not None and state.kind == "gemm"):
        st = state if state is not None else BiState(n, X.device, din, dout, kind="gemm")
        if st.kind != "gemm" or st.n != n:
            raise ValueError("bi-interaction state does not match the layer")
        work = _gemm_work(n, din, dout, X.device)
        _lib.call("kgat_biinter_fwd_gemm_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S), W1.data_ptr(),
                  b1.data_ptr(), W2.data_ptr(), b2.data_ptr(), out.data_ptr(), _ld(out), n, din, dout,
                  float(dropout_p), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), st.P.data_ptr(), work.data_ptr(),
                  work.numel(), stream_ptr(X.device))
        return out
    words = (dout + 63) // 64
    if state is not None and (state.kind not in ("fused", "bits") or state.norm.numel() < n
                              or state.mask.numel() < (n + 15) // 16 * 64 * words or dout > 128):
        raise ValueError("bi-interaction state too small or d_out > 128")
    _lib.call("kgat_biinter_fwd_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S), W1.data_ptr(), b1.data_ptr(),
              W2.data_ptr(), b2.data_ptr(), out.data_ptr(), _ld(out), n, din, dout, float(dropout_p),
              ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), state.norm.data_ptr() if state is not None else None,
              state.mask.data_ptr() if state is not None else None, stream_ptr(X.device))
    return out


def propagate_layer(graph: DeviceGraph, X, W1, b1, W2, b2, dropout_p: float = 0.0, seed: int = 0,
                    state: BiState | None = None):
    """One KGAT layer forward (aggregator.py:54-65): S = A . X, H = biinter(X, S); returns (S, H).
    (Row-block pipelining of the two launches on two streams and a one-pass propagation +
    bi-interaction kernel both measured slower)"""
    S = spmm(graph, X)
    return S, biinter_fwd(X, S, W1, b1, W2, b2, dropout_p, seed, state=state)


def biinter_fwd_rows(X, S, W1, b1, W2, b2, r0: int, n_rows: int, H, dropout_p: float = 0.0, seed: int = 0,
                     state: BiState | None = None) -> None:
    """kgat_biinter_fwd_rows_f32: the fused forward of rows [r0, r0 + n_rows) of the whole-table
    call (X, S, H whole tables; r0 a multiple of 16; the dropout draws and the saved state of those
    rows exactly the whole call's)."""
    n, din = X.shape
    dout = W1.shape[0]
    if r0 % 16 or r0 < 0 or n_rows < 0 or r0 + n_rows > n or (state is not None and not saved_state_supported(din, dout)):
        raise ValueError("biinter_fwd_rows: r0 a multiple of 16 inside the table; state only for saved-state shapes")
    if S.shape != X.shape or H.shape != (n, dout) or W1.shape != (dout, din) or not fused_supported(din, dout):
        raise ValueError("bi-interaction shape mismatch")
    ldx, lds, ldh = _ld(X), _ld(S), _ld(H)
    _lib.call("kgat_biinter_fwd_rows_f32", X.data_ptr() + 4 * r0 * ldx, ldx, S.data_ptr() + 4 * r0 * lds, lds,
              W1.data_ptr(), b1.data_ptr(), W2.data_ptr(), b2.data_ptr(), H.data_ptr() + 4 * r0 * ldh, ldh, n_rows,
              r0, din, dout, float(dropout_p), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
              state.norm.data_ptr() + 4 * r0 if state is not None else None,
              state.mask.data_ptr() + 8 * (r0 // 16) * 64 if state is not None else None, stream_ptr(X.device))


def biinter_bwd(X, S, dH, W1, b1, W2, b2, dropout_p: float = 0.0, seed: int = 0, dXd=None, dS=None,
                rows: torch.Tensor | None = None, H: torch.Tensor | None = None, state: BiState | None = None,
                dh_full: bool = False, split: bool = False):
    """Returns (dXd, dS, dW1, db1, dW2, db2).  With ``rows`` (int32 [n]), dH/dXd/dS are compact:
    row i belongs to node rows[i] of X and S (-1 = padding).  With the forward's output ``H`` and
    ``state``, the backward reads them instead of recomputing the forward.  ``dh_full`` (with rows):
    dH is indexed by node ([X rows, d_out]); the wide kinds then read every operand through the row
    list (kgat_biinter_bwd_gemm_rows_f32: no gathered copies, same bits).  ``split`` (that wide row-list
    case only): returns (dXd, dS, finish), finish() -> (dW1, db1, dW2, db2) -- the weight gradients run
    when the caller has started what depends on dXd / dS only."""
    src_rows, din = X.shape
    dout = W1.shape[0]
    _req(dH, "dH", dim=2)
    n = src_rows
    if rows is not None:
        _req(rows, "rows", dtype=torch.int32, dim=1)
        n = rows.numel()
    if dh_full:
        if rows is None or dH.shape != (src_rows, dout):
            raise ValueError("dh_full needs rows and a [nodes, d_out] dH")
        if state is not None and state.kind in ("gemm", "bits") and H is not None:
            return _biinter_bwd_rows(X, S, dH, W1, W2, dropout_p, seed, dXd, dS, rows, H, state, split=split)
        dH = gather_rows(dH, rows)
    if split:
        out = biinter_bwd(X, S, dH, W1, b1, W2, b2, dropout_p, seed, dXd, dS, rows, H, state)
        return out[0], out[1], lambda: out[2:]
    if dH.shape != (n, dout):
        raise ValueError("dH shape mismatch")
    if (H is None) != (state is None):
        raise ValueError("H and state go together")
    if H is not None:
        _req(H, "H", dim=2)
        if H.shape != (src_rows, dout):
            raise ValueError("H shape mismatch")
    dev = X.device
    dXd = torch.empty(n, din, dtype=torch.float32, device=dev) if dXd is None else dXd
    dS = torch.empty(n, din, dtype=torch.float32, device=dev) if dS is None else dS
    dW1 = torch.empty_like(W1)
    dW2 = torch.empty_like(W2)
    db1 = torch.empty_like(b1)
    db2 = torch.empty_like(b2)
    if state is not None and state.kind == "bits":
        _biinter_bwd_bits(X, S, dH, W1, W2, dropout_p, dXd, dS, dW1, db1, dW2, db2, rows, H, state)
        return dXd, dS, dW1, db1, dW2, db2
    if not fused_supported(din, dout) or (state is not None and state.kind == "gemm"):
        _biinter_bwd_gemm(X, S, dH, W1, b1, W2, b2, dropout_p, seed, dXd, dS, dW1, db1, dW2, db2, rows, H, state)
        return dXd, dS, dW1, db1, dW2, db2
    ws_n = int(_lib.lib().kgat_biinter_bwd_workspace(n, din, dout))
    if ws_n < 0:
        raise ValueError(f"unsupported bi-interaction shape {din}->{dout}")
    ws = torch.empty(max(ws_n, 1), dtype=torch.float32, device=dev)
    _lib.call("kgat_biinter_bwd_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S),
              H.data_ptr() if H is not None else None, _ld(H) if H is not None else 0,
              state.norm.data_ptr() if state is not None else None,
              state.mask.data_ptr() if state is not None else None, dH.data_ptr(), _ld(dH),
              W1.data_ptr(), b1.data_ptr(), W2.data_ptr(), b2.data_ptr(), dXd.data_ptr(), _ld(dXd), dS.data_ptr(),
              _ld(dS), dW1.data_ptr(), db1.data_ptr(), dW2.data_ptr(), db2.data_ptr(), n, din, dout,
              float(dropout_p), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
              rows.data_ptr() if rows is not None else None, src_rows, ws.data_ptr(), ws.numel(), stream_ptr(dev))
    return dXd, dS, dW1, db1, dW2, db2


def _biinter_bwd_rows(X, S, dH, W1, W2, p, seed, dXd, dS, rows, H, state, split: bool = False):
    """The wide backward on a row list, every operand read through it (kgat_biinter_bwd_gemm_rows_f32).
    ``split``: returns (dXd, dS, finish) after the dXd / dS half (kgat_biinter_bwd_gemm_rows_ex_f32 phase
    1); finish() runs the weight gradients (phase 2) and returns (dW1, db1, dW2, db2) -- same bits."""
    src_rows, din = X.shape
    dout = W1.shape[0]
    dev = X.device
    m = rows.numel()
    _req(H, "H", dim=2)
    if H.shape != (src_rows, dout) or state.n != src_rows:
        raise ValueError("bi-interaction state does not match the layer")
    dXd = torch.empty(m, din, dtype=torch.float32, device=dev) if dXd is None else dXd
    dS = torch.empty(m, din, dtype=torch.float32, device=dev) if dS is None else dS
    dW1, dW2 = torch.empty_like(W1), torch.empty_like(W2)
    db1 = torch.empty(dout, dtype=torch.float32, device=dev)
    db2 = torch.empty(dout, dtype=torch.float32, device=dev)
    w = int(_lib.lib().kgat_biinter_bwd_gemm_rows_work_floats(m, din, dout))
    if w < 0:
        raise ValueError(f"unsupported bi-interaction shape {din}->{dout}")
    work = torch.empty(max(w, 1), dtype=torch.float32, device=dev)
    gemm = state.kind == "gemm"

    def call(phases):
        _lib.call("kgat_biinter_bwd_gemm_rows_ex_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S), H.data_ptr(),
                  _ld(H), state.P.data_ptr() if gemm else None, None if gemm else state.norm.data_ptr(),
                  None if gemm else state.mask.data_ptr(), dH.data_ptr(), _ld(dH), rows.data_ptr(), m,
                  W1.data_ptr(), W2.data_ptr(), dXd.data_ptr(), _ld(dXd), dS.data_ptr(), _ld(dS), dW1.data_ptr(),
                  db1.data_ptr(), dW2.data_ptr(), db2.data_ptr(), src_rows, din, dout, float(p),
                  ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), work.data_ptr(), work.numel(), phases, stream_ptr(dev))
    if split:
        call(1)

        def finish():
            call(2)
            return dW1, db1, dW2, db2
        return dXd, dS, finish
    call(3)
    return dXd, dS, dW1, db1, dW2, db2


def _biinter_bwd_gemm(X, S, dH, W1, b1, W2, b2, p, seed, dXd, dS, dW1, db1, dW2, db2, rows, H, state) -> None:
    """Wide-layer backward (kgat_biinter_bwd_gemm_f32); frontier rows are gathered to a compact problem."""
    src_rows, din = X.shape
    dout = W1.shape[0]
    dev = X.device
    if H is None or state is None:  # no saved forward: recompute it
        state = BiState(src_rows, dev, din, dout, kind="gemm")
        H = biinter_fwd(X, S, W1, b1, W2, b2, p, seed, state=state)
    if state.kind != "gemm" or state.n != src_rows:
        raise ValueError("bi-interaction state does not match the layer")
    key = None
    if rows is not None:
        n = rows.numel()
        P1, P2, norm = state.gemm_views()
        Xc, Sc, Hc = gather_rows(X, rows), gather_rows(S, rows), gather_rows(H, rows)
        comp = BiState(n, dev, din, dout, kind="gemm")
        c1, c2, cn = comp.gemm_views()
        gather_rows(P1, rows, out=c1)
        gather_rows(P2, rows, out=c2)
        safe = rows.clamp_min(0)
        _lib.call("kgat_gather_f32", norm.data_ptr(), safe.data_ptr(), n, cn.data_ptr(), stream_ptr(dev))
        X, S, H, state, key = Xc, Sc, Hc, comp, rows
    n = X.shape[0]
    work = _gemm_work(n, din, dout, dev)
    _lib.call("kgat_biinter_bwd_gemm_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S), H.data_ptr(), _ld(H),
              state.P.data_ptr(), dH.data_ptr(), _ld(dH), W1.data_ptr(), W2.data_ptr(), dXd.data_ptr(), _ld(dXd),
              dS.data_ptr(), _ld(dS), dW1.data_ptr(), db1.data_ptr(), dW2.data_ptr(), db2.data_ptr(), n, din, dout,
              float(p), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), key.data_ptr() if key is not None else None,
              work.data_ptr(), work.numel(), stream_ptr(dev))


def _biinter_bwd_bits(X, S, dH, W1, W2, p, dXd, dS, dW1, db1, dW2, db2, rows, H, state) -> None:
    """Wide-layer backward from the fused forward's norm + sign/keep bits (kgat_biinter_bwd_gemm_bits_f32);
    frontier rows: X, S, H gathered to a compact problem, the state read by node id."""
    src_rows, din = X.shape
    dout = W1.shape[0]
    dev = X.device
    if H is None or state.n != src_rows:
        raise ValueError("bi-interaction state does not match the layer")
    key = None
    if rows is not None:
        X, S, H, key = gather_rows(X, rows), gather_rows(S, rows), gather_rows(H, rows), rows
    n = X.shape[0]
    m = int(_lib.lib().kgat_biinter_gemm_bits_work_floats(n, din, dout))
    if m < 0:
        raise ValueError(f"unsupported bi-interaction shape {din}->{dout}")
    work = torch.empty(max(m, 1), dtype=torch.float32, device=dev)
    _lib.call("kgat_biinter_bwd_gemm_bits_f32", X.data_ptr(), _ld(X), S.data_ptr(), _ld(S), H.data_ptr(), _ld(H),
              state.norm.data_ptr(), state.mask.data_ptr(), dH.data_ptr(), _ld(dH), W1.data_ptr(), W2.data_ptr(),
              dXd.data_ptr(), _ld(dXd), dS.data_ptr(), _ld(dS), dW1.data_ptr(), db1.data_ptr(), dW2.data_ptr(),
              db2.data_ptr(), n, din, dout, float(p), key.data_ptr() if key is not None else None, work.data_ptr(),
              work.numel(), stream_ptr(dev))


def make_tables(tables: list[torch.Tensor]) -> _lib.Tables:
    if not 1 <= len(tables) <= _lib.KGAT_MAX_TABLES:
        raise ValueError("1..8 tables supported")
    T = _lib.Tables()
    for i, t in enumerate(tables):
        _req(t, f"table{i}", dim=2)
        T.ptr[i] = t.data_ptr()
        T.ld[i] = _ld(t)
        T.width[i] = t.shape[1]
    T.count = len(tables)
    return T


_TICKETS: dict = {}


def ticket_word(device: torch.device, slot: int) -> torch.Tensor:
    """A device uint32 word that is 0 between launches (the in-launch reductions' arrival counters,
    e.g. kgat_bpr_fwd_ex_f32's): per (device, stream), one slot per kernel kind -- launches sharing a
    word are ordered by their stream, so two streams running the same kernel kind never share one."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (device.type, idx, torch.cuda.current_stream(idx).cuda_stream)
    buf = _TICKETS.get(key)
    if buf is None:
        buf = _TICKETS[key] = torch.zeros(64, dtype=torch.int32, device=device)
    return buf[slot:slot + 1]


TICKET_BPR_FWD = 0


def bpr_fwd(tables: list[torch.Tensor], users, pos, neg, reg: float):
    """(loss [1], coef [B]); one launch (kgat_bpr_fwd_ex_f32: the loss summed by the last block)."""
    for t, nm in ((users, "users"), (pos, "pos"), (neg, "neg")):
        _req(t, nm, dtype=torch.int64, dim=1)
    B = users.numel()
    if pos.numel() != B or neg.numel() != B or B == 0:
        raise ValueError("batch size mismatch")
    dev = users.device
    loss = torch.empty(1, dtype=torch.float32, device=dev)
    coef = torch.empty(2 * B, dtype=torch.float32, device=dev)  # [coef | per-sample terms]
    T = make_tables(tables)
    _lib.call("kgat_bpr_fwd_ex_f32", ctypes.byref(T), users.data_ptr(), pos.data_ptr(), neg.data_ptr(), B, float(reg),
              loss.data_ptr(), coef.data_ptr(), ticket_word(dev, TICKET_BPR_FWD).data_ptr(), stream_ptr(dev))
    return loss, coef


def bpr_bwd_multi(tables: list[torch.Tensor], t0: int, users, pos, neg, reg: float, coef, grad_out,
                  dsts: list, rows: torch.Tensor, count: torch.Tensor) -> None:
    """kgat_bpr_bwd_multi_f32: for t >= t0 with dsts[t] given, dsts[t][p] = dL/d tables[t][rows[p]] for the
    frontier rows p < count (frontier_build's list; written, rows [count, 3B) zeroed) -- every layer's
    batch-row term in one launch."""
    _req(grad_out, "grad_out")
    _req(rows, "rows", dtype=torch.int32, dim=1)
    _req(count, "count", dtype=torch.int32, dim=1)
    T = make_tables(tables)
    D = _lib.Tables()
    B = users.numel()
    for i, t in enumerate(tables):
        d = dsts[i] if i < len(dsts) else None
        if i >= t0 and d is not None:
            _req(d, f"dst{i}", dim=2)
            if d.shape[1] != t.shape[1] or d.shape[0] < 3 * B:
                raise ValueError(f"bpr_bwd_multi: dst{i} must be [>= 3B, {t.shape[1]}]")
            D.ptr[i], D.ld[i], D.width[i] = d.data_ptr(), _ld(d), t.shape[1]
    D.count = T.count
    _lib.call("kgat_bpr_bwd_multi_f32", ctypes.byref(T), int(t0), users.data_ptr(), pos.data_ptr(), neg.data_ptr(), B,
              float(reg), coef.data_ptr(), grad_out.data_ptr(), ctypes.byref(D), rows.data_ptr(), count.data_ptr(),
              stream_ptr(users.device))


def cf_begin(users, pos, neg, bound: int, bad_host: torch.Tensor, bad_dev: torch.Tensor | None,
             node_map: torch.Tensor, clear: tuple | None = None, tag: int = 0, mark=None):
    """kgat_cf_begin_ex: (checked int64 ids [3B] = users | pos | neg, frontier rows int32 [3B], count int32 [1]).
    ``clear`` = (bits0, bits1, words): kgat_frontier_hop's bitmaps, zeroed by the same launch; ``tag`` > 0:
    ``bad_host`` holds two pinned words, [0] the bad flag (set only) and [1] the tag, written when the
    check is done.  ``mark`` = (graph, (bits0, bits1)): the same launch marks the batch's first hop in that
    (zero) pair, a different one from ``clear`` (hop_bitmaps_next)."""
    for t, nm in ((users, "users"), (pos, "pos"), (neg, "neg")):
        _req(t, nm, dtype=torch.int64, dim=1)
    B = users.numel()
    if pos.numel() != B or neg.numel() != B or B == 0 or 3 * B > 4096:
        raise ValueError("cf_begin: three id arrays of one batch size, 3B <= 4096")
    dev = users.device
    ids = torch.empty(3 * B, dtype=torch.int64, device=dev)
    rows = torch.empty(3 * B, dtype=torch.int32, device=dev)
    count = torch.empty(1, dtype=torch.int32, device=dev)
    c0 = c1 = None
    words = 0
    if clear is not None:
        b0, b1, words = clear
        c0, c1 = b0.data_ptr(), b1.data_ptr()
    if not 0 <= tag < (1 << 29) or (tag and bad_host.numel() < 2):
        raise ValueError("cf_begin: tag in [0, 2^29); a tag needs two pinned words")
    desc = m0 = m1 = None
    if mark is not None:
        g, (b0, b1) = mark
        if g.n_nodes != int(bound) or b0.numel() * 32 < bound or b1.numel() * 32 < bound:
            raise ValueError("cf_begin: the marked bitmaps must cover the graph's nodes")
        desc = ctypes.byref(g.A.descriptor())
        m0, m1 = b0.data_ptr(), b1.data_ptr()
    _lib.call("kgat_cf_begin_ex", users.data_ptr(), pos.data_ptr(), neg.data_ptr(), B, int(bound), ids.data_ptr(),
              bad_host.data_ptr(), bad_dev.data_ptr() if bad_dev is not None else None, node_map.data_ptr(),
              rows.data_ptr(), count.data_ptr(), c0, c1, int(words), desc, m0, m1, int(tag), stream_ptr(dev))
    return ids, rows, count


def bpr_bwd(tables: list[torch.Tensor], t: int, users, pos, neg, reg: float, coef, grad_out, dst,
            row_map: torch.Tensor | None = None) -> None:
    """dst[id] += dL/d tables[t][id] for every gathered id (deterministic); with row_map, dst[row_map[id]]."""
    _req(dst, "dst", dim=2)
    _req(grad_out, "grad_out")
    if row_map is not None:
        _req(row_map, "row_map", dtype=torch.int32, dim=1)
    T = make_tables(tables)
    _lib.call("kgat_bpr_bwd_f32", ctypes.byref(T), t, users.data_ptr(), pos.data_ptr(), neg.data_ptr(),
              users.numel(), float(reg), coef.data_ptr(), grad_out.data_ptr(), dst.data_ptr(), _ld(dst),
              row_map.data_ptr() if row_map is not None else None, stream_ptr(dst.device))


def transr_fwd(emb, rel_emb, trans, heads, rels, pos, neg, reg: float):
    """(loss [1], work) for the TransR KG loss."""
    _req(emb, "emb", dim=2)
    _req(rel_emb, "rel_emb", dim=2)
    _req(trans, "trans", dim=3)
    ids = [heads, rels, pos, neg]
    for t, nm in zip(ids, ("heads", "rels", "pos", "neg")):
        _req(t, nm, dtype=torch.int64, dim=1)
    B = heads.numel()
    d, k = trans.shape[1], trans.shape[2]
    if emb.shape[1] != d or rel_emb.shape[1] != k or any(t.numel() != B for t in ids) or B == 0:
        raise ValueError("TransR shape mismatch")
    if not (trans.is_contiguous() and rel_emb.is_contiguous()):
        raise ValueError("trans / rel_emb must be contiguous")
    dev = emb.device
    loss = torch.empty(1, dtype=torch.float32, device=dev)
    work = torch.empty(int(_lib.lib().kgat_transr_work_floats(B, d, k)), dtype=torch.float32, device=dev)
    tok = _ev_begin("transr_fwd")
    _lib.call("kgat_transr_fwd_ex_f32", emb.data_ptr(), _ld(emb), rel_emb.data_ptr(), trans.data_ptr(), d, k,
              trans.shape[0], heads.data_ptr(), rels.data_ptr(), pos.data_ptr(), neg.data_ptr(), B, float(reg), loss.data_ptr(),
              work.data_ptr(), stream_ptr(dev))
    _ev_end(tok)
    return loss, work


def transr_bwd(emb, n_rel: int, k: int, heads, rels, pos, neg, work, grad_out):
    """(d_emb dense [N, d], d_rel [n_rel, k], d_trans [n_rel, d, k])."""
    dev = emb.device
    d = emb.shape[1]
    d_emb = zeros(emb.shape, dev)
    d_rel = torch.empty(n_rel, k, dtype=torch.float32, device=dev)
    d_trans = torch.empty(n_rel, d, k, dtype=torch.float32, device=dev)
    ws_n = int(_lib.lib().kgat_transr_bwd_workspace_floats(heads.numel(), d, k, n_rel))
    if ws_n < 0:
        raise ValueError("transr_bwd: bad shape")
    ws = torch.empty(ws_n, dtype=torch.float32, device=dev)
    tok = _ev_begin("transr_bwd")
    _lib.call("kgat_transr_bwd_f32", emb.data_ptr(), _ld(emb), d, k, heads.data_ptr(), rels.data_ptr(),
              pos.data_ptr(), neg.data_ptr(), heads.numel(), n_rel, work.data_ptr(), grad_out.data_ptr(),
              d_emb.data_ptr(), _ld(d_emb), d_rel.data_ptr(), d_trans.data_ptr(), ws.data_ptr(), ws.numel(),
              stream_ptr(dev))
    _ev_end(tok)
    return d_emb, d_rel, d_trans


def transr_bwd_compact(emb, n_rel: int, k: int, heads, rels, pos, neg, work, grad_out, row_map: torch.Tensor,
                       n_rows: int):
    """transr_bwd with the table gradient written compactly (kgat_transr_bwd_ex_f32): row row_map[id]
    of a zero-filled [n_rows, d] buffer per batch id (kgat_frontier_build's map).  Returns (Gc, d_rel,
    d_trans)."""
    _req(row_map, "row_map", dtype=torch.int32, dim=1)
    dev = emb.device
    d = emb.shape[1]
    Gc = zeros((max(n_rows, 1), d), dev)
    d_rel = torch.empty(n_rel, k, dtype=torch.float32, device=dev)
    d_trans = torch.empty(n_rel, d, k, dtype=torch.float32, device=dev)
    ws_n = int(_lib.lib().kgat_transr_bwd_workspace_floats(heads.numel(), d, k, n_rel))
    if ws_n < 0:
        raise ValueError("transr_bwd: bad shape")
    ws = torch.empty(ws_n, dtype=torch.float32, device=dev)
    tok = _ev_begin("transr_bwd")
    _lib.call("kgat_transr_bwd_ex_f32", emb.data_ptr(), _ld(emb), d, k, heads.data_ptr(), rels.data_ptr(),
              pos.data_ptr(), neg.data_ptr(), heads.numel(), n_rel, work.data_ptr(), grad_out.data_ptr(),
              Gc.data_ptr(), _ld(Gc), row_map.data_ptr(), d_rel.data_ptr(), d_trans.data_ptr(), ws.data_ptr(),
              ws.numel(), stream_ptr(dev))
    _ev_end(tok)
    return Gc, d_rel, d_trans


def adam_rows(p, m, v, row_map: torch.Tensor, Gc: torch.Tensor, step_size: float, beta1: float, beta2: float,
              bc2_sqrt: float, eps: float, skip: torch.Tensor | None = None) -> None:
    """Adam over the whole [N, d] table with row r's gradient Gc[row_map[r]] or 0 (kgat_adam_rows_f32)."""
    for t, nm in ((p, "param"), (m, "exp_avg"), (v, "exp_avg_sq")):
        _req(t, nm, dim=2)
        if not t.is_contiguous() or t.shape != p.shape:
            raise ValueError(f"{nm}: contiguous {tuple(p.shape)} expected")
    _req(row_map, "row_map", dtype=torch.int32, dim=1)
    _req(Gc, "Gc", dim=2)
    if row_map.numel() != p.shape[0] or Gc.shape[1] != p.shape[1]:
        raise ValueError("adam_rows: row_map must cover every row, Gc must be [rows, d]")
    tok = _ev_begin("adam_rows")
    _lib.call("kgat_adam_rows_f32", p.data_ptr(), m.data_ptr(), v.data_ptr(), p.shape[0], p.shape[1],
              row_map.data_ptr(), Gc.data_ptr(), _ld(Gc), step_size, beta1, beta2, bc2_sqrt, eps, _skip_ptr(skip),
              stream_ptr(p.device))
    _ev_end(tok)


def score_edges(plan, emb, trans, Wv, bv, Wo, bo, ln_w, ln_b, out: torch.Tensor, dropout_p: float = 0.0,
                seed: int = 0) -> None:
    """Edge scores of a plan: out[plan.out_pos[e]] (or out[e]) = logit of edge e; the fused MFMA
    scorer for d <= 128, the chunked GEMM scorer above."""
    d = emb.shape[1]
    tok = _ev_begin("edge_scores")
    if d not in (16, 32, 64, 128):  # wide embeddings: GEMM path (csrc/attention_gemm.hip)
        chunk = max(16, min(plan.n_edges, EDGE_GEMM_CHUNK))
        work = torch.empty(int(_lib.lib().kgat_edge_logits_gemm_work_floats(chunk, d)), dtype=torch.float32,
                           device=emb.device)
        _lib.call("kgat_edge_logits_gemm_f32", emb.data_ptr(), _ld(emb), emb.shape[0], trans.data_ptr(), d,
                  Wv.data_ptr(), bv.data_ptr(), Wo.data_ptr(), bo.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(),
                  plan.tails.data_ptr(), plan.weight.data_ptr(), plan.rel_perm.data_ptr(), plan.n_edges,
                  plan.seg_rel.ctypes.data, plan.seg_beg.ctypes.data, plan.seg_rel.size, float(dropout_p),
                  ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
                  plan.out_pos.data_ptr() if plan.out_pos is not None else None, out.data_ptr(), work.data_ptr(),
                  work.numel(), stream_ptr(emb.device))
    else:
        _lib.call("kgat_edge_logits_f32", emb.data_ptr(), _ld(emb), emb.shape[0], trans.data_ptr(), d,
                  Wv.data_ptr(), bv.data_ptr(), Wo.data_ptr(), bo.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(),
                  plan.tails.data_ptr(), plan.weight.data_ptr(), plan.rel_perm.data_ptr(), plan.tile_rel.data_ptr(),
                  plan.tile_beg.data_ptr(), plan.n_tiles, float(dropout_p), ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
                  plan.out_pos.data_ptr() if plan.out_pos is not None else None, out.data_ptr(),
                  stream_ptr(emb.device))
    _ev_end(tok)


def edge_logits(graph: DeviceGraph, plan, emb, trans, Wv, bv, Wo, bo, ln_w, ln_b, dropout_p: float = 0.0,
                seed: int = 0) -> torch.Tensor:
    """Per-slot (bijective plans) or per-edge attention logits."""
    for t, nm in ((emb, "emb"), (Wv, "Wv"), (Wo, "Wo")):
        _req(t, nm, dim=2)
    _req(trans, "trans", dim=3)
    d = emb.shape[1]
    if trans.shape[1:] != (d, d) or Wv.shape != (d, d) or Wo.shape != (d, d):
        raise ValueError("edge scorer needs cf_embedding_dim == kg_embedding_dim (multi_head_attention.py:13-15)")
    for t in (trans, Wv, Wo, bv, bo, ln_w, ln_b):
        if not t.is_contiguous():
            raise ValueError("edge scorer weights must be contiguous")
    n_out = graph.nnz if plan.out_pos is not None else plan.n_edges
    out = torch.empty(max(n_out, 1), dtype=torch.float32, device=emb.device)
    score_edges(plan, emb, trans, Wv, bv, Wo, bo, ln_w, ln_b, out, dropout_p, seed)
    if plan.out_pos is None:
        slot_logits = torch.empty(max(graph.nnz, 1), dtype=torch.float32, device=emb.device)
        _lib.call("kgat_slot_sum_f32", plan.slot_ptr.data_ptr(), plan.slot_order.data_ptr(), graph.nnz,
                  out.data_ptr(), slot_logits.data_ptr(), stream_ptr(emb.device))
        out = slot_logits
    return out[:graph.nnz]


LONG_THRESHOLD_SOFTMAX = 256  # kSoftmaxShort in csrc/attention.hip


def graph_long_threshold() -> int:
    from .graph import LONG_THRESHOLD
    return LONG_THRESHOLD


def row_softmax(graph: DeviceGraph, slot_logits: torch.Tensor) -> None:
    """A.val <- softmax over each row's stored entries; then A^T values follow."""
    _req(slot_logits, "slot_logits", dim=1)
    A = graph.A
    if LONG_THRESHOLD_SOFTMAX != graph_long_threshold():
        raise RuntimeError("row softmax long-row split must match the CSR plan")
    row_softmax_csr(A, slot_logits, A.val)
    graph.refresh_transpose()


def row_softmax_csr(A, slot_logits: torch.Tensor, val: torch.Tensor) -> None:
    """val <- softmax over each row's stored entries of a device CSR (graph._DeviceCSR or a shard's),
    hub rows by their fixed-length long-row plan segments (kgat_row_softmax_plan_f32)."""
    desc = A.softmax_descriptor()
    work = torch.empty(max(int(_lib.lib().kgat_row_softmax_work_floats(ctypes.byref(desc))), 1),
                       dtype=torch.float32, device=slot_logits.device)
    tok = _ev_begin("row_softmax")
    _lib.call("kgat_row_softmax_plan_f32", ctypes.byref(desc), slot_logits.data_ptr(), val.data_ptr(),
              work.data_ptr(), work.numel(), stream_ptr(slot_logits.device))
    _ev_end(tok)


def scores(tables: list[torch.Tensor], users, items) -> torch.Tensor:
    """[len(users), len(items)] fp32 dot products over the concatenated tables."""
    _req(users, "users", dtype=torch.int64, dim=1)
    _req(items, "items", dtype=torch.int64, dim=1)
    T = make_tables(tables)
    out = torch.empty(users.numel(), items.numel(), dtype=torch.float32, device=users.device)
    _lib.call("kgat_score_f32", ctypes.byref(T), users.data_ptr(), users.numel(), items.data_ptr(), items.numel(),
              out.data_ptr(), _ld(out) if out.numel() else max(1, items.numel()), stream_ptr(users.device))
    return out


def adam(p, g, m, v, step_size: float, beta1: float, beta2: float, bc2_sqrt: float, eps: float) -> None:
    for t, nm in ((p, "param"), (g, "grad"), (m, "exp_avg"), (v, "exp_avg_sq")):
        _req(t, nm)
        if not t.is_contiguous():
            raise ValueError(f"{nm} must be contiguous")
    _lib.call("kgat_adam_f32", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), step_size, beta1,
              beta2, bc2_sqrt, eps, stream_ptr(p.device))


ADAM_MAX_TENSORS = _lib.KGAT_ADAM_MAX_TENSORS  # tensors per adam_multi launch / per fused update's extra


def adam_multi(items, beta1: float, beta2: float, eps: float, skip: torch.Tensor | None = None) -> None:
    """One launch per <= 16 tensors: items = [(p, g, m, v, step_size, bc2_sqrt), ...]; ``skip``: the
    optimiser skip flag (nothing moves when it is set)."""
    tok = _ev_begin("adam_multi")
    for i in range(0, len(items), _lib.KGAT_ADAM_MAX_TENSORS):
        chunk = items[i:i + _lib.KGAT_ADAM_MAX_TENSORS]
        _lib.call("kgat_adam_multi_ex_f32", _adam_array(chunk), len(chunk), beta1, beta2, eps, _skip_ptr(skip),
                  stream_ptr(chunk[0][0].device))
    _ev_end(tok)


def _adam_array(items):
    """The kgat_adam_tensor array of adam_multi items (contiguous float32 tensors)."""
    arr = (_lib.AdamTensor * len(items))()
    for a, (p, g, m, v, step_size, bc2s) in zip(arr, items):
        for t, nm in ((p, "param"), (g, "grad"), (m, "exp_avg"), (v, "exp_avg_sq")):
            _req(t, nm)
            if not t.is_contiguous():
                raise ValueError(f"{nm} must be contiguous")
        a.p, a.g, a.m, a.v = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
        a.n, a.step_size, a.bc2_sqrt = p.numel(), step_size, bc2s
    return arr


def fill(t: torch.Tensor, value: float) -> torch.Tensor:
    _req(t, "t")
    if not t.is_contiguous():
        raise ValueError("fill needs a contiguous tensor")
    _lib.call("kgat_fill_f32", t.data_ptr(), t.numel(), float(value), stream_ptr(t.device))
    return t


def zeros(shape, device) -> torch.Tensor:
    return fill(torch.empty(shape, dtype=torch.float32, device=device), 0.0)
