"""Row-sharded KGAT across GPUs -- SURVEY §8(e) mode 2 (the C5 configuration).

A table of 50M x 256 fp32 rows plus two Adam states does not fit one GPU, so
rank k owns a contiguous row range [lo_k, hi_k) of every node table (X0, H1,
..., HL, the side S_l) and the same rows of the attentive matrix A.  Its rows
of A are cut by source shard into CSR blocks A[k][j] (columns rebased to shard
j) and their transposes.

Forward, per layer (ring all-gather, pipelined):
    S_k = sum_j A[k][j] . X_j      X_j travels the ring k -> k+1 while rank k
                                    multiplies the block it holds
    H_k = biinter(X_k, S_k)        row-local
Backward, per layer (ring reduce-scatter, fused):
    dX_j = dXd_j + sum_k A[k][j]^T . dS_k
    the partial for owner j starts at rank j+1, gains each rank's
    A[k][j]^T . dS_k on its way round the ring and ends at j -- one fixed
    summation order (deterministic); the last layer uses the batch frontier
    (masked SpMM), as the single-GPU path does.
The BPR loss is taken over the GLOBAL batch (every rank's pairs, as data-
parallel training would): the batch rows are assembled on every rank by one
exact all-reduce (each row has exactly one owner, the others add zeros), every
rank evaluates the same loss, and each scatters the row gradients into the rows
it owns.  Aggregator weight gradients are all-reduced (each rank holds the
contribution of its rows); relation / trans gradients of the KG step are
already identical on every rank.  Adam runs on the local shard + replicas.

Transport: RCCL point-to-point (``dist.batch_isend_irecv``) and collectives
on device buffers; with a non-NCCL backend (gloo, used to run several ranks on
one test GPU) buffers are staged through host memory.  All arithmetic is the
HIP kernels of libkgat_hip.so.

Attention refresh (UPDATE_ATTENTION): rank k scores the edges of its rows; the
X0 shards travel the same ring and each arriving shard scores the local edges
whose tail it holds; logits are soft-maxed over the local CSR rows and
gathered back into the blocks and their transposes.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist
from torch import nn

from . import kernels
from . import _lib
from .graph import GraphLayout, RefreshPlan, _DeviceCSR, degree_weights, stream_ptr
from .model import Aggregator, KGATArgs, KGATMode, MultiHeadAttention
from .optim import FusedAdam


# ---------------------------------------------------------------- transport
class _Pending:
    def __init__(self, works, host_recv=None, recv=None):
        self._works, self._host_recv, self._recv = works, host_recv, recv

    def wait(self) -> None:
        for w in self._works:
            w.wait()
        if self._host_recv is not None:
            self._recv.copy_(self._host_recv)


class Comm:
    """Ring + collectives over a torch.distributed group (rank k sends to k+1, receives from k-1)."""

    def __init__(self, group=None, host_staged: bool | None = None, force: bool = False):
        """``force``: collectives run even on a world of one rank (tests: RCCL at world 1)."""
        self.force = bool(force)
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        backend = dist.get_backend(group)
        self.host = (backend != "nccl") if host_staged is None else host_staged
        to_global = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
        self.next = to_global((self.rank + 1) % self.world)
        self.prev = to_global((self.rank - 1) % self.world)

    def exchange(self, send: torch.Tensor, recv: torch.Tensor) -> _Pending:
        """Start: send -> next rank, prev rank -> recv.  wait() completes both."""
        if self.host:
            s, r = send.detach().cpu(), torch.empty(recv.shape, dtype=recv.dtype)
            ops = [dist.P2POp(dist.isend, s, self.next, self.group), dist.P2POp(dist.irecv, r, self.prev, self.group)]
            return _Pending(dist.batch_isend_irecv(ops), r, recv)
        ops = [dist.P2POp(dist.isend, send, self.next, self.group),
               dist.P2POp(dist.irecv, recv, self.prev, self.group)]
        return _Pending(dist.batch_isend_irecv(ops))

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1 and not self.force:
            return t
        if self.host:
            c = t.detach().cpu()
            dist.all_reduce(c, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, group=self.group)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape], rank order."""
        if self.world == 1 and not self.force:
            return t.unsqueeze(0)
        if self.host:
            c = t.detach().cpu().contiguous()
            parts = [torch.empty_like(c) for _ in range(self.world)]
            dist.all_gather(parts, c, group=self.group)
            return torch.stack(parts).to(t.device)
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out


# ---------------------------------------------------------------- the plan
def shard_bounds(rowptr: np.ndarray, world: int) -> np.ndarray:
    """Contiguous row ranges balancing edges + rows (a row weighs its degree plus the mean degree)."""
    n = rowptr.size - 1
    mean = rowptr[-1] / max(n, 1)
    cum = rowptr.astype(np.float64) + mean * np.arange(n + 1)
    targets = cum[-1] * np.arange(1, world) / world
    cuts = np.searchsorted(cum, targets)
    b = np.concatenate([[0], np.clip(cuts, 0, n), [n]]).astype(np.int64)
    return np.maximum.accumulate(b)


class RowShard:
    """Rank k's rows of A, cut by source shard: blocks[j] = A[k][j], blocks_t[j] = A[k][j]^T.

    ``local=False``: rowptr / col / val are the whole CSR (every rank holds the graph).
    ``local=True``: they are this rank's rows only -- rowptr [hi-lo+1] from 0, global column
    ids (graph.HashedCKG.shard: the C4/C5 sizes, where no rank holds the whole graph)."""

    def __init__(self, rowptr: np.ndarray, col: np.ndarray, val: np.ndarray, bounds: np.ndarray, rank: int, device,
                 local: bool = False):
        self.bounds = np.asarray(bounds, np.int64)
        self.rank, self.world = rank, self.bounds.size - 1
        lo, hi = int(self.bounds[rank]), int(self.bounds[rank + 1])
        self.lo, self.hi, self.n = lo, hi, hi - lo
        self.n_nodes = int(self.bounds[-1])
        self.sizes = np.diff(self.bounds)
        if local:
            if rowptr.size != self.n + 1:
                raise ValueError(f"local rowptr has {rowptr.size - 1} rows, shard {rank} has {self.n}")
            lrp = np.asarray(rowptr, np.int64) - int(rowptr[0])
            e0, e1 = int(rowptr[0]), int(rowptr[-1])
        else:
            lrp = np.asarray(rowptr[lo:hi + 1], np.int64) - int(rowptr[lo])
            e0, e1 = int(rowptr[lo]), int(rowptr[hi])
        lrow = np.repeat(np.arange(self.n, dtype=np.int32), np.diff(lrp))
        lcol = np.asarray(col[e0:e1])
        lval = np.asarray(val[e0:e1], np.float32)
        sid = (np.searchsorted(self.bounds, lcol, side="right") - 1).astype(np.int32)
        # the local CSR (rows lo..hi, global columns): attention logits are soft-maxed here, then
        # gathered into the blocks (block_pos) and their transposes (block_t_pos)
        self.local_rowptr = torch.from_numpy(np.ascontiguousarray(lrp)).to(device)
        self._lrow, self._lcol = lrow, lcol
        self.local_val = torch.from_numpy(lval.copy()).to(device)
        self.block_pos, self.block_t_pos = [], []
        self.blocks, self.blocks_t, self.nnz = [], [], []
        for j in range(self.world):
            pos = np.flatnonzero(sid == j)
            r, c, v = lrow[pos], (lcol[pos] - self.bounds[j]).astype(np.int32), lval[pos]
            nj = int(self.sizes[j])
            rp = np.zeros(self.n + 1, np.int64)
            np.cumsum(np.bincount(r, minlength=self.n), out=rp[1:])
            self.blocks.append(_DeviceCSR(rp, c, torch.from_numpy(v.copy()).to(device), device))
            order = np.lexsort((r, c))
            self.block_pos.append(torch.from_numpy(pos.astype(np.int32)).to(device))
            self.block_t_pos.append(torch.from_numpy(pos[order].astype(np.int32)).to(device))
            rpt = np.zeros(nj + 1, np.int64)
            np.cumsum(np.bincount(c, minlength=nj), out=rpt[1:])
            self.blocks_t.append(_DeviceCSR(rpt, r[order], torch.from_numpy(v[order].copy()).to(device), device))
            self.nnz.append(int(pos.size))
            del pos, r, c, v, order

    @property
    def local_keys(self) -> np.ndarray:
        """row * n_nodes + col of the local CSR entries (row-major sorted; attention refresh only)."""
        k = self.__dict__.get("_keys")
        if k is None:
            k = self._keys = self._lrow.astype(np.int64) * self.n_nodes + self._lcol.astype(np.int64)
        return k


def ring_visit(shard: RowShard, comm: Comm, X: torch.Tensor, visit) -> None:
    """Ring all-gather of the row shards X_j (k -> k+1): visit(j, X_j) runs on each shard while the
    next one is in flight."""
    G, k, d = comm.world, comm.rank, X.shape[1]
    buf = X.contiguous()
    for s in range(G):
        j = (k - s) % G
        pend = None
        if s < G - 1:
            nxt = torch.empty(int(shard.sizes[(j - 1) % G]), d, dtype=torch.float32, device=X.device)
            pend = comm.exchange(buf, nxt)
        visit(j, buf)
        if pend is not None:
            pend.wait()
            buf = nxt


def ring_spmm(shard: RowShard, comm: Comm, X: torch.Tensor) -> torch.Tensor:
    """S_k = sum_j A[k][j] . X_j with X_j arriving over the ring (all-gather pipelined with the SpMM)."""
    S = torch.empty(shard.n, X.shape[1], dtype=torch.float32, device=X.device)
    first = [True]

    def visit(j, buf):
        kernels.spmm_block(shard.blocks[j], buf, S, accumulate=not first[0])
        first[0] = False

    ring_visit(shard, comm, X, visit)
    return S


def ring_spmm_t(shard: RowShard, comm: Comm, d: int, device, block_product) -> torch.Tensor:
    """dX_k = sum_r A[r][k]^T . dS_r: a ring reduce-scatter whose partial for owner j gains
    block_product(A[k][j]^T, out) at every rank it passes."""
    G, k = comm.world, comm.rank
    pend, recv = None, None
    for s in range(G):
        j = (k - 1 - s) % G
        part = torch.empty(int(shard.sizes[j]), d, dtype=torch.float32, device=device)
        block_product(shard.blocks_t[j], part)
        if pend is not None:
            pend.wait()
            kernels.add_(part, recv)
        if s == G - 1:
            return part
        recv = torch.empty(int(shard.sizes[(j - 1) % G]), d, dtype=torch.float32, device=device)
        pend = comm.exchange(part, recv)
    raise AssertionError("unreachable")


# ---------------------------------------------------------------- batch rows
class _BatchRows:
    """The distinct rows a global batch touches: compact index <-> global id <-> local row."""

    def __init__(self, ids: np.ndarray, lo: int, hi: int, device):
        uniq, inv = np.unique(ids, return_inverse=True)
        self.n = uniq.size
        self.inv = inv.astype(np.int64)
        owned = (uniq >= lo) & (uniq < hi)
        self.local_np = np.where(owned, uniq - lo, -1).astype(np.int32)
        self.local = torch.from_numpy(self.local_np).to(device)          # compact -> local row or -1
        self.frontier_np = self.local_np[owned]                           # owned local rows, compact order
        self.n_frontier = int(self.frontier_np.size)
        # never empty: a -1 row is padding every kernel reads as zero and writes nowhere
        fr = self.frontier_np if self.n_frontier else np.full(1, -1, np.int32)
        self.frontier = torch.from_numpy(fr.copy()).to(device)
        pos = np.full(self.n, -1, np.int32)
        pos[owned] = np.arange(int(owned.sum()), dtype=np.int32)
        self.pos = torch.from_numpy(pos).to(device)                       # compact -> frontier position or -1

    def gather(self, tables: list[torch.Tensor], comm: Comm) -> list[torch.Tensor]:
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


class _ShardedCFLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cu, cp, cn, cfg, X0, *ws):
        shard, comm, drops, seeds, reg, rows = cfg
        tables, sides, states = [X0], [], []
        x = X0
        for l in range(len(drops)):
            W1, b1, W2, b2 = ws[4 * l: 4 * l + 4]
            s = ring_spmm(shard, comm, x)
            st = kernels.make_state(x.shape[0], W1.shape[1], W1.shape[0], x.device)
            x = kernels.biinter_fwd(x, s, W1, b1, W2, b2, drops[l], seeds[l], state=st)
            sides.append(s)
            states.append(st)
            tables.append(x)
        Tc = rows.gather(tables, comm)
        loss, coef = kernels.bpr_fwd(Tc, cu, cp, cn, reg)
        ctx.cfg, ctx.saved = cfg, (tables, sides, states, Tc, coef, ws)
        ctx.ids = (cu, cp, cn)
        return loss.view(())

    @staticmethod
    def backward(ctx, gout):
        shard, comm, drops, seeds, reg, rows = ctx.cfg
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

        # ---- last layer on the owned batch frontier
        l = L - 1
        dHc = kernels.zeros((rows.frontier.numel(), tables[L].shape[1]), dev)
        kernels.bpr_bwd(Tc, L, cu, cp, cn, reg, coef, gout, dHc, row_map=rows.pos)
        dXdc, dSc, *g = kernels.biinter_bwd(tables[l], sides[l], dHc, *ws[4 * l: 4 * l + 4], drops[l], seeds[l],
                                            rows=rows.frontier, **saved(l))
        reduce_w(l, g)
        node_map = torch.full((shard.n,), -1, dtype=torch.int32, device=dev)
        if rows.n_frontier:
            node_map[rows.frontier.long()] = torch.arange(rows.n_frontier, dtype=torch.int32, device=dev)
        dX = ring_spmm_t(shard, comm, tables[l].shape[1], dev,
                         lambda blk, out: kernels.spmm_block_masked(blk, node_map, dSc, out))
        kernels.scatter_rows(dX, rows.frontier, dXdc, accumulate=True)
        kernels.bpr_bwd(Tc, l, cu, cp, cn, reg, coef, gout, dX, row_map=rows.local)
        # ---- remaining layers densely
        for l in range(L - 2, -1, -1):
            W1, b1, W2, b2 = ws[4 * l: 4 * l + 4]
            dXd, dS, *g = kernels.biinter_bwd(tables[l], sides[l], dX, W1, b1, W2, b2, drops[l], seeds[l], **saved(l))
            reduce_w(l, g)
            ring = ring_spmm_t(shard, comm, tables[l].shape[1], dev,
                               lambda blk, out, dS=dS: kernels.spmm_block(blk, dS, out, transpose=True))
            kernels.add_(dXd, ring)
            kernels.bpr_bwd(Tc, l, cu, cp, cn, reg, coef, gout, dXd, row_map=rows.local)
            dX = dXd
        ctx.saved = None
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

    Same modes as KGAT (model.py:421-431) for TRAIN_CF, TRAIN_KG and PREDICT; each
    rank passes ITS OWN batch and the loss is the mean over the global batch.
    """

    def __init__(self, args: KGATArgs, layout: GraphLayout | None, comm: Comm, device,
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
        self.to(device)

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
        with torch.no_grad():
            x = self._user_entity_embedding_shard.detach()
            tables = [x]
            for l, agg in enumerate(self._aggregator_layers):
                s = ring_spmm(self.shard, self.comm, x)
                x = kernels.biinter_fwd(x, s, *[w.detach() for w in agg.weights()], drops[l], seeds[l])
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
        cfg = (self.shard, self.comm, drops, seeds, float(self._regularization_params[0]), rows)
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
        """Per source shard j: a scoring plan over this rank's edges whose tail lies in shard j
        (tails rebased into X_j), logits landing by local edge id; slot sums onto the local CSR."""
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
        sid = np.searchsorted(sh.bounds, tl, side="right") - 1
        plans = []
        for j in range(sh.world):
            m = sid == j
            plans.append(RefreshPlan.for_edges(tl[m] - sh.bounds[j], rl[m], wl[m], eid[m], dev)
                         if m.any() else None)
        so = np.argsort(slot, kind="stable")
        slot_order = torch.from_numpy(so.astype(np.int32)).to(dev)
        slot_ptr = torch.from_numpy(np.searchsorted(slot[so], np.arange(sh.local_keys.size + 1)).astype(np.int64)).to(dev)
        plan = (plans, slot_ptr, slot_order, int(hl.size))
        self._att_plan = (key, plan)
        return plan

    @torch.no_grad()
    def _update_attention(self, heads, relations, tails, relation_indices) -> None:
        """UPDATE_ATTENTION (model.py:318-366) on this rank's rows: X0 shards pass on the ring, each
        scores the local edges whose tail it holds; softmax over the local rows; blocks refreshed."""
        h, r, t = (torch.as_tensor(x).cpu().numpy().astype(np.int64) for x in (heads, relations, tails))
        plans, slot_ptr, slot_order, n_edges = self._refresh_plan(h, r, t)
        sh, dev = self.shard, self._user_entity_embedding_shard.device
        mha = self._multi_head_attention
        p = mha.dropout if self.training else 0.0
        self._step += 1
        seed = (self._step * 0x632BE5AB + 31 * self.comm.rank + 1) & ((1 << 62) - 1) if p > 0 else 0
        W = [x.detach().contiguous() for x in (self._trans_matrix, mha._value_weight.weight, mha._value_weight.bias,
                                                mha._output.weight, mha._output.bias, mha._layer_norm.weight,
                                                mha._layer_norm.bias)]
        logits = torch.empty(max(n_edges, 1), dtype=torch.float32, device=dev)

        def visit(j, buf):
            if plans[j] is not None:
                kernels.score_edges(plans[j], buf, *W, logits, p, seed)

        ring_visit(sh, self.comm, self._user_entity_embedding_shard.detach(), visit)
        nnz = sh.local_keys.size
        slot_logits = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
        st = stream_ptr(dev)
        _lib.call("kgat_slot_sum_f32", slot_ptr.data_ptr(), slot_order.data_ptr(), nnz, logits.data_ptr(),
                  slot_logits.data_ptr(), st)
        _lib.call("kgat_row_softmax_f32", sh.local_rowptr.data_ptr(), sh.n, slot_logits.data_ptr(),
                  sh.local_val.data_ptr(), st)
        for j in range(sh.world):
            for blk, pos in ((sh.blocks[j], sh.block_pos[j]), (sh.blocks_t[j], sh.block_t_pos[j])):
                if pos.numel():
                    _lib.call("kgat_gather_f32", sh.local_val.data_ptr(), pos.data_ptr(), pos.numel(),
                              blk.val.data_ptr(), st)

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

    def update_cf_weights(self) -> None:
        self._cf_optimizer.step()
        self._cf_optimizer.zero_grad()

    def update_kg_weights(self) -> None:
        self._kg_optimizer.step()
        self._kg_optimizer.zero_grad()

    def forward(self, *args, mode: KGATMode):
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
