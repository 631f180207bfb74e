"""Data-parallel KGAT replicas: one process per GPU, gradients all-reduced over RCCL.

SURVEY §8(e)(1): every CF step already propagates the whole graph for its own
256-pair batch (model.py:188), so G GPUs run G independent steps on replicas
of the model and graph (global batch 256*G) and average their gradients once
per step.  There is no other data-path collective.  Bucketing follows xGMI's
shape: the [N, d] table gradient is one large all-reduce on its own; the many
small aggregator / relation / trans gradients are coalesced into one flat
bucket so they cost a single ring instead of one launch each.

``ShardedGradSync`` is the bandwidth-lean form used by bench.py: the big
row-major gradients (the [N, d] table) are reduce-scattered by row blocks
instead of all-reduced, every rank runs Adam on the rows it owns only (1/G of
the optimizer traffic, 1/G of its state), and the updated rows are
all-gathered back -- the same bytes on the wire as one all-reduce, with the
dense Adam pass cut G-fold.  Per element the arithmetic is the all-reduce
path's (mean gradient, same Adam), so replicas stay identical.

With ``replicate_table=True`` the table is not sharded at all: when the CF
backward's layer-0 hop set is small (the hop chain, model._CFLoss), the
replicas all-gather their compact hop-set terms (row list, dS rows, direct
dX rows -- ~2*|hop|*d floats instead of N*d), merge them in rank order
(kgat_rows_union / kgat_rows_merge_f32) and every rank computes the mean table
gradient A^T . mean(dS) + mean(dXd) itself with the masked product, then runs
the full Adam; no reduce-scatter, no all-gather of the 256 MB table.  Every
rank computes the same bits from the same gathered data, so the replicas stay
identical; against the all-reduce path only the summation order differs.
(If any rank's hop set is dense, that step all-reduces the dense gradient.)

Works with any torch.distributed backend: ``nccl`` (= RCCL on ROCm) on the
GPU box, ``gloo`` for the CPU tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

SMALL_BUCKET_BYTES = 32 << 20


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def broadcast_parameters(module: torch.nn.Module, src: int = 0) -> None:
    """Make every replica start from rank ``src``'s dense parameters."""
    if world() == 1:
        return
    for p in module.parameters():
        if not p.is_sparse:
            dist.broadcast(p.data, src)


def allreduce_gradients(params, average: bool = True) -> None:
    """Average ``p.grad`` over all ranks (params whose grad is None are skipped on every rank:
    the set must agree across ranks, which it does -- it depends only on the mode)."""
    n = world()
    if n == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    big = [g for g in grads if g.numel() * g.element_size() > SMALL_BUCKET_BYTES]
    small = [g for g in grads if g.numel() * g.element_size() <= SMALL_BUCKET_BYTES]
    for g in big:
        dist.all_reduce(g)
        if average:
            g.div_(n)
    if small:
        flat = torch.cat([g.reshape(-1) for g in small])
        dist.all_reduce(flat)
        if average:
            flat.div_(n)
        off = 0
        for g in small:
            k = g.numel()
            g.copy_(flat[off:off + k].view_as(g))
            off += k


def _rank() -> int:
    return dist.get_rank() if world() > 1 else 0


def _is_nccl() -> bool:
    return dist.get_backend() == "nccl"


class ShardedGradSync:
    """Reduce-scatter / own-rows Adam / all-gather for the big gradients (ZeRO-1 on rows).

    ``reduce()`` after ``loss.backward()``: every big gradient [R, ...] is split into G
    row blocks of s = R // G rows; rank k receives the mean of block k (in place,
    RCCL reduce-scatter) and the R - G*s tail rows are all-reduced.  Small gradients
    go through one flat all-reduce as in allreduce_gradients.  Returns the row
    ranges for ``FusedAdam.step(row_ranges=...)`` (own block + tail).  ``gather()``
    after the optimizer step all-gathers the owned blocks of the parameters."""

    def __init__(self, params, big_bytes: int = SMALL_BUCKET_BYTES, replicate_table: bool = False,
                 force: bool = False, pipeline: bool = False):
        """``force``: run the collectives even on a world of one rank (tests: RCCL at world 1).
        ``pipeline`` (with attach, sharded mode): the table's owned-block Adam and the broadcast of the
        updated block run inside the backward, block by block (see _owner_step)."""
        self.force = bool(force)
        self.pipeline = bool(pipeline)
        self._model = None
        self._bcast: list = []   # this step's block broadcasts (work handles), waited by gather()
        self._stepped = set()    # main blocks whose owner step + broadcast were issued this step
        self._side = None
        self.params = list(params)
        self.big_bytes = int(big_bytes)
        self.replicate_table = bool(replicate_table)
        self.replicated = False  # set by attach() on more than one rank with replicate_table
        self._done = None  # the table gradient already averaged by table_grad_hop / table_grad_dense
        self.stats: dict[str, int] = {}  # steps per table-exchange path ("hop", "dense")
        self._big: list[tuple[torch.Tensor, int, int]] = []
        self._table = None
        self.bounds: list[tuple[int, int]] = []
        self._early = None  # (gradient tensor, [work handles]) of the hooked table gradient
        self._announced = None  # this step's early (flag, hop count) all-gather: (device, pinned host, event)
        self.discarded = 0  # announcements dropped because their forward's backward never ran

    def attach(self, model) -> "ShardedGradSync":
        """Overlap the table gradient's exchange with its computation: the CF backward then
        computes the table's A^T . dS in the G row blocks of this rank layout (+ the tail)
        and calls ``block_ready`` after each, which starts block k's reduction to rank k
        (RCCL, async) while block k+1 is computed.  No-op on one rank."""
        n = world()
        if n == 1 and not self.force:
            return self
        table = model._user_entity_embedding.weight
        rows = table.shape[0]
        s = rows // n
        if s == 0:
            return self
        self._table = table
        self.bounds = [(k * s, (k + 1) * s) for k in range(n)] + ([(s * n, rows)] if s * n < rows else [])
        self.replicated = self.replicate_table
        self._model = model
        model._table_grad_hook = self
        return self

    # ---- replicate_table mode: the mean table gradient computed on every rank from gathered hop sets

    @staticmethod
    def _all_gather(t: torch.Tensor) -> torch.Tensor:
        """[G * t.numel()] (rank order) of a contiguous tensor, flattened."""
        n = world()
        flat = t.reshape(-1)
        if _is_nccl():
            out = torch.empty(n * flat.numel(), dtype=flat.dtype, device=flat.device)
            dist.all_gather_into_tensor(out, flat)
            return out
        parts = [torch.empty_like(flat) for _ in range(n)]
        dist.all_gather(parts, flat)
        return torch.cat(parts)

    def _gather_info(self, sparse: bool, count: torch.Tensor | None, dev):
        """[G, 2] int32 in rank order: each rank's layer-0 hop count (-1 for a rank whose backward is
        dense) and its count of discarded announcements (compared across ranks by _split_info)."""
        info = torch.full((2,), self.discarded, dtype=torch.int32, device=dev)
        if sparse:
            info[:1].copy_(count.reshape(1))
        else:
            info[:1].fill_(-1)
        return self._all_gather(info).view(-1, 2)

    @staticmethod
    def _split_info(both: torch.Tensor, host: list[int]) -> tuple[torch.Tensor, list[int]]:
        """(device [G] hop counts, host counts) of a _gather_info result; raises when the ranks dropped
        different numbers of announced forwards (their all-gathers would pair up different steps)."""
        counts, dropped = host[0::2], host[1::2]
        if len(set(dropped)) > 1:
            raise RuntimeError(f"ShardedGradSync: the ranks discarded different numbers of announced TRAIN_CF "
                               f"forwards (no backward ran): {dropped} -- every rank must run the same steps")
        return both[:, 0].contiguous(), counts

    def announce(self, sparse: bool, count: torch.Tensor | None) -> None:
        """All-gather this step's (hop flag, layer-0 hop count) early -- from the forward, when the
        hop set is known before the propagation (model._early_first_hop) -- and start copying the
        result to the host; _agree then reads it without stalling the GPU queue."""
        # A grad-enabled TRAIN_CF forward whose backward never ran (a loss only logged) left its
        # announcement open.  Every rank runs the same program, so every rank dropped the same
        # forward and made the same all-gather: the stale announcement is simply discarded.  That
        # forward's own backward cannot run later -- model._mark_batch marked its token stale.  That is
        # only safe while the ranks dropped the same forwards; the count is compared across ranks at the
        # next exchange (_agree), so diverging control flow raises instead of pairing up other steps'
        # all-gathers.
        if self._announced is not None:
            self.discarded += 1
        self._announced = None
        both = self._gather_info(sparse, count, count.device)
        host = torch.empty(tuple(both.shape), dtype=torch.int32, pin_memory=True)
        host.copy_(both, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._announced = (both, host, ev)

    def exchange_cap(self) -> int | None:
        """Rows every rank sends in this step's hop-set all-gather (the largest hop count), once the
        counts were announced and every rank's backward is sparse; else None."""
        ann = self._announced
        if ann is None:
            return None
        ann[2].synchronize()
        counts = ann[1].reshape(-1).tolist()[0::2]
        return max(1, max(counts)) if all(c >= 0 for c in counts) else None

    def _agree(self, sparse: bool, count: torch.Tensor | None, dev) -> tuple[torch.Tensor, list[int], bool]:
        """All-gather every rank's hop count (-1: dense): (device [G] counts, host counts, all sparse).
        Announced early (the usual 2-layer case): the copy finished long ago, no stall; otherwise
        the step's one host synchronisation."""
        ann, self._announced = self._announced, None
        if ann is not None:
            both, host_t, ev = ann
            ev.synchronize()
            host = host_t.reshape(-1).tolist()
        else:
            both = self._gather_info(sparse, count, dev)
            host = both.reshape(-1).cpu().tolist()  # the gather sizes
        counts_dev, counts = self._split_info(both, host)
        return counts_dev, counts, all(c >= 0 for c in counts)

    def table_grad_hop(self, graph, hmap, hrows, hcount, dSc, dXdc, rank_words, deferral=None, packed=None):
        """The mean table gradient from this rank's compact layer-0 hop-set terms (model._CFLoss):
        hop rows (ascending, hcount of them), dS and direct dX rows in hop order.  With a
        ``deferral`` (model._TableUpdate) that accepts it, the merged terms are handed over and
        the product runs later, fused with the table's Adam step: returns None.  ``packed``: the
        [exchange_cap(), 2d] buffer dSc | dXdc are the halves of (sent as it is, no copies)."""
        from . import kernels

        n = world()
        d = dSc.shape[1]
        both, counts, all_sparse = self._agree(True, hcount, dSc.device)
        if all_sparse:
            # every rank sends [cap] rows, cap = the largest count; rows past a rank's own count are
            # never read (the union / merge kernels stop at each list's count)
            cap = max(1, max(counts))
            if packed is not None and packed.shape[0] == cap:
                pack = packed
            else:
                k = min(cap, dSc.shape[0])
                pack = torch.empty(cap, 2 * d, dtype=torch.float32, device=dSc.device)
                pack[:k, :d].copy_(dSc[:k])
                pack[:k, d:].copy_(dXdc[:k])
            if hrows.numel() >= cap:
                hl = hrows[:cap]
            else:
                hl = torch.empty(cap, dtype=hrows.dtype, device=hrows.device)
                hl[:hrows.numel()].copy_(hrows)
            lists = self._all_gather(hl)
            vals = self._all_gather(pack).view(n * cap, 2 * d)
            cnt = both
            urows, umap, ucount, urank = kernels.rows_union(graph, lists, cnt, cap)
            merged = kernels.rows_merge(lists, cnt, cap, vals, urows, ucount, min(graph.n_nodes, n * cap), 1.0 / n)
            if deferral is not None and deferral.defer(graph, umap, merged[:, :d], merged[:, d:], urank):
                self._done = None
                self.stats["hop"] = self.stats.get("hop", 0) + 1
                return None
            dX = kernels.spmm_masked(graph, umap, merged[:, :d], Yc_init=merged[:, d:], transpose=True,
                                     src_rank=urank)
        else:  # some rank's hop set is dense this step: every rank all-reduces its dense gradient
            dX = kernels.spmm_masked(graph, hmap, dSc, Yc_init=dXdc, transpose=True, src_rank=rank_words)
            dist.all_reduce(dX)
            dX.div_(n)
        self._done = dX
        key = "hop" if all_sparse else "dense"
        self.stats[key] = self.stats.get(key, 0) + 1
        return dX

    def table_grad_dense(self, graph, dS, dXd) -> torch.Tensor:
        """The dense-backward counterpart of table_grad_hop: dXd += A^T . dS, all-reduced, mean."""
        from . import kernels

        n = world()
        self._agree(False, None, dS.device)
        kernels.spmm(graph, dS, out=dXd, transpose=True, accumulate=True)
        dist.all_reduce(dXd)
        dXd.div_(n)
        self._done = dXd
        self.stats["dense"] = self.stats.get("dense", 0) + 1
        return dXd

    def block_ready(self, k: int, grad: torch.Tensor) -> None:
        n = world()
        if self._early is None or self._early[0] is not grad:
            self._early = (grad, [])
            self._bcast, self._stepped = [], set()
            self._advanced = []  # this step's owner-block optimiser counters advanced by _owner_step
        r0, r1 = self.bounds[k]
        view = grad[r0:r1]
        if k < n and _is_nccl():
            self._early[1].append(dist.reduce(view, dst=k, async_op=True))
        else:  # the tail rows (every rank steps them), and gloo (no CUDA reduce): all-reduce
            self._early[1].append(dist.all_reduce(view, async_op=True))
        if self.pipeline and 1 <= k <= n:
            # block k-1's owner step + broadcast, issued behind block k's reduce (the same collective order
            # on every rank); it runs while the next blocks are computed
            self._owner_step(k - 1, self._early)

    def _side_stream(self, dev) -> torch.cuda.Stream:
        if self._side is None:
            self._side = torch.cuda.Stream(device=dev)
        return self._side

    def _owner_step(self, j: int, early) -> None:
        """Pipelined sharded exchange (``pipeline``): the owner of main block j (rank j) takes its Adam step on
        the block as soon as the block's reduce lands -- on a side stream, behind that reduce only -- and
        broadcasts the updated rows; every other rank receives them into its replica.  Block j's wire time
        then overlaps blocks j+1.. of the backward product instead of following the whole update (the
        all-gather of gather()).  Per element: the same mean (the reduced sum / G) and the same Adam step with
        the owned block's own state -- the bits of the reduce-scatter / owned-row Adam / all-gather path."""
        n = world()
        rank = _rank()
        grad = early[0]
        p = self._table
        r0, r1 = self.bounds[j]
        self._stepped.add(j)
        if rank == j:
            model = self._model
            opt = model._cf_optimizer
            side = self._side_stream(grad.device)
            with torch.cuda.stream(side):
                early[1][j].wait()  # the side stream waits for the reduce; the compute stream does not
                gv = grad[r0:r1]
                gv.div_(n)
                from . import kernels
                st, step_size, bc2s = opt._advance((id(p), r0, r1), p.data[r0:r1])
                self._advanced.append((opt, (id(p), r0, r1)))
                kernels.adam_multi([(p.data[r0:r1], gv, st["exp_avg"], st["exp_avg_sq"], step_size, bc2s)],
                                   opt.beta1, opt.beta2, opt.eps, model._ids.skip_flag())
                self._bcast.append(dist.broadcast(p.data[r0:r1], src=j, async_op=True))
            grad.record_stream(side)
        else:
            self._bcast.append(dist.broadcast(p.data[r0:r1], src=j, async_op=True))

    def abandon_step(self) -> None:
        """The step was abandoned before its update (KGAT._raise_or_abandon: an earlier step's device-side
        id error surfaced).  The pipelined owner step already took its block's Adam step inside the backward
        -- a no-op on p / m / v under the device skip flag, but its step counter advanced; it is taken back,
        so every block's bias correction stays the eager path's (which advances nothing)."""
        for opt, key in getattr(self, "_advanced", []):
            st = opt.state.get(key)
            if st is not None and st["step"] > 0:
                st["step"] -= 1
        self._advanced = []

    def reduce(self) -> dict | None:
        n = world()
        self._big = []
        if n == 1 and not self.force:
            return None
        rank = _rank()
        ranges: dict = {}
        small = []
        early, self._early = self._early, None
        done, self._done = self._done, None
        for p in self.params:
            if early is not None and p is self._table and not self.replicated:
                # the attached backward left the table gradient to this exchange (model._CFLoss returns none
                # to autograd: its blocks were already in flight)
                if p.grad is not None:
                    raise RuntimeError("ShardedGradSync: another gradient reached the table after its exchange "
                                       "started (backward a second loss before reduce())")
                p.grad = early[0]
            g = p.grad
            if g is None:
                continue
            if self.replicated and p is self._table and done is not None:
                if g.data_ptr() != done.data_ptr():  # autograd kept a copy of the averaged gradient
                    g.copy_(done)
                continue  # already the mean on every rank: full Adam, nothing to gather
            if self.replicate_table and g.numel() * g.element_size() > self.big_bytes:
                dist.all_reduce(g)  # replicated mode shards nothing
                g.div_(n)
                continue
            if early is not None and p is self._table and len(early[1]) == len(self.bounds):
                s = self.bounds[0][1]
                main = s * n
                if self.pipeline:
                    for j in range(n):
                        if j not in self._stepped:
                            self._owner_step(j, early)
                    rr = []
                    if main < g.shape[0]:  # the tail rows: all-reduced, every rank steps them
                        early[1][n].wait()
                        g[main:].div_(n)
                        rr.append((main, g.shape[0]))
                    ranges[id(p)] = rr  # the owned block was stepped by _owner_step
                    continue
                for w in early[1]:
                    w.wait()
                g[rank * s:(rank + 1) * s].div_(n)
                rr = [(rank * s, (rank + 1) * s)]
                if main < g.shape[0]:
                    g[main:].div_(n)
                    rr.append((main, g.shape[0]))
                ranges[id(p)] = rr
                self._big.append((p, s, main))
                continue
            if g.dim() >= 1 and g.shape[0] >= n and g.numel() * g.element_size() > self.big_bytes \
                    and g.is_contiguous() and p.data.is_contiguous():
                rows = g.shape[0]
                s = rows // n
                main = s * n
                own = g[rank * s:(rank + 1) * s]
                if _is_nccl():
                    dist.reduce_scatter_tensor(own, g[:main])  # in place: recv = send + rank * s rows
                else:  # gloo has no reduce-scatter: the same sums, all ranks
                    dist.all_reduce(g[:main])
                own.div_(n)
                rr = [(rank * s, (rank + 1) * s)]
                if main < rows:
                    tail = g[main:]
                    dist.all_reduce(tail)
                    tail.div_(n)
                    rr.append((main, rows))
                ranges[id(p)] = rr
                self._big.append((p, s, main))
            else:
                small.append(p)
        if small:
            # one flat bucket; the parameters' gradients become views of it (no copy-back kernels)
            flat = torch.cat([p.grad.reshape(-1) for p in small])
            dist.all_reduce(flat)
            flat.div_(n)
            off = 0
            for p in small:
                k = p.grad.numel()
                p.grad = flat[off:off + k].view_as(p.grad)
                off += k
        return ranges

    @torch.no_grad()
    def gather(self) -> None:
        n = world()
        if n == 1 and not self.force:
            return
        bc, self._bcast, self._stepped = self._bcast, [], set()
        # the step is complete (stepped, or abandoned before this call): its owner-block counters may no
        # longer be taken back by a later abandon_step
        self._advanced = []
        for w in bc:  # the pipelined blocks' broadcasts: the current stream waits for the last of them
            w.wait()
        rank = _rank()
        for p, s, main in self._big:
            full = p.data[:main]
            own = full[rank * s:(rank + 1) * s]
            if _is_nccl():
                dist.all_gather_into_tensor(full, own)  # in place: send = recv + rank * s rows
            else:
                parts = list(full.split(s))
                dist.all_gather(parts, own.clone())
                # gloo fills the views of `full` in place
        self._big = []
