"""Drop-in NFM model on the MI355X HIP path (src/model/NFM/model.py:12-154).

Same ``NFMArgs`` / ``NFMMode`` / parameter names and creation order as the
reference (so ``torch.manual_seed`` gives the same initial weights and
``state_dict`` keys match), same ``forward(pos_x, neg_x, mode=TRAIN)`` /
``forward(x, mode=PREDICT)``, ``build_optimizer(lr)`` and ``update_weights()``.
The feature batches are the reference's sparse COO tensors; they are
coalesced (an index sort on the device) and turned into CSR row pointers, then
every score, loss and gradient comes from csrc/nfm.hip.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from enum import IntEnum
from typing import Any

import numpy as np
import torch
from torch import nn

from . import _lib, kernels
from .graph import stream_ptr
from .optim import FusedAdam


@dataclass
class NFMArgs:
    user_num: int
    item_num: int
    entity_num: int
    embedding_dim: int = 64
    loss_lambda: float = 1e-5
    hidden_dim: list[int] = field(default_factory=lambda: [64, 32, 16])
    message_dropout: list[float] = field(default_factory=lambda: [0.1, 0.1, 0.1])


class NFMMode(IntEnum):
    TRAIN = 0
    PREDICT = 1


class HiddenLayer(nn.Module):
    """Parameter holder of hidden_layer.py:15-29 (Linear -> ReLU -> Dropout)."""

    def __init__(self, input_dim: int, output_dim: int, dropout: float) -> None:
        super().__init__()
        self._dropout = float(dropout)
        self._linear = nn.Linear(input_dim, output_dim)
        nn.init.xavier_uniform_(self._linear.weight)


@dataclass
class NFMBatch:
    """A feature batch already in the HIP path's layout (NFMBatcher's output): the
    COO row / column / value of every entry, rows sorted and columns ascending
    within a row, plus CSR row pointers.  ``NFM.forward`` takes it wherever the
    reference takes a sparse COO tensor; ``to_sparse_coo`` gives that tensor."""
    rows: torch.Tensor
    cols: torch.Tensor
    vals: torch.Tensor
    rowptr: torch.Tensor
    shape: tuple[int, int]

    def to_sparse_coo(self) -> torch.Tensor:
        x = torch.sparse_coo_tensor(torch.stack([self.rows, self.cols]), self.vals, self.shape)
        return x._coalesced_(True)


def _csr(x, row_offset: int = 0):
    """(rows int64, cols int64, vals fp32) of a sparse COO batch, row-sorted."""
    if isinstance(x, NFMBatch):
        return (x.rows + row_offset if row_offset else x.rows), x.cols, x.vals
    if not x.is_sparse:
        raise ValueError("NFM feature batches are sparse COO tensors (NFM/preprocess.py:290-356)")
    x = x.coalesce()
    idx = x.indices()
    rows = idx[0] + row_offset if row_offset else idx[0]
    return rows, idx[1].contiguous(), x.values().to(torch.float32).contiguous()


class _NFMLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rows, cols, vals, batch, model, V, w_lin, b_lin, W_out, *hidden):
        net = model._net(model.training)
        n_rows = 2 * batch
        rowptr = model._rowptr(rows, n_rows)
        act = torch.empty(max(1, int(_lib.lib().kgat_nfm_act_floats(ctypes.byref(net), n_rows))),
                          dtype=torch.float32, device=V.device)
        y = torch.empty(n_rows, dtype=torch.float32, device=V.device)
        dev = V.device
        _lib.call("kgat_nfm_fwd_f32", ctypes.byref(net), rowptr.data_ptr(), cols.data_ptr(), vals.data_ptr(), n_rows,
                  act.data_ptr(), y.data_ptr(), stream_ptr(dev))
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        dy = torch.empty(n_rows, dtype=torch.float32, device=dev)
        _lib.call("kgat_nfm_loss_f32", ctypes.byref(net), y.data_ptr(), batch, float(model._loss_lambda),
                  loss.data_ptr(), dy.data_ptr(), stream_ptr(dev))
        ctx.model, ctx.net, ctx.batch = model, net, batch
        ctx.keep = (rows, cols, vals, act, dy, V, w_lin, b_lin, W_out, hidden)
        return loss.view(())

    @staticmethod
    def backward(ctx, gout):
        rows, cols, vals, act, dy, V, w_lin, b_lin, W_out, hidden = ctx.keep
        net, model = ctx.net, ctx.model
        n_rows = 2 * ctx.batch
        dev = V.device
        gout = gout.reshape(1).to(torch.float32).contiguous()
        dV = kernels.zeros(V.shape, dev)
        dw = kernels.zeros(w_lin.shape, dev)
        db_lin = torch.empty_like(b_lin)
        dW_out = torch.empty_like(W_out)
        L = len(hidden) // 2
        dWs = [torch.empty_like(hidden[2 * l]) for l in range(L)]
        dbs = [torch.empty_like(hidden[2 * l + 1]) for l in range(L)]
        pw = (ctypes.c_void_p * max(1, L))(*[t.data_ptr() for t in dWs])
        pb = (ctypes.c_void_p * max(1, L))(*[t.data_ptr() for t in dbs])
        ws = torch.empty(max(1, int(_lib.lib().kgat_nfm_bwd_workspace(ctypes.byref(net), n_rows, cols.numel()))),
                         dtype=torch.float32, device=dev)
        _lib.call("kgat_nfm_bwd_f32", ctypes.byref(net), rows.data_ptr(), cols.data_ptr(), vals.data_ptr(),
                  cols.numel(), n_rows, act.data_ptr(), dy.data_ptr(), gout.data_ptr(), float(model._loss_lambda),
                  dV.data_ptr(), V.stride(0), dw.data_ptr(), db_lin.data_ptr(), pw, pb, dW_out.data_ptr(),
                  ws.data_ptr(), ws.numel(), stream_ptr(dev))
        hidden_grads = []
        for l in range(L):
            hidden_grads += [dWs[l], dbs[l]]
        ctx.keep = None
        return (None, None, None, None, None, dV, dw, db_lin, dW_out, *hidden_grads)


class NFM(nn.Module):
    def __init__(self, args: NFMArgs) -> None:
        super().__init__()
        self._user_num = args.user_num
        self._item_num = args.item_num
        self._entity_num = args.entity_num
        self._feature_num = self._user_num + self._entity_num
        self._embedding_dim = args.embedding_dim
        self._loss_lambda = args.loss_lambda
        self._hidden_dim = list(args.hidden_dim)
        self._message_dropout = list(args.message_dropout)
        self._layer_size = len(self._hidden_dim)
        if self._layer_size > _lib.KGAT_NFM_MAX_LAYERS:
            raise ValueError(f"at most {_lib.KGAT_NFM_MAX_LAYERS} hidden layers")
        # creation / init order as the reference (NFM/model.py:31-71)
        self._linear = nn.Linear(self._feature_num, 1)
        self._feature_embedding = nn.Parameter(torch.Tensor(self._feature_num, self._embedding_dim))
        self._hidden_layers = nn.ModuleList()
        dims = [self._embedding_dim, *self._hidden_dim]
        for l in range(self._layer_size):
            self._hidden_layers.append(HiddenLayer(dims[l], dims[l + 1], self._message_dropout[l]))
        self._output_layer = nn.Linear(dims[-1], 1, bias=False)
        nn.init.xavier_uniform_(self._linear.weight)
        nn.init.xavier_uniform_(self._feature_embedding)
        nn.init.xavier_uniform_(self._output_layer.weight)

    def _hidden_params(self) -> list[torch.Tensor]:
        return [t for hl in self._hidden_layers for t in (hl._linear.weight, hl._linear.bias)]

    def _net(self, training: bool) -> _lib.NFMNet:
        V = self._feature_embedding
        if V.device.type != "cuda":
            raise RuntimeError("NFM runs on the MI355X HIP path only: move the model to a GPU first")
        n = _lib.NFMNet()
        n.V, n.ld_v = V.data_ptr(), V.stride(0)
        n.w_lin, n.b_lin = self._linear.weight.data_ptr(), self._linear.bias.data_ptr()
        dims = [self._embedding_dim, *self._hidden_dim]
        for l, hl in enumerate(self._hidden_layers):
            n.W[l], n.b[l] = hl._linear.weight.data_ptr(), hl._linear.bias.data_ptr()
        for l, dv in enumerate(dims):
            n.dims[l] = dv
        n.n_layers = self._layer_size
        n.W_out = self._output_layer.weight.data_ptr()
        ps = {hl._dropout for hl in self._hidden_layers} if training else {0.0}
        if len(ps) > 1:
            raise ValueError("per-layer dropout rates must be equal on the HIP path")
        n.dropout_p = float(next(iter(ps))) if ps else 0.0
        n.seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if n.dropout_p > 0 else 0
        return n

    @staticmethod
    def _rowptr(rows: torch.Tensor, n_rows: int) -> torch.Tensor:
        rowptr = torch.empty(n_rows + 1, dtype=torch.int64, device=rows.device)
        _lib.call("kgat_coo_rowptr", rows.data_ptr(), rows.numel(), n_rows, rowptr.data_ptr(), stream_ptr(rows.device))
        return rowptr

    def _calc_score(self, feature_values: torch.Tensor) -> torch.Tensor:
        dev = self._feature_embedding.device
        if isinstance(feature_values, NFMBatch):
            rows, cols, vals = _csr(feature_values)
            rowptr = feature_values.rowptr
        else:
            rows, cols, vals = _csr(feature_values.to(dev))
            rowptr = None
        n_rows = feature_values.shape[0]
        net = self._net(self.training)
        if rowptr is None:
            rowptr = self._rowptr(rows, n_rows)
        y = torch.empty(n_rows, dtype=torch.float32, device=dev)
        with torch.no_grad():
            _lib.call("kgat_nfm_fwd_f32", ctypes.byref(net), rowptr.data_ptr(), cols.data_ptr(), vals.data_ptr(),
                      n_rows, None, y.data_ptr(), stream_ptr(dev))
        return y.squeeze()

    def _calc_loss(self, positive_feature_values: torch.Tensor, negative_feature_values: torch.Tensor) -> torch.Tensor:
        dev = self._feature_embedding.device
        B = positive_feature_values.shape[0]
        if negative_feature_values.shape[0] != B:
            raise ValueError("positive and negative batches must have the same number of rows")
        rp, cp, vp = _csr(positive_feature_values if isinstance(positive_feature_values, NFMBatch)
                          else positive_feature_values.to(dev))
        rn, cn, vn = _csr(negative_feature_values if isinstance(negative_feature_values, NFMBatch)
                          else negative_feature_values.to(dev), row_offset=B)
        rows, cols, vals = torch.cat([rp, rn]), torch.cat([cp, cn]), torch.cat([vp, vn])
        return _NFMLoss.apply(rows, cols, vals, B, self, self._feature_embedding, self._linear.weight,
                              self._linear.bias, self._output_layer.weight, *self._hidden_params())

    def build_optimizer(self, lr: float) -> None:
        self._optimizer = FusedAdam(self.parameters(), lr=lr)

    def update_weights(self) -> None:
        self._optimizer.step()
        self._optimizer.zero_grad()

    def forward(self, *args: Any, mode: NFMMode) -> torch.Tensor:
        if mode == NFMMode.TRAIN:
            return self._calc_loss(*args)
        if mode == NFMMode.PREDICT:
            return self._calc_score(*args)
        raise ValueError(f"unknown mode {mode}")


class NFMBatcher:
    """NFM batch generation (NFM/preprocess.py:150-356) with the feature rows built on the device.

    The item feature matrix is the reference's ``_get_user_and_feature_matrices``
    (preprocess.py:150-193): each item's one-hot plus the tails of the KG triplets
    whose head is that problem, duplicates summed, over entity_num columns.
    ``generate_train_batch`` draws (users, positive, negative) with the native CF
    sampler (sampler.BatchSampler, the same draws as preprocess.py:195-270) and
    returns two ``NFMBatch``; ``generate_test_batch(user_ids)`` is the users x all
    items grid of preprocess.py:309-334.  Rows come from kgat_nfm_batch_rowptr /
    kgat_nfm_batch_fill (csrc/nfm_batch.hip)."""

    def __init__(self, user_num: int, item_num: int, entity_num: int, feature_heads, feature_tails,
                 interaction_dict, device, train_batch_size: int = 1024, seed: int = 2024):
        from .sampler import BatchSampler

        self.user_num, self.item_num, self.entity_num = int(user_num), int(item_num), int(entity_num)
        self.device = torch.device(device)
        h = np.concatenate([np.arange(self.item_num, dtype=np.int64), np.asarray(feature_heads, np.int64)])
        t = np.concatenate([np.arange(self.item_num, dtype=np.int64), np.asarray(feature_tails, np.int64)])
        if h.size and (h.min() < 0 or h.max() >= self.item_num or t.min() < 0 or t.max() >= self.entity_num):
            raise IndexError("feature triplets must have problem heads < item_num and tails < entity_num")
        key = h * self.entity_num + t
        uniq, counts = np.unique(key, return_counts=True)  # coo -> csr sums duplicates
        rows, cols = uniq // self.entity_num, uniq % self.entity_num
        rowptr = np.zeros(self.item_num + 1, np.int64)
        np.cumsum(np.bincount(rows, minlength=self.item_num), out=rowptr[1:])
        self.feature_rowptr = torch.from_numpy(rowptr).to(self.device)
        self.feature_col = torch.from_numpy(cols.astype(np.int64)).to(self.device)
        self.feature_val = torch.from_numpy(counts.astype(np.float32)).to(self.device)
        self._sampler = BatchSampler(interaction_dict, self.item_num, np.zeros(0, np.int64), np.zeros(0, np.int64),
                                     np.zeros(0, np.int64), max(1, self.user_num + self.entity_num),
                                     cf_batch_size=train_batch_size, seed=seed)

    @property
    def n_features(self) -> int:
        return self.user_num + self.entity_num

    def build(self, users: torch.Tensor, items: torch.Tensor | None = None) -> NFMBatch:
        """Rows (users[r], items[r]); items None: every user of ``users`` x every item."""
        dev = self.device
        users = torch.as_tensor(users, dtype=torch.int64).to(dev).contiguous()
        if users.numel() and (int(users.min()) < 0 or int(users.max()) >= self.user_num):
            raise IndexError("user id out of range")
        if items is not None:
            items = torch.as_tensor(items, dtype=torch.int64).to(dev).contiguous()
            if items.shape != users.shape:
                raise ValueError("users and items must have the same length")
            if items.numel() and (int(items.min()) < 0 or int(items.max()) >= self.item_num):
                raise IndexError("item id out of range")
            n_rows = items.numel()
        else:
            n_rows = users.numel() * self.item_num
        lib = _lib.lib()
        rowptr = torch.empty(n_rows + 1, dtype=torch.int64, device=dev)
        work = torch.empty(max(1, int(lib.kgat_nfm_batch_work_bytes(n_rows))), dtype=torch.uint8, device=dev)
        st = stream_ptr(dev)
        ip = items.data_ptr() if items is not None else None
        _lib.call("kgat_nfm_batch_rowptr", users.data_ptr(), ip, n_rows, self.item_num, self.feature_rowptr.data_ptr(),
                  rowptr.data_ptr(), work.data_ptr(), work.numel(), st)
        nnz = int(rowptr[-1].item())
        rows = torch.empty(nnz, dtype=torch.int64, device=dev)
        cols = torch.empty(nnz, dtype=torch.int64, device=dev)
        vals = torch.empty(nnz, dtype=torch.float32, device=dev)
        _lib.call("kgat_nfm_batch_fill", users.data_ptr(), ip, n_rows, self.item_num, self.user_num,
                  self.feature_rowptr.data_ptr(), self.feature_col.data_ptr(), self.feature_val.data_ptr(),
                  rowptr.data_ptr(), rows.data_ptr(), cols.data_ptr(), vals.data_ptr(), st)
        return NFMBatch(rows, cols, vals, rowptr, (n_rows, self.n_features))

    def generate_train_batch(self) -> tuple[NFMBatch, NFMBatch]:
        """(positive, negative) feature batches (preprocess.py:284-307)."""
        users, pos, neg = self._sampler.generate_cf_batch()
        return self.build(users, pos), self.build(users, neg)

    def generate_test_batch(self, batch_user_ids) -> NFMBatch:
        """Users x all items, row u * item_num + i (preprocess.py:309-334)."""
        return self.build(torch.as_tensor(batch_user_ids, dtype=torch.int64))
