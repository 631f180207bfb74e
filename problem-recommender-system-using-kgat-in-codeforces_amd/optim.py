"""Fused dense Adam on the HIP path (src/model/KGAT/model.py:393-419).

Drop-in for ``torch.optim.Adam(params, lr)`` as the reference uses it:
betas (0.9, 0.999), eps 1e-8, no weight decay, ``zero_grad`` sets grads to
None and parameters whose grad is None are skipped (their state untouched).
The reference builds TWO independent instances over the same parameters
(CF lr 1e-3, KG lr 1e-4); each keeps its own exp_avg / exp_avg_sq.
"""
from __future__ import annotations

import math

import torch

from . import kernels


class FusedAdam:
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8):
        self.params = [p for p in params]
        self.lr = float(lr)
        self.beta1, self.beta2 = float(betas[0]), float(betas[1])
        self.eps = float(eps)
        self.state: dict[int, dict] = {}

    def _advance(self, key, like: torch.Tensor) -> tuple[dict, float, float]:
        """Count one more step for state ``key`` (created zeroed like ``like``): (state, step_size, bc2_sqrt)."""
        st = self.state.get(key)
        if st is None:
            st = {"step": 0, "exp_avg": kernels.zeros(like.shape, like.device),
                  "exp_avg_sq": kernels.zeros(like.shape, like.device)}
            self.state[key] = st
        st["step"] += 1
        t = st["step"]
        return st, self.lr / (1.0 - self.beta1 ** t), math.sqrt(1.0 - self.beta2 ** t)

    @torch.no_grad()
    def step(self, row_ranges: dict | None = None, fused: dict | None = None,
             skip: torch.Tensor | None = None) -> None:
        """Every parameter with a gradient in one kgat_adam_multi_f32 launch (per 16 tensors).

        ``row_ranges`` {id(param): [(r0, r1), ...]} restricts a parameter's update to those
        row ranges, each with its own optimizer state (replicas.ShardedGradSync: every rank
        steps only the table rows it owns; the arithmetic per element is unchanged).

        ``fused`` {id(param): launch} steps a parameter whose gradient was never materialised
        (grad None): ``launch(exp_avg, exp_avg_sq, step_size, bc2_sqrt, beta1, beta2, eps)``
        runs the kernel that computes the gradient and applies this step to it
        (model._TableUpdate: the table's layer-0 A^T product fused with its Adam).

        ``skip``: a device int32 flag (the model's device-side id check); when it is set as the
        kernels run, no parameter or moment moves (the step counters still advance)."""
        items = []
        runs = []
        for p in self.params:
            launch = fused.get(id(p)) if fused else None
            if launch is not None:
                if p.grad is not None:
                    # the fused kernel computes the gradient itself and never reads .grad: a gradient
                    # already there would be dropped without a trace
                    raise RuntimeError("FusedAdam: a parameter stepped by a fused launch also has a .grad "
                                       "(materialise the deferred gradient into it first)")
                st, step_size, bc2s = self._advance(id(p), p.data)
                runs.append((launch, st, step_size, bc2s))
                continue
            g = p.grad
            if g is None:
                continue
            if p.is_sparse or g.is_sparse:
                raise RuntimeError("FusedAdam: sparse parameters/gradients are not supported")
            g = g.contiguous()
            ranges = row_ranges.get(id(p)) if row_ranges else None
            views = [(id(p), p.data, g)] if ranges is None else \
                [((id(p), r0, r1), p.data[r0:r1], g[r0:r1]) for r0, r1 in ranges if r1 > r0]
            for key, pv, gv in views:
                st, step_size, bc2s = self._advance(key, pv)
                items.append((pv, gv, st["exp_avg"], st["exp_avg_sq"], step_size, bc2s))
        # the other tensors' Adam rides in the last fused launch pair's fix-up launch when it can take them
        # (_TableUpdate: kgat_spmm_csr_masked_adam_multi_f32, one launch fewer per CF step); otherwise it follows
        # the fused launch(es) on the same stream -- beside them on a side stream (round 5) it waited ~120 us
        # for CU slots and its join cost the C2 step 15-17 us (profiles/r06_small_adam_ab.md)
        carry = bool(items) and bool(runs) and getattr(runs[-1][0], "takes_extra", False) \
            and len(items) <= kernels.ADAM_MAX_TENSORS
        for k, (launch, st, step_size, bc2s) in enumerate(runs):
            if carry and k == len(runs) - 1:
                launch(st["exp_avg"], st["exp_avg_sq"], step_size, bc2s, self.beta1, self.beta2, self.eps, skip,
                       extra=items)
            else:
                launch(st["exp_avg"], st["exp_avg_sq"], step_size, bc2s, self.beta1, self.beta2, self.eps, skip)
        if items and not carry:
            kernels.adam_multi(items, self.beta1, self.beta2, self.eps, skip)

    def zero_grad(self, set_to_none: bool = True) -> None:
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                kernels.fill(p.grad, 0.0)

    def state_dict(self) -> dict:
        return {"lr": self.lr, "betas": (self.beta1, self.beta2), "eps": self.eps,
                "state": {i: dict(self.state[id(p)]) for i, p in enumerate(self.params) if id(p) in self.state}}
