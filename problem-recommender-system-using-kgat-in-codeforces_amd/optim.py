"""Fused dense Adam on the HIP path (src/model/KGAT/model.py:393-419).

Drop-in for ``torch.optim.Adam(params, lr)`` as the reference uses it:
betas (0.9, 0.999), eps 1e-8, no weight decay, ``zero_grad`` sets grads to
None and parameters whose grad is None are skipped (their state untouched).
The reference builds TWO independent instances over the same parameters
(CF lr 1e-3, KG lr 1e-4); each keeps its own exp_avg / exp_avg_sq.
"""
from __future__ import annotations

import math
import os

import torch

from . import kernels


# The small tensors' Adam beside a fused launch: on a side stream (1, the default) or after it on the
# current stream (0) -- an A/B switch (profiles/r06_small_adam_ab.md)
SMALL_ADAM_SIDE = os.environ.get("KGAT_SMALL_ADAM_SIDE", "1") != "0"


class FusedAdam:
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8):
        self.params = [p for p in params]
        self.lr = float(lr)
        self.beta1, self.beta2 = float(betas[0]), float(betas[1])
        self.eps = float(eps)
        self.state: dict[int, dict] = {}
        self._side: dict = {}  # device -> side stream of step()

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
        ready = None
        if items and runs and items[0][0].is_cuda and SMALL_ADAM_SIDE:
            ready = torch.cuda.Event()
            ready.record()  # every gradient of this step is in place (current stream)
        for launch, st, step_size, bc2s in runs:
            launch(st["exp_avg"], st["exp_avg_sq"], step_size, bc2s, self.beta1, self.beta2, self.eps, skip)
        if ready is not None:
            # the small tensors' Adam (one short launch) runs on a side stream beside the fused launch(es),
            # which hold every CU for hundreds of microseconds (issued first, so the host work of the fork
            # overlaps them); the current stream waits for it at the end
            dev = items[0][0].device
            side = self._side.get(dev)
            if side is None:
                side = self._side[dev] = torch.cuda.Stream(device=dev)
            side.wait_event(ready)
            with torch.cuda.stream(side):
                kernels.adam_multi(items, self.beta1, self.beta2, self.eps, skip)
            torch.cuda.current_stream(dev).wait_stream(side)
        elif items:
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
