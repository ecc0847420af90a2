"""``nn.Linear`` whose bias gradient is a native deterministic column sum.

Forward and the two GEMMs of the backward are unchanged (hipBLASLt).  The bias gradient
``g.sum(0)`` runs csrc/linear.hip (two launches, fixed summation order) instead of
PyTorch-ROCm's multi-block ``reduce_kernel``, which returned wrong bias gradients for some
DistilBERT layers when replayed inside a captured hipGraph (tools/diag_bert_graph_vs_eager.py)
and cost ~18 µs per call.  Same parameters / ``state_dict`` as ``nn.Linear``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ext

__all__ = ["Linear"]


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        n, k = weight.shape
        g2 = g.reshape(-1, n)
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = (g2 @ weight).view(x.shape)
        if ctx.needs_input_grad[1]:
            dw = g2.t() @ x.reshape(-1, k)
        if ctx.needs_input_grad[2]:
            db = torch.empty(n, device=g.device, dtype=g.dtype)
            ext().colsum(g2, db)
        return dx, dw, db


class Linear(nn.Linear):
    """Drop-in ``nn.Linear`` (device fp32 with bias and out_features % 4 == 0 -> native bias grad)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if (x.is_cuda and self.bias is not None and x.dtype == torch.float32 and self.weight.dtype == torch.float32
                and self.out_features % 4 == 0 and torch.is_grad_enabled()):
            return _LinearFn.apply(x, self.weight, self.bias)
        return super().forward(x)
