"""``nn.Linear`` whose bias gradient is a native deterministic column sum.

Forward and the two GEMMs of the backward are unchanged (hipBLASLt).  The bias gradient
``g.sum(0)`` runs csrc/linear.hip (two launches, fixed summation order) instead of
PyTorch-ROCm's multi-block ``reduce_kernel``, which returned wrong bias gradients for some
DistilBERT layers when replayed inside a captured hipGraph (tools/diag_bert_graph_vs_eager.py)
and cost ~18 µs per call.  Same parameters / ``state_dict`` as ``nn.Linear``.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ext
from .gradarena import grad_buffer
from .gradlink import InjectGrad

__all__ = ["Linear", "linear", "linear_gelu"]

# =1: the fused native GELU-backward + bias-sum pass.  Exact (tests/test_linear_gpu.py) but
# measured slower on 1x MI355X, DistilBERT r=8: 21.39 / 21.41 vs 21.27 ms (its column-strip
# grid has ~250 workgroups; ATen's GELU backward streams with the whole chip) -> off.
_FUSED_GELU = os.environ.get("NDP_FUSED_GELU", "0") != "0"


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, link=None):
        ctx.save_for_backward(x, weight)
        ctx.link = link  # ops/gradlink.GradLink: a residual gradient added into grad-x (addmm_)
        ctx.params = (weight, bias)  # the Parameters (ops/gradarena.py)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        n, k = weight.shape
        g2 = g.reshape(-1, n)
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        dx = dw = db = None
        addend = ctx.link.take() if ctx.link is not None else None
        if ctx.needs_input_grad[0]:
            if addend is not None:  # in place on the residual gradient buffer: GEMM with beta = 1
                dx = addend.reshape(-1, k).addmm_(g2, weight).view(x.shape)
            else:
                dx = (g2 @ weight).view(x.shape)
        elif addend is not None:
            dx = addend.view(x.shape)
        if ctx.needs_input_grad[1]:  # straight into the dense arm's arena slice when registered
            dw = torch.mm(g2.t(), x.reshape(-1, k), out=grad_buffer(ctx.params[0]))
        if ctx.needs_input_grad[2]:
            db = grad_buffer(ctx.params[1])
            ext().colsum(g2, db)
        return dx, dw, db, None


class _LinearGeluFn(torch.autograd.Function):
    """``gelu(linear(x))`` (exact GELU): forward = the library GEMM with bias epilogue + ATen's
    GELU; backward = ONE native pass computing ``dh = da * gelu'(h)`` and the bias column sums
    (csrc/linear.hip), then the grad-x (optionally onto a GradLink addend) and grad-W GEMMs."""

    @staticmethod
    def forward(ctx, x, weight, bias, link=None):
        h = F.linear(x, weight, bias)
        ctx.save_for_backward(x, weight, h)
        ctx.link = link
        return F.gelu(h)

    @staticmethod
    def backward(ctx, da):
        x, weight, h = ctx.saved_tensors
        n, k = weight.shape
        g2 = da.reshape(-1, n)
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        h2 = h.reshape(-1, n)
        dh = torch.empty_like(h2)
        db = torch.empty(n, device=da.device, dtype=da.dtype)
        ext().gelu_bwd_colsum(g2, h2, dh, db)
        addend = ctx.link.take() if ctx.link is not None else None
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = (addend.reshape(-1, k).addmm_(dh, weight) if addend is not None else dh @ weight).view(x.shape)
        elif addend is not None:
            dx = addend.view(x.shape)
        if ctx.needs_input_grad[1]:
            dw = dh.t() @ x.reshape(-1, k)
        return dx, dw, (db if ctx.needs_input_grad[2] else None), None


def linear_gelu(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, link=None) -> torch.Tensor:
    """``F.gelu(F.linear(x, weight, bias))`` with the fused native backward where it applies."""
    if _native_ok(x, weight, bias) and _FUSED_GELU:
        return _LinearGeluFn.apply(x, weight, bias, link)
    return F.gelu(linear(x, weight, bias, link))


def _native_ok(x, weight, bias) -> bool:
    return (x.is_cuda and bias is not None and x.dtype == torch.float32 and weight.dtype == torch.float32
            and weight.shape[0] % 4 == 0 and torch.is_grad_enabled())


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, link=None) -> torch.Tensor:
    """``F.linear`` with the native deterministic bias gradient where it applies.  ``link``
    (ops/gradlink.GradLink): a residual-branch gradient folded into this layer's grad-x."""
    if _native_ok(x, weight, bias):
        return _LinearFn.apply(x, weight, bias, link)
    return F.linear(InjectGrad.apply(x, link) if link is not None else x, weight, bias)


class Linear(nn.Linear):
    """Drop-in ``nn.Linear`` (device fp32 with bias and out_features % 4 == 0 -> native bias grad)."""

    def forward(self, x: torch.Tensor, link=None) -> torch.Tensor:
        if _native_ok(x, self.weight, self.bias):
            return _LinearFn.apply(x, self.weight, self.bias, link)
        return super().forward(InjectGrad.apply(x, link) if link is not None else x)
