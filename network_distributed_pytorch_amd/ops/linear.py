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

from . import gradfinish
from ._ext import ext
from .gradarena import grad_buffer, registered
from .gradlink import InjectGrad
from ..knobs import fusion_on

__all__ = ["Linear", "linear", "linear_gelu", "packed_qkv"]

# the fused native GELU-backward + bias-sum pass (NDP_FUSION_OFF=fused_gelu: ATen GELU backward + the
# native bias sum).  Exact (tests/test_linear_gpu.py).  Round 3 measured it slower (~250
# column-strip workgroups, one load in flight per thread); with ~1024 workgroups and 4 rows in
# flight per thread it is on: DistilBERT r=8, 1x MI355X, 20.70 vs 20.74 ms (profiles/r4).
_FUSED_GELU = fusion_on("fused_gelu")


def _deferrable(out: torch.Tensor, params) -> bool:
    """The final fixed-order sum of a bias gradient may wait for gradfinish's batched launch
    (one ``slab_sum_many`` for every deferred gradient of the backward pass)."""
    return (gradfinish.enabled() and out.data_ptr() % 16 == 0 and out.is_contiguous()
            and all(p is not None and gradfinish.can_defer(p) for p in params))


def _bias_sum(g2: torch.Tensor, db: torch.Tensor, params) -> None:
    """db = g2.sum(0) (csrc/linear.hip colsum), its last pass deferred when allowed."""
    if _deferrable(db, params):
        M, N = g2.shape
        part = torch.empty(ext().colsum_chunks(M, N) * N, device=g2.device, dtype=g2.dtype)
        gradfinish.defer_slab(part, db, ext().colsum(g2, db, part))
    else:
        ext().colsum(g2, db)


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
            _bias_sum(g2, db, (ctx.params[1],))
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
        ctx.bias = bias
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
        if ctx.needs_input_grad[2] and _deferrable(db, (ctx.bias,)):
            M = g2.shape[0]
            part = torch.empty(ext().colsum_chunks(M, n) * n, device=da.device, dtype=da.dtype)
            gradfinish.defer_slab(part, db, ext().gelu_bwd_colsum(g2, h2, dh, db, part))
        else:
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


def _adjacent(ts):
    """One [sum rows, ...] view over tensors that already sit back to back in one storage
    (the PowerSGD parameter arena lays q / k / v out consecutively), else None."""
    t0 = ts[0]
    off = t0.numel()
    for t in ts[1:]:
        if not (t.is_contiguous() and t.dtype == t0.dtype and t.device == t0.device and t.shape[1:] == t0.shape[1:]
                and t.untyped_storage().data_ptr() == t0.untyped_storage().data_ptr()
                and t.data_ptr() == t0.data_ptr() + off * t0.element_size()):
            return None
        off += t.numel()
    if not t0.is_contiguous():
        return None
    rows = sum(t.shape[0] for t in ts)
    return torch.as_strided(t0.detach(), (rows,) + tuple(t0.shape[1:]), t0.detach().stride(), t0.storage_offset())


class _PackedQKVFn(torch.autograd.Function):
    """One [B*S, 3D] projection GEMM for the three attention projections whose weights stay
    three Parameters (HF keys, the reference's PowerSGD layout and byte count): read in place
    when they are consecutive in memory (the PowerSGD arena), concatenated otherwise; their
    gradients come back as views of one grad-W / one bias-sum buffer (or, for parameters
    registered in the dense arena, straight into their arena slices)."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv, bq, bk, bv, link=None):
        w = _adjacent((wq, wk, wv))
        b = _adjacent((bq, bk, bv))
        if w is None:
            w = torch.cat([wq.detach(), wk.detach(), wv.detach()])
        if b is None:
            b = torch.cat([bq.detach(), bk.detach(), bv.detach()])
        ctx.save_for_backward(x, w)
        ctx.link = link
        ctx.params = (wq, wk, wv, bq, bk, bv)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        n, k = w.shape
        d = n // 3
        g2 = g.reshape(-1, n)
        if not g2.is_contiguous():
            g2 = g2.contiguous()
        x2 = x.reshape(-1, k)
        addend = ctx.link.take() if ctx.link is not None else None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (addend.reshape(-1, k).addmm_(g2, w) if addend is not None else g2 @ w).view(x.shape)
        elif addend is not None:
            dx = addend.view(x.shape)
        wq, wk, wv, bq, bk, bv = ctx.params
        if any(registered(p) for p in (wq, wk, wv)):
            # dense arena slices (reverse order, not adjacent): one GEMM each, written in place
            dws = [torch.mm(g2[:, i * d:(i + 1) * d].t(), x2, out=grad_buffer(p)) for i, p in enumerate((wq, wk, wv))]
        else:
            dw = torch.empty(n, k, device=g.device, dtype=g.dtype)
            torch.mm(g2.t(), x2, out=dw)
            dws = [dw[i * d:(i + 1) * d] for i in range(3)]
        db = torch.empty(n, device=g.device, dtype=g.dtype)
        _bias_sum(g2, db, (bq, bk, bv))
        dbs = [db[i * d:(i + 1) * d] for i in range(3)]
        return (dx,) + tuple(dws) + tuple(dbs) + (None,)


def packed_qkv(x: torch.Tensor, q, k, v, link=None) -> torch.Tensor:
    """[q(x) | k(x) | v(x)] as one GEMM (Linear modules q / k / v, same shapes)."""
    return _PackedQKVFn.apply(x, q.weight, k.weight, v.weight, q.bias, k.bias, v.bias, link)


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
