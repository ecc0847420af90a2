"""``nn.LayerNorm`` with an optional fused residual add — gfx950 kernels (csrc/layernorm.hip).

DistilBERT (ddp_powersgd_distillBERT_IMDb/ddp_init.py:150, HF ``DistilBertModel``) computes
``LayerNorm(sublayer(x) + x)`` twice per block plus once after the embeddings.  On device
:class:`AddLayerNorm` runs ``forward(x, residual)`` as ONE kernel (add + statistics +
affine, the sum saved for backward) and the backward as one row kernel plus one fixed-order
reduction of the [dgamma | dbeta] partials — deterministic and hipGraph-replayable — instead
of PyTorch-ROCm's add + LayerNorm + three backward kernels.  Same parameters / ``state_dict``
as ``nn.LayerNorm`` (HF checkpoints load unchanged).  CPU tensors, other dtypes, unsupported
widths (last dim not 256/512/768/1024) or ``NDP_FUSION_OFF=fused_ln`` run the PyTorch ops.

HF DistilBERT's hidden dropouts ride in the same kernels: ``p_in`` drops the sublayer output
before the residual add (FFN: ``LN(dropout(lin2(.)) + x)``), ``p_out`` drops the normalised
output (embeddings: ``dropout(LN(word + pos))``).  The keep mask is a stateless hash of
(seed, row, column) (:func:`ln_keep_mask` is its host twin) with the seed a device int32 drawn
from torch's generator per call, so backward regenerates it and hipGraph replays draw fresh
masks — no mask tensor, no ATen dropout / masked-scale kernels.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import gradfinish
from ._ext import ext
from ..knobs import fusion_on

__all__ = ["AddLayerNorm", "add_layer_norm", "ln_keep_mask"]

_ENABLED = fusion_on("fused_ln")
_WIDTHS = (256, 512, 768, 1024)
_M32 = 0xFFFFFFFF


def ln_keep_mask(seed: int, R: int, D: int, p: float, device="cpu") -> torch.Tensor:
    """Host twin of csrc/layernorm.hip ``ln_hash``: the [R, D] keep mask for ``seed``."""
    thr = min(int(p * 4294967296.0), _M32)
    r = torch.arange(R, dtype=torch.int64, device=device).view(-1, 1)
    c = torch.arange(D, dtype=torch.int64, device=device).view(1, -1)
    h = ((seed & _M32) * 0x9E3779B1 & _M32) ^ (((r + 0x7F4A7C15) & _M32) * 0x85EBCA77 & _M32)
    h = ((h ^ (h >> 15)) * 0x2C1B3C6D) & _M32
    h = h ^ (((c + 0x165667B1) & _M32) * 0xC2B2AE3D & _M32)
    h = ((h ^ (h >> 13)) * 0x297A2D39) & _M32
    h = h ^ (h >> 16)
    return h >= thr


def _seed(device) -> torch.Tensor:
    return torch.randint(0, 2 ** 31 - 1, (1,), device=device, dtype=torch.int32)


class _AddLayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, link=None, mode=0, p=0.0, seed=None):
        x = x.contiguous()
        r = residual.contiguous() if residual is not None else None
        D = x.shape[-1]
        R = x.numel() // D
        y = torch.empty_like(x)
        s = torch.empty_like(x)
        mean = torch.empty(R, device=x.device, dtype=torch.float32)
        rstd = torch.empty(R, device=x.device, dtype=torch.float32)
        ext().ln_fwd(x, r, weight, bias, y, s, mean, rstd, float(eps), mode, p, seed)
        ctx.has_res = r is not None
        ctx.link = link  # ops/gradlink.GradLink: the residual's gradient goes there instead
        ctx.mode, ctx.p = mode, p
        ctx.params = (weight, bias)
        ctx.save_for_backward(s, mean, rstd, weight, seed)
        return y

    @staticmethod
    def backward(ctx, dy):
        s, mean, rstd, weight, seed = ctx.saved_tensors
        dx = torch.empty_like(s)
        D = s.shape[-1]
        dgb = torch.empty(2 * D, device=s.device, dtype=torch.float32)
        # input dropout: the sublayer's gradient is the masked copy written by the same pass
        da = torch.empty_like(s) if ctx.mode == 1 else None
        part = None
        if gradfinish.enabled() and all(gradfinish.can_defer(p) for p in ctx.params):
            # the [dgamma | dbeta] partial sum waits for gradfinish's one batched launch
            part = torch.empty(ext().ln_bwd_wgs(s.numel() // D) * 2 * D, device=s.device, dtype=s.dtype)
        left = ext().ln_bwd(dy.contiguous(), s, mean, rstd, weight, dx, dgb, ctx.mode, ctx.p, seed, da, part)
        if part is not None:
            gradfinish.defer_slab(part, dgb, left)
        # d(x + residual) reaches both inputs unchanged; with a link the residual's copy is
        # added by the sublayer's first GEMM (after every reader of dx for x has run)
        dres = dx if ctx.has_res else None
        if ctx.link is not None and dres is not None:
            ctx.link.put(dres)
            dres = None
        return (da if da is not None else dx), dres, dgb[:D].view_as(weight), dgb[D:].view_as(weight), None, None, \
            None, None, None


def add_layer_norm(x: torch.Tensor, residual: Optional[torch.Tensor], weight: torch.Tensor, bias: torch.Tensor,
                   eps: float, link=None, p_in: float = 0.0, p_out: float = 0.0,
                   seed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.layer_norm(dropout(x, p_in) + residual, (D,), weight, bias, eps)`` followed by
    ``dropout(., p_out)`` (residual may be None; at most one of the dropouts).  ``link``
    (ops/gradlink.GradLink, fused path only): the residual's gradient is deposited there (the
    residual is taken detached) for the consumer GEMM that folds it in.  ``seed`` pins the
    fused path's dropout mask (:func:`ln_keep_mask`)."""
    assert not (p_in > 0 and p_out > 0), "one dropout per LayerNorm"
    if (_ENABLED and x.is_cuda and x.dtype == torch.float32 and x.shape[-1] in _WIDTHS and weight is not None
            and bias is not None and weight.dtype == torch.float32
            and (residual is None or (residual.dtype == torch.float32 and residual.shape == x.shape))):
        if link is not None and residual is not None:
            residual = residual.detach()
        mode, p = (1, float(p_in)) if p_in > 0 else ((2, float(p_out)) if p_out > 0 else (0, 0.0))
        if mode and seed is None:
            seed = _seed(x.device)
        return _AddLayerNormFn.apply(x, residual, weight, bias, eps, link, mode, p, seed if mode else None)
    assert link is None or link.grad is None
    if p_in > 0:
        x = F.dropout(x, p_in)
    h = x if residual is None else x + residual
    y = F.layer_norm(h, (x.shape[-1],), weight, bias, eps)
    return F.dropout(y, p_out) if p_out > 0 else y


class AddLayerNorm(nn.LayerNorm):
    """Drop-in ``nn.LayerNorm`` (1-D normalized shape, affine) with ``forward(x, residual=None)``.
    ``native = False`` keeps PyTorch's ops (the stock-kernels arm)."""

    native = True

    def fused_ok(self, x: torch.Tensor, residual: Optional[torch.Tensor]) -> bool:
        """Whether forward(x, residual) takes the native kernel (a GradLink is only honoured there)."""
        return (self.native and _ENABLED and len(self.normalized_shape) == 1 and self.elementwise_affine
                and x.is_cuda and x.dtype == torch.float32 and x.shape[-1] in _WIDTHS
                and (residual is None or (residual.dtype == torch.float32 and residual.shape == x.shape)))

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, link=None, p_in: float = 0.0,
                p_out: float = 0.0, seed: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``LN(dropout(x, p_in) + residual)``, then ``dropout(., p_out)`` (dropouts fused on device;
        ``seed`` a device int32 for their mask, None draws one)."""
        if self.native and len(self.normalized_shape) == 1 and self.elementwise_affine:
            return add_layer_norm(x, residual, self.weight, self.bias, self.eps,
                                  link if self.fused_ok(x, residual) else None, p_in, p_out, seed)
        if p_in > 0:
            x = F.dropout(x, p_in)
        y = super().forward(x if residual is None else x + residual)
        return F.dropout(y, p_out) if p_out > 0 else y
