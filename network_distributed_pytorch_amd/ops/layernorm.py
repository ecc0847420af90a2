"""``nn.LayerNorm`` with an optional fused residual add — gfx950 kernels (csrc/layernorm.hip).

DistilBERT (ddp_powersgd_distillBERT_IMDb/ddp_init.py:150, HF ``DistilBertModel``) computes
``LayerNorm(sublayer(x) + x)`` twice per block plus once after the embeddings.  On device
:class:`AddLayerNorm` runs ``forward(x, residual)`` as ONE kernel (add + statistics +
affine, the sum saved for backward) and the backward as one row kernel plus one fixed-order
reduction of the [dgamma | dbeta] partials — deterministic and hipGraph-replayable — instead
of PyTorch-ROCm's add + LayerNorm + three backward kernels.  Same parameters / ``state_dict``
as ``nn.LayerNorm`` (HF checkpoints load unchanged).  CPU tensors, other dtypes, unsupported
widths (last dim not 256/512/768/1024) or ``NDP_FUSED_LN=0`` run the PyTorch ops.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ext

__all__ = ["AddLayerNorm", "add_layer_norm"]

_ENABLED = os.environ.get("NDP_FUSED_LN", "1") != "0"
_WIDTHS = (256, 512, 768, 1024)


class _AddLayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, link=None):
        x = x.contiguous()
        r = residual.contiguous() if residual is not None else None
        D = x.shape[-1]
        R = x.numel() // D
        y = torch.empty_like(x)
        s = torch.empty_like(x)
        mean = torch.empty(R, device=x.device, dtype=torch.float32)
        rstd = torch.empty(R, device=x.device, dtype=torch.float32)
        ext().ln_fwd(x, r, weight, bias, y, s, mean, rstd, float(eps))
        ctx.has_res = r is not None
        ctx.link = link  # ops/gradlink.GradLink: the residual's gradient goes there instead
        ctx.save_for_backward(s, mean, rstd, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        s, mean, rstd, weight = ctx.saved_tensors
        dx = torch.empty_like(s)
        D = s.shape[-1]
        dgb = torch.empty(2 * D, device=s.device, dtype=torch.float32)
        ext().ln_bwd(dy.contiguous(), s, mean, rstd, weight, dx, dgb)
        # d(x + residual) reaches both inputs unchanged; with a link the residual's copy is
        # added by the sublayer's first GEMM (after every reader of dx for x has run)
        dres = dx if ctx.has_res else None
        if ctx.link is not None and dres is not None:
            ctx.link.put(dres)
            dres = None
        return dx, dres, dgb[:D].view_as(weight), dgb[D:].view_as(weight), None, None


def add_layer_norm(x: torch.Tensor, residual: Optional[torch.Tensor], weight: torch.Tensor, bias: torch.Tensor,
                   eps: float, link=None) -> torch.Tensor:
    """``F.layer_norm(x + residual, (D,), weight, bias, eps)`` (residual may be None).
    ``link`` (ops/gradlink.GradLink, fused path only): the residual's gradient is deposited
    there (the residual is taken detached) for the consumer GEMM that folds it in."""
    if (_ENABLED and x.is_cuda and x.dtype == torch.float32 and x.shape[-1] in _WIDTHS and weight is not None
            and bias is not None and weight.dtype == torch.float32
            and (residual is None or (residual.dtype == torch.float32 and residual.shape == x.shape))):
        if link is not None and residual is not None:
            residual = residual.detach()
        return _AddLayerNormFn.apply(x, residual, weight, bias, eps, link)
    assert link is None or link.grad is None
    h = x if residual is None else x + residual
    return F.layer_norm(h, (x.shape[-1],), weight, bias, eps)


class AddLayerNorm(nn.LayerNorm):
    """Drop-in ``nn.LayerNorm`` (1-D normalized shape, affine) with ``forward(x, residual=None)``.
    ``native = False`` keeps PyTorch's ops (the stock-kernels arm)."""

    native = True

    def fused_ok(self, x: torch.Tensor, residual: Optional[torch.Tensor]) -> bool:
        """Whether forward(x, residual) takes the native kernel (a GradLink is only honoured there)."""
        return (self.native and _ENABLED and len(self.normalized_shape) == 1 and self.elementwise_affine
                and x.is_cuda and x.dtype == torch.float32 and x.shape[-1] in _WIDTHS
                and (residual is None or (residual.dtype == torch.float32 and residual.shape == x.shape)))

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, link=None) -> torch.Tensor:
        if self.native and len(self.normalized_shape) == 1 and self.elementwise_affine:
            return add_layer_norm(x, residual, self.weight, self.bias, self.eps, link if self.fused_ok(x, residual)
                                  else None)
        return super().forward(x if residual is None else x + residual)
