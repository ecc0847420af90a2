"""Strided / tabled implicit-GEMM convolutions (csrc/tgemm.hip) behind an autograd Function.

The ``pointwise`` family the direct kernels (ops/conv.py) do not cover — 1x1 stride-1 convs on
any power-of-two map of >= 2 pixels: the bottleneck conv1 / conv3 and stride-1 downsample of
ResNet-50/101/152, the reference's own models (ddp_guide_cifar10/ddp_init.py:108,
ddp_powersgd_guide_cifar10/ddp_init.py:111) — forward / grad-x / grad-W all on one
hand-written gfx950 MFMA GEMM kernel.  (The small-map tabled family for ResNet layer3 / layer4
measured 0.46-0.72x the hipBLASLt Toeplitz GEMMs, profiles/r3/tg_bench.md, stayed off and was
deleted in round 6; so was the switch for 1x1 maps, where the plain GEMM is faster.)

Split-K slabs are summed in a fixed order (deterministic) — by the kernel's own slab sum,
by the fused BN kernel that consumes the conv (``slab_out`` / ``grad_slab``,
ops/slablink.py) or by gradfinish's batched sum (grad-W).  ``NDP_FUSION_OFF=tgemm`` disables
the path, restoring Toeplitz / MIOpen.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from . import gradfinish
from ._ext import ext
from .gradarena import grad_buffer
from ..knobs import fusion_on

__all__ = ["tg_plan", "TgConvFn", "enabled"]

_PLANS: dict = {}
_ON = fusion_on("tgemm")
POINTWISE = 0


def enabled() -> bool:
    return _ON


def tg_plan(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: int) -> Optional[Tuple]:
    """(geom, cls, fwd_slabs, dgrad_slabs, wgrad_slabs) if the tgemm path covers this conv."""
    if not (_ON and x.is_cuda and x.dtype == torch.float32 and weight.dtype == torch.float32 and x.dim() == 4):
        return None
    B, C, H, W = x.shape
    Co, Ci, KH, KW = weight.shape
    if Ci != C or KH != 1 or KW != 1:
        return None
    geom = (C, H, W, Co, KH, KW, int(stride), int(padding))
    key = (geom, int(B))
    if key not in _PLANS:  # the extension's answer is cached
        cls, fs, ds, ws = ext().tg_plan(list(geom), int(B))
        _PLANS[key] = (geom, int(cls), int(fs), int(ds), int(ws)) if cls >= 0 else None
    return _PLANS[key]


def _scratch(n_slabs: int, numel: int, like: torch.Tensor) -> Optional[torch.Tensor]:
    return torch.empty(n_slabs * numel, device=like.device, dtype=like.dtype) if n_slabs > 1 else None


class TgConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, plan, link=None, branch=None, slab_out=None, grad_slab=None):
        geom, cls, fs, _, _ = plan
        C, H, W, Co, KH, KW, s, p = geom
        x = x.contiguous()
        w = weight.contiguous()
        B = x.shape[0]
        OH = (H + 2 * p - KH) // s + 1
        OW = (W + 2 * p - KW) // s + 1
        y = torch.empty(B, Co, OH, OW, device=x.device, dtype=x.dtype)
        part = _scratch(fs, y.numel(), x)
        left = ext().tg_fwd(x, w, y, list(geom), part, slab_out is not None)
        if left > 1:
            slab_out.put_fwd(part, left)  # y is filled by the consuming fused BN kernel
        ctx.save_for_backward(x, w)
        ctx.plan = plan
        ctx.weight = weight  # the Parameter: a deferred grad-W finish writes its adopted .grad
        ctx.link = link      # ops/gradlink.GradLink: residual-branch gradient added in the epilogue
        ctx.grad_slab = grad_slab
        ctx.branch = branch
        if branch is not None:
            branch.join()    # ops/gradlink.BranchLink: grad-x shared with a sibling conv
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        geom, _, _, ds, ws = ctx.plan
        dy = dy.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[1]:
            dw = grad_buffer(ctx.weight, w)  # the dense arm's arena slice when registered
            defer = gradfinish.can_defer(ctx.weight)
            part = _scratch(ws, dw.numel(), x)
            left = ext().tg_wgrad(x, dy, dw, list(geom), part, defer)
            if left > 1:
                gradfinish.defer_slab(part, dw, left)
        if ctx.needs_input_grad[0]:
            addend = ctx.link.take() if ctx.link is not None else None
            br = ctx.branch if ctx.branch is not None and ctx.branch.active() else None
            other = None
            if br is not None:
                other = br.take()
                if addend is None:
                    addend = other
                elif other is not None:
                    addend = addend + other
            part = _scratch(ds, x.numel(), x)
            if addend is not None:  # dx = grad-x + addend, written in place over the addend buffer
                addend = addend.contiguous()
                ext().tg_dgrad(dy, w, addend, list(geom), part, addend, False)
                dx = addend
            else:
                dx = torch.empty_like(x)
                defer = ctx.grad_slab is not None and br is None
                left = ext().tg_dgrad(dy, w, dx, list(geom), part, None, defer)
                if left > 1:
                    ctx.grad_slab.put_bwd(part, left)  # dx stays unwritten: the BN backward sums the slabs
                if br is not None and other is None:  # first of the two: the sibling adds onto it
                    br.put(dx)
                    dx = None
        return dx, dw, None, None, None, None, None
