"""Strided / tabled implicit-GEMM convolutions (csrc/tgemm.hip) behind an autograd Function.

Two shape families the direct kernels (ops/conv.py) do not cover, forward / grad-x / grad-W
all on one hand-written gfx950 MFMA GEMM kernel:

* ``pointwise`` — 1x1 stride-1 convs on any power-of-two map: the bottleneck conv1 / conv3
  and stride-1 downsample of ResNet-50/101/152, the reference's own models
  (ddp_guide_cifar10/ddp_init.py:108, ddp_powersgd_guide_cifar10/ddp_init.py:111), which
  otherwise run on MIOpen;
* ``small`` — any conv from a <= 16-pixel map to a <= 4-pixel map (ResNet layer3 / layer4 on
  32x32 inputs): the Toeplitz product with the weight operand gathered through a tap table
  in the kernel arguments, so there is no W_big buffer and no expand launch; grad-W is
  W_big's gradient folded by the existing deterministic fold (batched, ops/gradfinish.py).

Split-K slabs are summed in a fixed order (deterministic) — by the kernel's own slab sum,
by the fused BN kernel that consumes the conv (``slab_out`` / ``grad_slab``,
ops/slablink.py) or by gradfinish's batched sum (grad-W).  ``NDP_FUSION_OFF=tgemm`` disables the path, restoring Toeplitz / MIOpen.  The ``small``
family and the pointwise kernel on 1x1 maps are off (measured slower; tests switch them on
through the module constants).
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
# small-map family off by default: measured 0.46-0.72x the hipBLASLt Toeplitz GEMMs on the
# ResNet-18 layer3 / layer4 shapes at batch 64 / 512 (tools/tg_bench.py, profiles/r3/tg_bench.md)
_SMALL = False
_PW = True
_PW1 = False  # pointwise on 1x1 maps (measured slower: off)
POINTWISE, SMALL = 0, 1


def enabled() -> bool:
    return _ON


def tg_plan(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: int) -> Optional[Tuple]:
    """(geom, cls, fwd_slabs, dgrad_slabs, wgrad_slabs) if the tgemm path covers this conv."""
    if not (_ON and x.is_cuda and x.dtype == torch.float32 and weight.dtype == torch.float32 and x.dim() == 4):
        return None
    B, C, H, W = x.shape
    Co, Ci, KH, KW = weight.shape
    if Ci != C or KH * KW > 9:  # the grad-W fold handles <= 3x3 kernels
        return None
    if KH == KW == 1 and stride == 1 and H * W == 1 and not _PW1:
        return None  # 1x1 conv on a 1x1 map: the plain hipBLASLt GEMM (Toeplitz path) is faster
    geom = (C, H, W, Co, KH, KW, int(stride), int(padding))
    key = (geom, int(B))
    if key not in _PLANS:  # the extension's answer is cached; the family switches apply per call
        cls, fs, ds, ws = ext().tg_plan(list(geom), int(B))
        _PLANS[key] = (geom, int(cls), int(fs), int(ds), int(ws)) if cls >= 0 else None
    plan = _PLANS[key]
    if plan is None or not ((plan[1] == POINTWISE and _PW) or (plan[1] == SMALL and _SMALL)):
        return None
    return plan


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
        geom, cls, _, ds, ws = ctx.plan
        C, H, W, Co, KH, KW, s, p = geom
        dy = dy.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[1]:
            dw = grad_buffer(ctx.weight, w)  # the dense arm's arena slice when registered
            defer = gradfinish.can_defer(ctx.weight)
            if cls == POINTWISE:
                part = _scratch(ws, dw.numel(), x)
                left = ext().tg_wgrad(x, dy, dw, list(geom), part, defer)
                if left > 1:
                    gradfinish.defer_slab(part, dw, left)
            else:
                OH = (H + 2 * p - KH) // s + 1
                OW = (W + 2 * p - KW) // s + 1
                dwt = torch.empty(Co * OH * OW, C * H * W, device=x.device, dtype=x.dtype)
                ext().tg_wgrad(x, dy, dwt, list(geom), _scratch(ws, dwt.numel(), x), False)
                if defer:
                    gradfinish.defer_fold(dwt, dw, geom)
                else:
                    ext().toeplitz_fold(dwt, dw, list(geom))
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
