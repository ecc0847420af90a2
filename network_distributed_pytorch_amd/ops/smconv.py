"""Small-map convolutions (csrc/smallconv.hip) behind an autograd Function.

ResNet on 32x32 inputs runs layer3 / layer4 at 4x4 -> 2x2 -> 1x1 maps.  Every such conv of
the 8 geometries the kernels cover (3x3 on 2x2 / 1x1, the stride-2 entry convs, the stride-2
1x1 downsamples, 1x1 on 2x2 / 1x1) runs forward, grad-x and grad-W on hand-written
16x16x4 f32 MFMA kernels whose pair list (input pixel, output pixel, tap) is a compile-time
constant: no W_big expand, no grad-W fold, no vendor GEMM.  Replaces the hipBLASLt Toeplitz
path (models/conv_gemm.py) and the tabled tgemm family for these shapes.

Split-K slabs (small per-GPU batches) are summed in a fixed order — by the fused BN kernel
that consumes the conv (``slab_out`` / ``grad_slab``, ops/slablink.py), by the kernel's own
slab sum, or (grad-W, batch splits) by gradfinish's batched sum.

OFF by default (``NDP_SM=1`` turns it on for every covered geometry, ``NDP_SM=l3entry`` only for
the two 4x4-input convs of layer3's entry block — the 3x3 / 2 and the 1x1 / 2): measured on 1x MI355X (profiles/r4/smallconv.md) the
kernels are at parity with hipBLASLt on the 3x3 convs, faster on the layer3 entry / downsample,
and 2.5x slower on the layer4 entry (2x2 -> 1x1, 4 of 9 taps gathered as scalars); the whole
ResNet-18 step is slower with them (batch 512: 2.16 vs 1.93 ms, batch 64: 1.10 vs 1.00 ms).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from . import gradfinish
from ._ext import ext
from .gradarena import grad_buffer

__all__ = ["sm_plan", "SmConvFn", "enabled"]

_PLANS: dict = {}
_MODE = os.environ.get("NDP_SM", "0")
_ON = _MODE != "0"


def enabled() -> bool:
    """Every covered geometry on the small-map kernels (the fused stage needs them all)."""
    return _ON and _MODE != "l3entry"


def _wanted(H: int, W: int) -> bool:
    return _MODE != "l3entry" or (H == 4 and W == 4)


def sm_plan(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: int) -> Optional[Tuple]:
    """(geom, cls, fwd_slabs, dgrad_slabs, wgrad_slabs) if a small-map kernel covers this conv."""
    if not (_ON and x.is_cuda and x.dtype == torch.float32 and weight.dtype == torch.float32 and x.dim() == 4):
        return None
    B, C, H, W = x.shape
    Co, Ci, KH, KW = weight.shape
    if Ci != C or not _wanted(H, W):
        return None
    geom = (C, H, W, Co, KH, KW, int(stride), int(padding))
    key = (geom, int(B))
    if key not in _PLANS:
        cls, fs, ds, ws = ext().sm_plan(list(geom), int(B))
        _PLANS[key] = (geom, int(cls), int(fs), int(ds), int(ws)) if cls >= 0 else None
    return _PLANS[key]


def _scratch(n_slabs: int, numel: int, like: torch.Tensor) -> Optional[torch.Tensor]:
    return torch.empty(n_slabs * numel, device=like.device, dtype=like.dtype) if n_slabs > 1 else None


class SmConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, plan, link=None, branch=None, slab_out=None, grad_slab=None):
        geom, _, fs, _, _ = plan
        C, H, W, Co, KH, KW, s, p = geom
        x = x.contiguous()
        w = weight.contiguous()
        B = x.shape[0]
        OH = (H + 2 * p - KH) // s + 1
        OW = (W + 2 * p - KW) // s + 1
        y = torch.empty(B, Co, OH, OW, device=x.device, dtype=x.dtype)
        part = _scratch(fs, y.numel(), x)
        left = ext().sm_fwd(x, w, y, list(geom), part, slab_out is not None)
        if left > 1:
            slab_out.put_fwd(part, left)  # y is filled by the consuming fused BN kernel
        ctx.save_for_backward(x, w)
        ctx.plan = plan
        ctx.weight = weight  # the Parameter: a deferred grad-W slab sum writes its adopted .grad
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
            if ws > 1:  # batch-split slabs: summed later in one batched launch (or now)
                part = torch.empty(ws * w.numel(), device=x.device, dtype=x.dtype)
                ext().sm_wgrad(x, dy, part, list(geom))
                if gradfinish.can_defer(ctx.weight):
                    gradfinish.defer_slab(part, dw, ws)
                else:
                    ext().slab_sum(part, dw.view(-1), ws)
            else:
                ext().sm_wgrad(x, dy, dw, list(geom))
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
                ext().sm_dgrad(dy, w, addend, list(geom), part, addend, False)
                dx = addend
            else:
                dx = torch.empty_like(x)
                defer = ctx.grad_slab is not None and br is None
                left = ext().sm_dgrad(dy, w, dx, list(geom), part, None, defer)
                if left > 1:
                    ctx.grad_slab.put_bwd(part, left)  # dx stays unwritten: the BN backward sums the slabs
                if br is not None and other is None:  # first of the two: the sibling adds onto it
                    br.put(dx)
                    dx = None
        return dx, dw, None, None, None, None, None
