"""Fused BatchNorm2d (+ residual add) (+ ReLU) — gfx950 kernels with a torch fallback.

:class:`BatchNormAct2d` is a drop-in ``nn.BatchNorm2d`` (same parameters, buffers and
``state_dict`` keys, so torchvision checkpoints load unchanged) whose forward optionally
fuses the residual add and the ReLU that follow BN in every ResNet block:
``y = relu(bn(x) + residual)``.  On device it runs two kernels per direction
(csrc/batchnorm.hip) instead of MIOpen BN + ATen ReLU + ATen add + the
``num_batches_tracked`` increment; on CPU it computes the same math with torch ops.
Training statistics follow ``torch.nn.BatchNorm2d`` exactly (biased variance for the
normalisation, unbiased in ``running_var``, momentum 0.1).
"""
from __future__ import annotations

import os

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ext
from .gradarena import grad_buffer
from ..knobs import fusion_on

__all__ = ["BatchNormAct2d", "bn_act", "bn_pair_act"]


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, weight, bias, running_mean, running_var, nbt, part, eps, momentum, relu, single=False,
                link=None, slab_in=None, grad_slab=None):
        X = ext()
        x = x.contiguous()
        if res is not None:
            res = res.contiguous()
        C = x.shape[1]
        y = torch.empty_like(x)
        save_mean = torch.empty(C, device=x.device, dtype=torch.float32)
        save_invstd = torch.empty(C, device=x.device, dtype=torch.float32)
        xpart, nslab = slab_in.take_fwd() if slab_in is not None else (None, 0)
        # statistics from the producing conv's epilogue (ops/slablink.py): no statistics pass
        xstats, xS = slab_in.take_stats() if slab_in is not None else (None, 0)
        X.bn_fwd(x, res, y, weight, bias, running_mean, running_var, nbt, save_mean, save_invstd, part,
                 float(eps), float(momentum), bool(relu), True, bool(single), xpart, nslab, xstats, xS)
        ctx.grad_slab = grad_slab  # ops/slablink.py: dy may arrive as the next conv's grad-x slabs
        if (grad_slab is not None and relu and _BWD_STATS
                and X.bn_two_kernel_path(x.shape[0], C, x.numel() // (x.shape[0] * C), bool(single))):
            # the conv producing dy may emit this BN's backward statistics (grad-x epilogue)
            grad_slab.bn_saved = (x, y, save_mean, save_invstd)
        ctx.relu = bool(relu)
        ctx.single = bool(single)
        ctx.has_res = res is not None
        ctx.link = link  # ops/gradlink.py: the residual gradient goes here, not to `res`
        ctx.has_w = weight is not None
        ctx.params = (weight, bias)  # the Parameters: their arena slices take the gradients
        ctx.save_for_backward(x, y if relu else None, weight, save_mean, save_invstd, part)
        ctx.mark_non_differentiable(save_mean, save_invstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, weight, save_mean, save_invstd, part = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if ctx.has_res else None
        # the dense arm's arena slices when registered (ops/gradarena.py)
        dgamma = grad_buffer(ctx.params[0], weight) if ctx.has_w else None
        dbeta = grad_buffer(ctx.params[1], weight) if ctx.has_w else None
        dypart, nslab = ctx.grad_slab.take_bwd() if ctx.grad_slab is not None else (None, 0)
        dyadd = ctx.grad_slab.take_bwd_add() if ctx.grad_slab is not None else None
        dstats, dS = ctx.grad_slab.take_bwd_stats() if ctx.grad_slab is not None else (None, 0)
        if ctx.grad_slab is not None:
            ctx.grad_slab.bn_saved = None
        ext().bn_bwd(dy, y, x, weight, save_mean, save_invstd, dx, dres, dgamma, dbeta, part, ctx.relu, ctx.single,
                     dypart, nslab, dyadd, None, dstats if dypart is None else None, dS if dypart is None else 0)
        if ctx.link is not None and dres is not None:
            ctx.link.put(dres)
            dres = None
        return dx, dres, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None


class _BNReluPoolFn(torch.autograd.Function):
    """Training BN -> ReLU -> MaxPool(3, 2, 1) (csrc/batchnorm.hip bn_relu_maxpool): the BN
    output is never stored; backward = the native pool backward, then the BN backward with its
    ReLU mask recomputed from x (``mbeta``)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, part, eps, momentum, single, slab_in=None):
        X = ext()
        x = x.contiguous()
        N, C, H, W = x.shape
        y = torch.empty(N, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1, device=x.device, dtype=x.dtype)
        idx = torch.empty(y.shape, device=x.device, dtype=torch.uint8)
        save_mean = torch.empty(C, device=x.device, dtype=torch.float32)
        save_invstd = torch.empty(C, device=x.device, dtype=torch.float32)
        xstats, xS = slab_in.take_stats() if slab_in is not None else (None, 0)
        X.bn_relu_maxpool(x, y, idx, weight, bias, running_mean, running_var, nbt, save_mean, save_invstd, part,
                          float(eps), float(momentum), xstats, xS)
        ctx.save_for_backward(x, weight, bias, save_mean, save_invstd, part, idx)
        ctx.params = (weight, bias)
        ctx.single = bool(single)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, save_mean, save_invstd, part, idx = ctx.saved_tensors
        dx = torch.empty_like(x)
        dgamma = grad_buffer(ctx.params[0], weight)
        dbeta = grad_buffer(ctx.params[1], weight)
        N, C, H, W = x.shape
        if _BWD_STATS and _STEM_BWD and H == 16 and W == 16:
            # statistics-only pool backward, then ONE pass from the pooled gradient to the BN input
            # gradient (csrc/batchnorm.hip stem_pool_bwd_apply_kernel): the routed 16x16 gradient
            # is never stored (bitwise equal to the two-pass path below)
            dy = dy.contiguous()
            stats = torch.empty(C * N * 2, device=x.device, dtype=torch.float64)
            ext().maxpool_bwd_bnstats(dy, idx, None, x, weight, bias, save_mean, save_invstd, stats)
            ext().stem_pool_bwd_apply(dy, idx, x, weight, bias, save_mean, save_invstd, stats, dx, dgamma, dbeta)
            return dx, dgamma, dbeta, None, None, None, None, None, None, None, None
        dz = torch.empty_like(x)  # gradient of the (unstored) BN output = the pool's input
        if _BWD_STATS and H == 16 and W == 16:  # the pool backward also emits the BN's statistics
            stats = torch.empty(C * N * 2, device=x.device, dtype=torch.float64)
            ext().maxpool_bwd_bnstats(dy.contiguous(), idx, dz, x, weight, bias, save_mean, save_invstd, stats)
            ext().bn_bwd(dz, None, x, weight, save_mean, save_invstd, dx, None, dgamma, dbeta, part, True, ctx.single,
                         None, 0, None, bias, stats, N)
        else:
            ext().maxpool_bwd(dy.contiguous(), idx, dz, 3, 2, 1)
            ext().bn_bwd(dz, None, x, weight, save_mean, save_invstd, dx, None, dgamma, dbeta, part, True, ctx.single,
                         None, 0, None, bias)
        return dx, dgamma, dbeta, None, None, None, None, None, None, None, None


class _BNPairFn(torch.autograd.Function):
    """relu(bn(x) + bn2(x2)) — a ResNet downsample block's bn2 and downsample BN in one launch per
    direction (csrc/batchnorm.hip BnPair).  The downsample BN's output is never stored; backward
    forms both BNs' sums from the shared dz = dy * (y > 0) and writes both input gradients."""

    @staticmethod
    def forward(ctx, x, x2, w, b, rm, rv, nbt, w2, b2, rm2, rv2, nbt2, eps, momentum, slab_in=None, slab_in2=None,
                grad_slab=None):
        x, x2 = x.contiguous(), x2.contiguous()
        C = x.shape[1]
        y = torch.empty_like(x)
        sm, si, sm2, si2 = (torch.empty(C, device=x.device, dtype=torch.float32) for _ in range(4))
        xpart, nslab = slab_in.take_fwd() if slab_in is not None else (None, 0)
        x2part, nslab2 = slab_in2.take_fwd() if slab_in2 is not None else (None, 0)
        for link in (slab_in, slab_in2):  # the kernel forms its own statistics
            if link is not None:
                link.take_stats()
        ext().bn_pair_fwd(x, x2, y, w, b, rm, rv, nbt, sm, si, w2, b2, rm2, rv2, nbt2, sm2, si2, float(eps),
                          float(momentum), xpart, nslab, x2part, nslab2)
        ctx.grad_slab = grad_slab
        ctx.params = (w, b, w2, b2)
        ctx.save_for_backward(x, x2, y, w, w2, sm, si, sm2, si2)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, x2, y, w, w2, sm, si, sm2, si2 = ctx.saved_tensors
        dy = dy.contiguous()
        dx, dx2 = torch.empty_like(x), torch.empty_like(x2)
        pw, pb, pw2, pb2 = ctx.params
        dg, db = grad_buffer(pw, w), grad_buffer(pb, w)
        dg2, db2 = grad_buffer(pw2, w2), grad_buffer(pb2, w2)
        dypart, nslab, dyadd = None, 0, None
        if ctx.grad_slab is not None:
            dypart, nslab = ctx.grad_slab.take_bwd()
            dyadd = ctx.grad_slab.take_bwd_add()
            ctx.grad_slab.take_bwd_stats()
            ctx.grad_slab.bn_saved = None
        ext().bn_pair_bwd(dy, y, x, x2, w, sm, si, w2, sm2, si2, dx, dx2, dg, db, dg2, db2, dypart, nslab, dyadd)
        return (dx, dx2, dg, db, None, None, None, dg2, db2, None, None, None, None, None, None, None, None)


# the downsample block's two BNs in one launch per direction (NDP_FUSION_OFF=bn_pair: two launches)
BN_PAIR = fusion_on("bn_pair")


def bn_pair_act(bn: "BatchNormAct2d", bn2: "BatchNormAct2d", x: torch.Tensor, x2: torch.Tensor, slab_in=None,
                slab_in2=None, grad_slab=None) -> Optional[torch.Tensor]:
    """``relu(bn(x) + bn2(x2))`` as one training launch per direction where the single-launch
    small-map kernels apply, else None (the caller runs the two BNs)."""
    if not (BN_PAIR and x.is_cuda and x.dtype == torch.float32 and x2.dtype == torch.float32
            and torch.is_grad_enabled() and bn.training and bn2.training and x.shape == x2.shape and x.dim() == 4
            and bn.fused_small and bn2.fused_small and bn.eps == bn2.eps and bn.momentum == bn2.momentum
            and all(m.affine and m.track_running_stats and m.momentum is not None for m in (bn, bn2))):
        return None
    N, C = x.shape[:2]
    if not ext().bn_pair_ok(N, C, x.shape[2] * x.shape[3]):
        return None
    return _BNPairFn.apply(x, x2, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                           bn2.weight, bn2.bias, bn2.running_mean, bn2.running_var, bn2.num_batches_tracked,
                           bn.eps, bn.momentum, slab_in, slab_in2, grad_slab)


# BN backward statistics from the grad-x epilogue of the conv producing dy (ops/slablink.py;
# NDP_FUSION_OFF=bn_bwd_stats: the BN's own statistics pass)
_BWD_STATS = fusion_on("bn_bwd_stats")

# the stem tail BN -> ReLU -> MaxPool in one pass (NDP_FUSION_OFF=stem_pool: BN kernel + pool kernel)
STEM_POOL = fusion_on("stem_pool")
# its backward without the stored 16x16 pool gradient (NDP_FUSION_OFF=stem_bwd: pool backward +
# BN backward apply)
_STEM_BWD = fusion_on("stem_bwd")


def bn_act(x, weight, bias, running_mean, running_var, nbt, part, training, momentum, eps,
           residual=None, relu=False, single=False, link=None, slab_in=None, grad_slab=None):
    needs_grad = torch.is_grad_enabled() and (x.requires_grad or (weight is not None and weight.requires_grad)
                                              or (residual is not None and residual.requires_grad))
    fused = x.is_cuda and training and x.dtype == torch.float32
    if slab_in is not None and slab_in.fwd is not None and not fused:  # no fused consumer: finish the sum
        sp, n = slab_in.take_fwd()
        ext().slab_sum(sp, x, n)
    if slab_in is not None and not fused:
        slab_in.take_stats()  # x is complete; the epilogue statistics go unused
    if x.is_cuda and (training or not needs_grad):  # eval + autograd: differentiable torch path below
        if x.dtype != torch.float32:  # bf16 autocast: normalise in fp32 (stats are fp64 anyway)
            x = x.float()
            residual = residual.float() if residual is not None else None
        if training:
            if link is not None and residual is not None:
                residual = residual.detach()  # its gradient travels through `link`
            return _BNActFn.apply(x, residual, weight, bias, running_mean, running_var, nbt, part, eps,
                                  momentum, relu, single, link, slab_in, grad_slab)
        y = torch.empty_like(x := x.contiguous())
        C = x.shape[1]
        sm = torch.empty(C, device=x.device)
        si = torch.empty(C, device=x.device)
        ext().bn_fwd(x, residual.contiguous() if residual is not None else None, y, weight, bias, running_mean,
                     running_var, None, sm, si, part, float(eps), 0.0, bool(relu), False, False)
        return y
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if training and nbt is not None:
        nbt.add_(1)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class BatchNormAct2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` with optional fused residual add and ReLU (same state_dict)."""

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1, **kw):
        super().__init__(num_features, eps=eps, momentum=momentum, **kw)
        # per-(channel, slice) fp64 partials: C * S * 2 with S <= ceil(1024 / C) (bn_slices)
        self.register_buffer("_part", torch.zeros((num_features + 1024) * 2, dtype=torch.float64),
                             persistent=False)
        # single-launch small-map kernels (HW <= 16, N <= 512); False: the 3-kernel path (tests)
        self.fused_small = True

    def _ensure_part(self, x: torch.Tensor) -> None:
        """Grow the fp64 partial-sum scratch to what this input shape needs (first call for
        a shape happens eagerly — warm-up — never inside a graph capture)."""
        key = (x.shape[0], x.shape[1], x.numel() // max(1, x.shape[0] * x.shape[1]))
        if key != getattr(self, "_part_key", None):
            need = int(ext().bn_part_numel(*key))
            if self._part.numel() < need or self._part.device != x.device:
                self._part = torch.zeros(need, dtype=torch.float64, device=x.device)
            self._part_key = key

    def relu_maxpool(self, x: torch.Tensor, pool: nn.Module, slab_in=None) -> Optional[torch.Tensor]:
        """``pool(relu(self(x)))`` in one pass for a training ``MaxPool2d(3, 2, 1)`` on device
        (the ResNet stem tail; the BN output is never stored), or None where the fused kernel
        does not apply (the caller runs the two modules)."""
        k, st, p = pool.kernel_size, pool.stride, pool.padding
        if not (STEM_POOL and self.training and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
                and torch.is_grad_enabled() and self.affine and self.track_running_stats
                and self.momentum is not None and (slab_in is None or slab_in.fwd is None)
                and isinstance(pool, nn.MaxPool2d) and k in (3, (3, 3)) and st in (2, (2, 2))
                and p in (1, (1, 1)) and pool.dilation in (1, (1, 1)) and not pool.ceil_mode
                and not pool.return_indices and (x.shape[2] * x.shape[3]) % 4 == 0):
            return None
        N, C = x.shape[:2]
        if not ext().bn_two_kernel_path(N, C, x.shape[2] * x.shape[3], self.fused_small):
            return None
        self._ensure_part(x)
        return _BNReluPoolFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                                   self.num_batches_tracked, self._part, self.eps, self.momentum, self.fused_small,
                                   slab_in)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, relu: bool = False, link=None,
                slab_in=None, grad_slab=None):
        """``link`` (ops/gradlink.GradLink, training on device only): deposit the residual's
        gradient there instead of returning it (the caller's conv absorbs it).
        ``slab_in`` / ``grad_slab`` (ops/slablink.SlabLink): x / the gradient of the output
        may arrive as a direct conv's unsummed split-K slabs (summed inside the BN kernel)."""
        if slab_in is not None and slab_in.fwd is not None and (
                self.momentum is None or not self.track_running_stats):
            sp, n = slab_in.take_fwd()
            ext().slab_sum(sp, x, n)
        if slab_in is not None and (self.momentum is None or not self.track_running_stats):
            slab_in.take_stats()
        if self.momentum is None or not self.track_running_stats:
            y = super().forward(x)
            if residual is not None:
                y = y + residual
            return F.relu(y) if relu else y
        training = self.training
        if x.is_cuda:
            self._ensure_part(x)
        return bn_act(x, self.weight, self.bias, self.running_mean, self.running_var,
                      self.num_batches_tracked if training else None, self._part, training, self.momentum,
                      self.eps, residual, relu, x.is_cuda and self.fused_small, link, slab_in, grad_slab)
