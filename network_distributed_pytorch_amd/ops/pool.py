"""Deterministic max-pool 2-D (gfx950 kernels, csrc/pool.hip) as a drop-in ``nn.MaxPool2d``.

ResNet's stem pool (``MaxPool2d(3, 2, 1)``, torchvision resnet as used by the reference at
ddp_powersgd_guide_cifar10/ddp_init.py:111) runs in PyTorch-ROCm as a forward that writes
int64 indices and an atomic-scatter backward into a zero-filled gradient.  The native pair
stores a uint8 window offset and gathers the gradient per input element in a fixed order
(no atomics, no fill; bitwise reproducible).  CPU tensors and configurations the kernel
does not cover (dilation, ceil_mode, return_indices, non-fp32) use ``nn.MaxPool2d``.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ._ext import ext

__all__ = ["MaxPool2d", "max_pool2d"]


def _out(n: int, k: int, s: int, p: int) -> int:
    return (n + 2 * p - k) // s + 1


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        x = x.contiguous()
        N, C, H, W = x.shape
        OH, OW = _out(H, k, s, p), _out(W, k, s, p)
        y = torch.empty((N, C, OH, OW), device=x.device, dtype=x.dtype)
        idx = torch.empty((N, C, OH, OW), device=x.device, dtype=torch.uint8)
        ext().maxpool_fwd(x, y, idx, k, s, p)
        ctx.save_for_backward(idx)
        ctx.geom = (k, s, p, H, W)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        k, s, p, H, W = ctx.geom
        dy = dy.contiguous()
        dx = torch.empty((dy.shape[0], dy.shape[1], H, W), device=dy.device, dtype=dy.dtype)
        ext().maxpool_bwd(dy, idx, dx, k, s, p)
        return dx, None, None, None


def _single(v) -> int:
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            return -1
        v = v[0]
    return int(v)


def max_pool2d(x: torch.Tensor, kernel_size, stride=None, padding=0) -> torch.Tensor:
    k = _single(kernel_size)
    s = _single(stride if stride is not None else kernel_size)
    p = _single(padding)
    native = (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and k > 0 and s > 0 and p >= 0
              and 2 * p <= k and k * k <= 256)
    if not native:
        return torch.nn.functional.max_pool2d(x, kernel_size, stride, padding)
    return _MaxPoolFn.apply(x, k, s, p)


class MaxPool2d(nn.MaxPool2d):
    """``nn.MaxPool2d`` whose square, undilated, floor-mode fp32 device case runs natively."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if (x.is_cuda and not self.return_indices and not self.ceil_mode and _single(self.dilation) == 1):
            return max_pool2d(x, self.kernel_size, self.stride, self.padding)
        return super().forward(x)
