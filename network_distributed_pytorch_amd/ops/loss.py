"""Fused softmax cross-entropy on gfx950 (csrc/loss.hip), a drop-in for
``torch.nn.CrossEntropyLoss()`` / ``F.cross_entropy`` with the reference's settings (mean
reduction, ``ignore_index=-100``, no class weights, no label smoothing).

The reference computes its training loss with ``nn.CrossEntropyLoss`` (e.g.
ddp_powersgd_guide_cifar10/ddp_init.py:145; HF DistilBERT's classification head for the
IMDb workload).  PyTorch-ROCm lowers that to log_softmax + nll_loss forward and a zero fill
+ nll_loss_backward + log_softmax_backward: 5 launches per step, ~30 µs of a ResNet-18
step at per-GPU batch 64 (profiles/r2/).  Here it is one forward launch — row losses, the
saved gradient ``softmax - onehot`` and a fixed-order mean by the last workgroup — and one
backward launch that scales the saved gradient.  CPU tensors and other settings fall back
to ``F.cross_entropy``; on device the native path is required (no silent fallback).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ext
from ..knobs import fusion_on

__all__ = ["cross_entropy", "CrossEntropyLoss"]

_CTR: dict = {}
_ENABLED = fusion_on("fused_ce")  # =0: PyTorch-ROCm's loss kernels (A/B)


def _counter(device: torch.device) -> torch.Tensor:
    """The kernel's last-workgroup counter, re-armed to 0 by every launch.  One per device:
    per-stream counters would be created inside a graph capture (the warm-up runs on another
    stream) and cost a memset node per replay; the framework never runs two losses of one
    device concurrently."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    c = _CTR.get(idx)
    if c is None:  # first use is eager (warm-up), never inside a capture
        c = _CTR[idx] = torch.zeros(1, dtype=torch.int32, device=device)
    return c


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, acc=None):
        x = logits.contiguous()
        t = target.contiguous()
        dl = torch.empty_like(x)
        scratch = torch.empty(x.shape[0] + 1, device=x.device, dtype=torch.float32)
        loss = torch.empty((), device=x.device, dtype=torch.float32)
        ext().ce_fwd(x, t, dl, scratch, loss, _counter(x.device), int(ignore_index), acc)
        ctx.save_for_backward(dl, scratch)
        return loss

    @staticmethod
    def backward(ctx, g):
        dl, scratch = ctx.saved_tensors
        dx = torch.empty_like(dl)
        ext().ce_bwd(dl, g.reshape(1).contiguous().float(), scratch, dx)
        return dx, None, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100,
                  accumulate: "torch.Tensor | None" = None) -> torch.Tensor:
    """``accumulate`` (optional one-element fp32 tensor): ``accumulate += loss`` as well (a
    running loss sum for logging; inside the kernel on device, no separate add launch)."""
    if (_ENABLED and logits.is_cuda and logits.dim() == 2 and logits.dtype == torch.float32 and target.dtype == torch.int64
            and target.dim() == 1 and logits.shape[0] >= 1):
        return _CrossEntropyFn.apply(logits, target, ignore_index, accumulate)
    loss = F.cross_entropy(logits, target, ignore_index=ignore_index)
    if accumulate is not None:
        accumulate.add_(loss.detach())
    return loss


class CrossEntropyLoss(nn.CrossEntropyLoss):
    """``nn.CrossEntropyLoss`` whose default configuration runs the fused kernel on device."""

    # optional running loss sum (``cross_entropy(accumulate=)``), e.g. the trainer's epoch loss
    accumulate: "torch.Tensor | None" = None

    def forward(self, input: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if (self.weight is None and self.reduction == "mean" and self.label_smoothing == 0.0):
            return cross_entropy(input, target, self.ignore_index, self.accumulate)
        loss = super().forward(input, target)
        if self.accumulate is not None:
            self.accumulate.add_(loss.detach())
        return loss
