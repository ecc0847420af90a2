"""Native ops: flat-arena / multi-tensor kernels with device dispatch.

Device tensors -> hand-written gfx950 HIP kernels (``_C``); CPU tensors -> pure torch.
The PowerSGD grouped kernels are driven from
:mod:`network_distributed_pytorch_amd.parallel.powersgd` through the plan tables.
"""
from __future__ import annotations

from typing import Sequence

import torch

from ._ext import ext, extension_path, native_available  # noqa: F401

__all__ = [
    "ext",
    "native_available",
    "extension_path",
    "add",
    "sgd_momentum_",
    "seg_copy",
    "delay_ns",
    "checksum",
]


def add(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out = a + b (EF pack, ddp_powersgd_guide_cifar10/ddp_init.py:156-157)."""
    if out.is_cuda:
        ext().add(a, b, out)
    else:
        torch.add(a, b, out=out)
    return out


def sgd_momentum_(x: torch.Tensor, g: torch.Tensor, buf: torch.Tensor, lr: float, momentum: float,
                  div: float = 1.0) -> None:
    """Flat-arena ``torch.optim.SGD(momentum)`` step with the all-reduce mean folded in.

    Matches ``b = mu*b + g/div ; x -= lr*b`` with a zero-initialised buffer, which is the
    reference's first-step ``buf = g.clone()`` (ddp_guide_cifar10/ddp_init.py:111,125).
    """
    if x.is_cuda:
        ext().sgd_momentum(x, g, buf, float(lr), float(momentum), float(div))
    else:
        gg = g / div if div != 1.0 else g
        buf.mul_(momentum).add_(gg)
        x.add_(buf, alpha=-lr)


def seg_copy(specs: Sequence[tuple], device: torch.device) -> "SegPlan":
    """Build a reusable multi-tensor reduce-copy table (see :class:`SegPlan`)."""
    return SegPlan(specs, device)


class SegPlan:
    """One-launch multi-tensor reduce-copy: ``dst_i = (sum_c src_i[c*stride_i:]) / div_i``.

    ``specs`` = list of (src_tensor, dst_tensor, chunks, stride, div); src/dst are flat
    float32 tensors (views are fine).  On device the table is uploaded once and the whole
    list is ONE kernel launch; the tensors must stay alive and keep their storage.
    """

    def __init__(self, specs: Sequence[tuple], device: torch.device):
        self.specs = list(specs)
        self.device = torch.device(device)
        self._dev = None
        if self.device.type == "cuda" and self.specs:
            rows = []
            for src, dst, chunks, stride, div in self.specs:
                rows.append((src.data_ptr(), dst.data_ptr(), dst.numel(), int(stride), int(chunks), float(div)))
            ent, prefix, n_ent, n_blocks = ext().make_seg_table(rows)
            self._dev = (ent.to(self.device), prefix.to(self.device), int(n_ent), int(n_blocks))

    def run(self) -> None:
        if not self.specs:
            return
        if self._dev is not None:
            ent, prefix, n_ent, n_blocks = self._dev
            ext().seg_reduce(ent, prefix, n_ent, n_blocks)
            return
        for src, dst, chunks, stride, div in self.specs:
            n = dst.numel()
            acc = src[:n].clone()
            for c in range(1, chunks):
                acc += src[c * stride: c * stride + n]
            if div != 1.0:
                acc /= div
            dst.copy_(acc.view_as(dst))


def delay_ns(ns: int) -> None:
    """Stall the current HIP stream for ``ns`` wall nanoseconds (link emulation)."""
    if ns > 0:
        ext().delay_ns(int(ns))


def checksum(x: torch.Tensor) -> float:
    """Deterministic fp64 checksum of a flat float32 tensor (replica-divergence detector)."""
    if x.is_cuda:
        out = torch.empty(257, dtype=torch.float64, device=x.device)
        ext().checksum(x.reshape(-1), out)
        return float(out[0].item())
    return float(x.double().sum().item())
