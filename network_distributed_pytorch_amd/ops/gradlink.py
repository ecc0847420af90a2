"""Hand a residual block's identity-branch gradient to the conv that can absorb it.

``y = relu(bn2(conv2(h)) + x)`` with ``h = relu(bn1(conv1(x)))``: autograd would compute
``d(identity)`` in the BN2 backward and ``d(conv1 input)`` in conv1's grad-x, then add them
in a separate elementwise launch (9 per ResNet-18 backward).  With a :class:`GradLink` the
fused BN2 backward deposits its residual gradient here instead of returning it (the
residual is passed detached), and conv1's backward — which always runs after BN2's,
being upstream of it on the same path — folds it into its grad-x: the direct conv kernels'
epilogue / split-K sum (``addend``), or ``addmm``'s beta for the Toeplitz GEMM.
"""
from __future__ import annotations

from typing import Optional

import torch

__all__ = ["GradLink", "InjectGrad", "BranchLink"]


class GradLink:
    __slots__ = ("grad",)

    def __init__(self):
        self.grad: Optional[torch.Tensor] = None

    def put(self, g: torch.Tensor) -> None:
        assert self.grad is None, "GradLink: residual gradient deposited twice"
        self.grad = g

    def take(self) -> Optional[torch.Tensor]:
        g, self.grad = self.grad, None
        return g


class InjectGrad(torch.autograd.Function):
    """Identity forward; backward adds the link's gradient (fallback for convs whose
    grad-x kernel takes no addend, e.g. MIOpen)."""

    @staticmethod
    def forward(ctx, x, link):
        ctx.link = link
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        extra = ctx.link.take()
        return (g if extra is None else g + extra), None


class BranchLink:
    """Two convolutions reading the same input — a downsample block's conv1 and its 1x1
    downsample: autograd would sum their two grad-x tensors with an elementwise add launch.
    Every conv that takes the link in forward ``join``s it; in backward (either order) the
    first member deposits its grad-x and returns None (a zero gradient to autograd), the
    second accumulates its product onto the deposit in place (``addmm_``, beta = 1) and
    returns the sum.  With fewer than two members the link is inert."""

    __slots__ = ("members", "direct", "grad")

    def __init__(self):
        self.members = 0
        self.direct = 0  # members on the direct conv kernels (ops/conv.DirectConvFn)
        self.grad = None  # the first member's grad-x, or (direct pair) its deferred grad-x kernel

    def join(self, direct: bool = False) -> None:
        self.members += 1
        self.direct += int(direct)

    def active(self) -> bool:
        return self.members == 2

    def all_direct(self) -> bool:
        """Both members are direct convs: the first may deposit a callable that runs its
        grad-x kernel with the second's grad-x as the epilogue addend."""
        return self.direct == 2

    def put(self, g) -> None:
        assert self.grad is None, "BranchLink: grad-x deposited twice"
        self.grad = g

    def take(self):
        g, self.grad = self.grad, None
        return g
