"""Hand a direct convolution's split-K partial slabs to the fused BN kernel next to it.

At the strong-scaling per-GPU batches (512 / N = 64 ... 256) the direct conv kernels of
ResNet layer1 / layer2 split their reduction over input channels (``conv_ksplit``) to fill
the 256 CUs, and a separate ``conv_slab_sum`` launch adds the slabs.  Every such conv
feeds exactly one BatchNorm: in forward conv -> BN, in backward conv2's grad-x -> the
grad of BN1's output.  With a :class:`SlabLink` the conv leaves its slabs in scratch
(``defer=True``) and the fused single-launch BN kernel sums them while it reads its input
(csrc/batchnorm.hip ``src``), in the same slab order as ``conv_slab_sum`` (bitwise-equal
values): one launch fewer per conv, ~5 µs each on MI355X.  The forward BN also stores the
sum to the conv's output buffer (BN saves its input for backward).  Where no fused BN
kernel covers the shape, ``launch_bn_fwd`` / ``launch_bn_bwd`` run the plain slab sum
themselves first, so a deferred sum is always finished.

A grad-x addend (the residual-branch gradient of ops/gradlink.py) travels with the slabs and
is added after them, as the conv's own split-K sum would; this also links a block's conv1
to the PREVIOUS block's BN2 (models/resnet.py), whose output gradient that grad-x is.

Where the conv runs unsplit and its forward BN takes the two-kernel large-map path (the
ResNet stem and layer1), the link carries the BN's statistics instead: the conv epilogue
emits per-channel, per-batch-tile fp64 sums of its output (csrc/conv.hip ``stats``) and the
BN's apply kernel folds them, so the BN skips its statistics launch and its full read of x.

In backward the same idea runs the other way: a BN whose ReLU output is known deposits
(x, y, mean, invstd) in its gradient link, and the direct conv producing that gradient emits
the BN backward's per-channel partial sums of dz and dz * xhat from its grad-x epilogue.

Only wired inside the fused ResNet blocks (models/resnet.py), where each conv output /
grad-x has exactly that one consumer.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

__all__ = ["SlabLink"]


class SlabLink:
    __slots__ = ("fwd", "bwd", "bwd_add", "stats", "bn_saved", "bstats")

    def __init__(self):
        self.fwd: Optional[Tuple[torch.Tensor, int]] = None  # conv output slabs -> BN forward
        self.bwd: Optional[Tuple[torch.Tensor, int]] = None  # conv grad-x slabs -> BN backward
        self.bwd_add: Optional[torch.Tensor] = None  # the grad-x addend, added after the slabs
        self.stats: Optional[Tuple[torch.Tensor, int]] = None  # conv epilogue BN partial sums [C][S][2]
        # backward: the BN's (x, y, save_mean, save_invstd), deposited by its forward, so the conv
        # producing its output gradient can emit the BN backward's partial sums (bstats)
        self.bn_saved: Optional[tuple] = None
        self.bstats: Optional[Tuple[torch.Tensor, int]] = None

    def put_bwd_stats(self, stats: torch.Tensor, n: int) -> None:
        assert self.bstats is None, "SlabLink: backward statistics deposited twice"
        self.bstats = (stats, int(n))

    def take_bwd_stats(self) -> Tuple[Optional[torch.Tensor], int]:
        v, self.bstats = self.bstats, None
        return v if v is not None else (None, 0)

    def put_stats(self, stats: torch.Tensor, n: int) -> None:
        assert self.stats is None, "SlabLink: statistics deposited twice"
        self.stats = (stats, int(n))

    def take_stats(self) -> Tuple[Optional[torch.Tensor], int]:
        v, self.stats = self.stats, None
        return v if v is not None else (None, 0)

    def put_fwd(self, part: torch.Tensor, n: int) -> None:
        assert self.fwd is None, "SlabLink: forward slabs deposited twice"
        self.fwd = (part, int(n))

    def take_fwd(self) -> Tuple[Optional[torch.Tensor], int]:
        v, self.fwd = self.fwd, None
        return v if v is not None else (None, 0)

    def put_bwd(self, part: torch.Tensor, n: int, addend: Optional[torch.Tensor] = None) -> None:
        assert self.bwd is None, "SlabLink: grad-x slabs deposited twice"
        self.bwd = (part, int(n))
        self.bwd_add = addend

    def take_bwd(self) -> Tuple[Optional[torch.Tensor], int]:
        v, self.bwd = self.bwd, None
        return v if v is not None else (None, 0)

    def take_bwd_add(self) -> Optional[torch.Tensor]:
        """The addend deposited with the grad-x slabs (a residual / sibling gradient the conv's
        split-K sum would have added last), or None; take it with the slabs."""
        a, self.bwd_add = self.bwd_add, None
        return a
