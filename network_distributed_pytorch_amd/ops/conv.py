"""Direct fp32-MFMA convolutions (csrc/conv.hip) for ResNet's CIFAR-shape layers.

``conv2d_direct(x, weight, stride, padding)`` runs forward, grad-input and grad-weight on
hand-written gfx950 kernels for the shape classes the extension reports through
``conv_plan`` (ResNet stem 7x7/2 on 32x32, layer1 3x3 on 8x8, layer2 3x3 on 4x4, its
strided 8x8->4x4 entry conv and its 1x1/2 downsample).  Grad-input of the strided 3x3 class
runs natively as the layer1 grad-x kernel on the zero-inserted dY (zeros from the LDS staging;
exact; MIOpen's find-database-dependent algorithm for it was found non-deterministic and
NaN-producing under hipGraph capture);  the 1x1/2
downsample's grad-input is the transposed 1x1 product written to the even pixels; the stem's
input never needs a gradient.
:func:`direct_plan` returns None for every other geometry, so callers keep their MIOpen /
Toeplitz paths there.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from . import gradfinish
from ._ext import ext
from .gradarena import grad_buffer
from ..knobs import fusion_on

__all__ = ["direct_plan", "conv2d_direct", "DirectConvFn", "WinoBank", "set_winograd", "hold_forward", "flush_forward"]

_PLANS: dict = {}
_STATS: dict = {}

# BatchNorm statistics from the forward epilogue where the consuming BN takes the large-map
# path (stem, layer1; ops/slablink.py).  NDP_FUSION_OFF=conv_bnstats restores the BN statistics pass.
CONV_BN_STATS = fusion_on("conv_bnstats")
# layer1 Winograd grad-x + grad-W of one conv in one launch (csrc/winograd.hip wino_bwd_pair_kernel)
_PAIR = fusion_on("wino_pair")
# a downsample block's 1x1/2 forward held for conv1's launch (csrc/conv.hip ds_fwd_pair_kernel)
_DS_FWD_PAIR = fusion_on("ds_fwd_pair")
_HOLD_FWD = [False]
_HELD: list = []


class hold_forward:
    """Within the block, a direct 1x1 stride-2 forward may be held back by the extension and run
    in the same launch as the next 3x3 stride-2 forward of the same input (the downsample block's
    conv1); :func:`flush_forward` launches one that was not taken.  Used by models/resnet.py."""

    def __init__(self, on: bool):
        self.on = bool(on) and _DS_FWD_PAIR

    def __enter__(self):
        _HOLD_FWD[0] = self.on
        return self

    def __exit__(self, *exc):
        _HOLD_FWD[0] = False
        return False


def flush_forward() -> None:
    ext().conv_flush_pending_fwd()
    _HELD.clear()  # every held launch is enqueued: its scratch may be reused by later launches


_WINO: dict = {}


class WinoBank:
    """Winograd weight transforms (csrc/winograd.hip, forward + grad-x layouts) of every Winograd
    layer of one model, rebuilt by ONE launch per forward pass instead of one per layer — the
    scheme of models/conv_gemm.ToeplitzBank: layers join on their first device forward (eager
    warm-up, never inside a capture); afterwards the first member to run in a pass transforms
    every member.  Valid because weights change only between passes (optimizer step); a
    transform saved for backward is rebuilt by the NEXT forward.

    Which layers take the Winograd path depends on the batch size (``wino_dirs``), so "the
    first member of a pass" is recorded per batch size (forward order is fixed, so for one batch
    size it is always the same layer), not taken to be member 0: in a Bottleneck ResNet at
    per-GPU batch 20 the first Winograd layer is layer2.0.conv2, and a refresh tied to member 0
    would leave it one step stale."""

    MAX = 16  # csrc/ndp_kernels.h kMaxWino

    def __init__(self):
        self.members: list = []  # [(weight Parameter, u)]
        self._index: dict = {}
        self._lead: dict = {}  # batch size -> index of the first member to run in a pass

    def get(self, weight: torch.Tensor, batch: int) -> torch.Tensor:
        key = id(weight)
        i = self._index.get(key)
        numel = 32 * weight.numel() // 9
        if i is None or self.members[i][1].device != weight.device or self.members[i][1].numel() != numel:
            assert not torch.cuda.is_current_stream_capturing(), "Winograd bank grows during capture"
            u = torch.empty(numel, device=weight.device, dtype=torch.float32)
            ext().wino_weights(weight.contiguous(), u)
            if i is None:
                i = self._index[key] = len(self.members)
                self.members.append((weight, u))
            else:
                self.members[i] = (weight, u)
            self._lead.setdefault(int(batch), i)
            return u
        if self._lead.setdefault(int(batch), i) == i:
            batch_ = [(w, u) for w, u in self.members]
            for j in range(0, len(batch_), self.MAX):
                ext().wino_weights_many(batch_[j: j + self.MAX])
        return self.members[i][1]


def set_winograd(on: bool) -> None:
    """Switch the Winograd kernels on / off (csrc/winograd.hip) and drop every cached decision
    that depends on the switch (plans, Winograd directions, epilogue statistics slices)."""
    ext().wino_set_enabled(bool(on))
    _PLANS.clear()
    _WINO.clear()
    _STATS.clear()


def wino_dirs(geom, B: int) -> Tuple[bool, bool]:
    """(forward, grad-x) of this conv take the Winograd kernel (csrc/winograd.hip)."""
    key = (tuple(geom), int(B))
    if key not in _WINO:
        _WINO[key] = (bool(ext().conv_wino(list(geom), int(B), False)), bool(ext().conv_wino(list(geom), int(B), True)))
    return _WINO[key]


def stats_slices(geom, B: int) -> int:
    """Batch-tile partials of the BN statistics the forward epilogue emits for this conv (0: none)."""
    key = (tuple(geom), int(B))
    if key not in _STATS:
        _STATS[key] = int(ext().conv_stats_slices(list(geom), int(B))) if CONV_BN_STATS else 0
    return _STATS[key]


def direct_plan(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: int) -> Optional[Tuple]:
    """(geom, fwd_imgs, wgrad_imgs, dgrad_direct, fwd_ksplit, dgrad_ksplit) if a direct kernel
    covers this conv at this batch size (the split-K factors and grad-W slice size adapt to
    the batch so that small per-GPU batches still fill the 256 CUs)."""
    if not (x.is_cuda and x.dtype == torch.float32 and weight.dtype == torch.float32 and x.dim() == 4):
        return None
    B, C, H, W = x.shape
    Co, Ci, KH, KW = weight.shape
    if Ci != C:
        return None
    geom = (C, H, W, Co, KH, KW, int(stride), int(padding))
    key = (geom, int(B))
    if key not in _PLANS:
        cls, fi, wi, dd, ksf, ksd = ext().conv_plan(list(geom), int(B))
        _PLANS[key] = None if cls < 0 else (geom, int(fi), int(wi), bool(dd), int(ksf), int(ksd))
    plan = _PLANS[key]
    if plan is None or B % plan[1] or B % plan[2]:
        return None
    return plan


# batch quantum of the direct kernels: images per forward / grad-x workgroup (1 / 2 / 4) and
# per grad-W slice (2 .. 16) always divide 16
_BATCH_QUANT = 16


def direct_plan_padded(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: int) -> Optional[Tuple]:
    """(plan, padded batch) for a batch the direct kernels cannot tile (a ragged last batch:
    B not a multiple of their images per workgroup / slice): the conv then runs on the batch
    zero-padded to a multiple of 16 instead of falling back to another library path (MIOpen's
    algorithm choice is not deterministic run to run).  None if the geometry is not covered."""
    B = x.shape[0]
    Bp = -(-B // _BATCH_QUANT) * _BATCH_QUANT
    if Bp == B or not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4):
        return None
    plan = direct_plan(x.new_empty((Bp,) + tuple(x.shape[1:])), weight, stride, padding)
    return (plan, Bp) if plan is not None else None


class DirectConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, plan, link=None, slab_out=None, grad_slab=None, branch=None, wbank=None):
        """``slab_out`` / ``grad_slab`` (ops/slablink.py): leave the forward / grad-x split-K
        slabs for the fused BN kernel that consumes them instead of summing them here.
        ``branch`` (ops/gradlink.BranchLink): grad-x shared with a sibling conv of the same input
        (a downsample block's conv1 and 1x1 downsample), summed in a kernel epilogue."""
        wparam = weight
        ctx.link = link  # ops/gradlink.py: residual-branch gradient folded into grad-x
        ctx.grad_slab = grad_slab
        ctx.branch = branch
        if branch is not None:
            branch.join(direct=True)
        geom, _, wgrad_imgs, dgrad_direct, ks_fwd, _ = plan
        C, H, W, Co, KH, KW, s, p = geom
        x = x.contiguous()
        weight = weight.contiguous()
        B = x.shape[0]
        OH = (H + 2 * p - KH) // s + 1
        OW = (W + 2 * p - KW) // s + 1
        y = torch.empty(B, Co, OH, OW, device=x.device, dtype=x.dtype)
        part = torch.empty(ks_fwd * y.numel(), device=x.device, dtype=x.dtype) if ks_fwd > 1 else None
        S = stats_slices(geom, B) if slab_out is not None else 0
        stats = torch.empty(Co * S * 2, device=x.device, dtype=torch.float64) if S > 0 else None
        # Winograd layers (csrc/winograd.hip): the weight transform once per pass, shared by the
        # forward and the grad-x launch (saved for backward)
        wf, wd = wino_dirs(geom, B)
        wu = None
        if (wf or wd) and wbank is not None:  # the model's bank: one transform launch per pass
            wu = wbank.get(wparam, B)
        elif wf or wd:
            wu = torch.empty(32 * weight.numel() // 9, device=x.device, dtype=x.dtype)  # fwd + grad-x layouts
            ext().wino_weights(weight, wu)
        left = ext().conv_fwd(x, weight, y, list(geom), part, slab_out is not None and part is not None, stats,
                              wu if wf else None, _HOLD_FWD[0])
        if _HOLD_FWD[0]:  # a held launch still writes its split-K scratch: alive until flush_forward()
            _HELD.append(part)
        ctx.wu = wu if wd else None
        if left > 1:
            slab_out.put_fwd(part, left)  # y is filled by the consuming BN kernel
        if stats is not None:
            slab_out.put_stats(stats, S)  # the consuming BN skips its statistics pass
        ctx.save_for_backward(x, weight)
        ctx.plan = plan
        ctx.weight = wparam  # the Parameter itself: its .grad is where a deferred sum lands
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        geom, _, wgrad_imgs, dgrad_direct, _, ks_dgrad = ctx.plan
        s, p = geom[6], geom[7]
        dy = dy.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[1]:
            B = x.shape[0]
            dw = grad_buffer(ctx.weight, weight)  # the dense arm's arena slice when registered
            part = torch.empty((B // wgrad_imgs) * weight.numel(), device=x.device, dtype=x.dtype)
            if gradfinish.can_defer(ctx.weight):  # slabs now, one batched sum later
                # pair=True: a Winograd-class grad-W waits for this conv's grad-x (below, or in the
                # BranchLink sibling's backward) and both run in one launch (csrc/conv.hip
                # launch_conv_dgrad); one that no grad-x took is launched by gradfinish.flush()
                ext().conv_wgrad(x, dy, part, None, list(geom), _PAIR)
                gradfinish.defer_slab(part, dw, B // wgrad_imgs, keep=(x, dy) if _PAIR else ())
            else:
                ext().conv_wgrad(x, dy, part, dw, list(geom))
        dx = DirectConvFn._grad_x(ctx, dy, x, weight, geom, s, p, dgrad_direct, ks_dgrad)
        return dx, dw, None, None, None, None, None, None

    @staticmethod
    def _grad_x(ctx, dy, x, weight, geom, s, p, dgrad_direct, ks_dgrad):
        dx = None
        addend = ctx.link.take() if ctx.link is not None else None
        if ctx.needs_input_grad[0]:
            grad_slab = ctx.grad_slab
            if ctx.branch is not None and not (ctx.branch.active() and ctx.branch.all_direct()):
                # a sibling outside the link, or one that is not a direct kernel (its grad-x is
                # added later): the previous BN2 must not take this grad-x alone
                grad_slab = None

            def dgrad(addend):
                if not dgrad_direct:
                    dx = torch.ops.aten.convolution_backward(dy, x, weight, None, [s, s], [p, p], [1, 1], False,
                                                             [0, 0], 1, [True, False, False])[0]
                    return dx if addend is None else dx + addend
                dx = torch.empty_like(x)
                part = None
                if ks_dgrad > 1:  # partials in dx layout (the 1x1 stride-2 class: its compact 4x4 map)
                    ups = geom[4] == 1 and geom[6] == 2
                    slab = (dy.numel() // geom[3]) * geom[0] if ups else x.numel()
                    part = torch.empty(ks_dgrad * slab, device=x.device, dtype=x.dtype)
                fuse = addend is not None and _takes_addend(geom)
                if fuse:
                    addend = addend.contiguous()
                # split-K slabs (and the addend, added after them) left to the consuming BN
                defer = grad_slab is not None and part is not None and (addend is None or fuse)
                # unsplit: the consuming BN's backward statistics from this epilogue (ops/slablink.py)
                bn = grad_slab.bn_saved if (grad_slab is not None and part is None and (addend is None or fuse)) \
                    else None
                S = int(ext().conv_dgrad_stats_slices(list(geom), x.shape[0])) if bn is not None else 0
                if S > 0:
                    stats = torch.empty(x.shape[1] * S * 2, device=x.device, dtype=torch.float64)
                    ext().conv_dgrad(dy, weight, dx, list(geom), None, addend if fuse else None, False, stats, *bn,
                                     wino_u=ctx.wu)
                    grad_slab.put_bwd_stats(stats, S)
                    return dx
                left = ext().conv_dgrad(dy, weight, dx, list(geom), part, addend if fuse else None, defer,
                                        wino_u=ctx.wu)
                if left > 1:  # dx stays unwritten: the BN backward sums the slabs (+ the addend)
                    grad_slab.put_bwd(part, left, addend if fuse else None)
                return dx + addend if (addend is not None and not fuse) else dx

            br = ctx.branch if ctx.branch is not None and ctx.branch.active() else None
            other = br.take() if br is not None else None
            if br is not None and other is None and br.all_direct() and addend is None and dgrad_direct \
                    and _takes_addend(geom):
                # first of two direct siblings, and this grad-x kernel can add the sibling's
                # grad-x in its epilogue: run it once the sibling's exists (no add launch)
                br.put(dgrad)
            elif callable(other):  # the sibling waits for this grad-x as its addend
                dx = other(dgrad(addend))
            else:
                if other is not None:
                    addend = other if addend is None else addend + other
                dx = dgrad(addend)
                if br is not None and other is None:  # first of the two: the sibling adds onto it
                    br.put(dx)
                    dx = None
        return dx


def _takes_addend(geom) -> bool:
    """The grad-x kernel adds an addend in its epilogue / split-K sum: every direct class (the
    3x3 ones on their stride-1 / zero-inserted maps, the 1x1 stride-2 ones in the even-pixel
    scatter epilogue, whose odd pixels then carry the addend alone)."""
    return (geom[4] == 3 and geom[5] == 3) or (geom[4] == 1 and geom[5] == 1 and geom[6] == 2)


def conv2d_direct(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: int, plan=None,
                  link=None, slab_out=None, grad_slab=None) -> torch.Tensor:
    plan = plan if plan is not None else direct_plan(x, weight, stride, padding)
    assert plan is not None, "no direct kernel for this convolution"
    return DirectConvFn.apply(x, weight, plan, link, slab_out, grad_slab)
