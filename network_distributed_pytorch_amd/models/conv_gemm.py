"""Small-spatial convolutions as exact dense GEMMs ("Toeplitz" convolution).

ResNet on 32x32 inputs runs layer3 / layer4 at 4x4 -> 2x2 -> 1x1 feature maps.  There,
MIOpen's fp32 Winograd / implicit-GEMM kernels work on mostly-padding tiles: a 3x3 conv on
a 1x1 map is really a 512x512 matrix product (8 of its 9 taps only ever see padding), yet
it costs ~125 µs fwd+bwd per layer on MI355X (tools/conv_bench.py, profiles/).

For an input of C x H x W with H*W small, the convolution is a linear map
    out.view(B, Co*OH*OW) = x.view(B, C*H*W) @ W_big,
where W_big[(ci,ih,iw), (co,oh,ow)] = W[co, ci, ih - oh*s + p, iw - ow*s + p] (0 outside
the kernel).  Both views are plain NCHW, so forward, grad-input and grad-weight are three
hipBLASLt GEMMs; W_big is built from W and grad-W is folded back from grad-W_big by two
gfx950 kernels (csrc/conv.hip) with a fixed-order sum (deterministic, no atomics).  Only the taps that can ever touch real
pixels cost FLOPs.  On device the stride of a 1x1 strided conv stays inside W_big; on CPU
the input is subsampled first.

``GemmConv2d`` is a drop-in ``nn.Conv2d`` (same parameters / state_dict) that picks, per
input geometry, the fastest native path:
  1. a direct fp32-MFMA kernel (csrc/conv.hip via ops/conv.py) for the ResNet CIFAR shapes
     it covers (stem 7x7/2 on 32x32, 3x3 on 8x8 and 4x4, 3x3/2 8x8->4x4);
  2. the strided / tabled MFMA GEMM kernel (csrc/tgemm.hip via ops/tgconv.py): 1x1 stride-1
     convs on any power-of-two map;
  3. the hipBLASLt Toeplitz GEMM form for the layer3 / layer4 small maps (``NDP_FUSION_OFF=tgemm``
     sends the 1x1 convs there too), and the CPU path;
  4. MIOpen otherwise.
(Round 4's compile-time pair-list small-map kernels were correct but lost to the hipBLASLt
Toeplitz GEMMs in the step — profiles/r4/smallconv.md — and were removed in round 5.)
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import gradfinish
from ..ops._ext import ext
from ..ops.conv import DirectConvFn, direct_plan, direct_plan_padded
from ..ops.gradarena import grad_buffer
from ..ops.gradlink import InjectGrad
from ..ops.tgconv import TgConvFn, tg_plan

__all__ = ["GemmConv2d", "ToeplitzBank", "toeplitz_maps", "eligible"]


def eligible(h: int, w: int, oh: int, ow: int) -> bool:
    return h * w <= 16 and oh * ow <= 4


def toeplitz_maps(C: int, H: int, W: int, Co: int, KH: int, KW: int, s: int, p: int):
    """Index maps for W_big (K x N) and for gathering grad-W back (numel(W) x R)."""
    OH = (H + 2 * p - KH) // s + 1
    OW = (W + 2 * p - KW) // s + 1
    K, N = C * H * W, Co * OH * OW
    nw = Co * C * KH * KW
    co, ci, kh, kw, oh, ow = torch.meshgrid(torch.arange(Co), torch.arange(C), torch.arange(KH), torch.arange(KW),
                                            torch.arange(OH), torch.arange(OW), indexing="ij")
    ih = oh * s - p + kh
    iw = ow * s - p + kw
    ok = (ih >= 0) & (ih < H) & (iw >= 0) & (iw < W)
    widx = ((co * C + ci) * KH + kh) * KW + kw
    row = (ci * H + ih.clamp(0, H - 1)) * W + iw.clamp(0, W - 1)
    col = (co * OH + oh) * OW + ow
    flat = row * N + col
    src = torch.full((K * N,), nw, dtype=torch.long)            # nw -> the appended zero
    src[flat[ok]] = widx[ok]
    # grad-W: every tap lists the W_big positions it was copied to (<= OH*OW of them)
    R = OH * OW
    dst = torch.where(ok, flat, torch.full_like(flat, K * N))   # K*N -> appended zero
    dst = dst.reshape(nw, R)
    return src.view(K, N), dst, (OH, OW)


class ToeplitzBank:
    """Persistent W_big^T buffers of every Toeplitz layer of one model, (re)built by ONE
    launch per forward pass (csrc/conv.hip toeplitz_expand_many) instead of one expand
    kernel per layer.

    Layers join the bank on their first device forward (eager: warm-up, never inside a
    capture) and are expanded on their own that time.  Afterwards the first member to run
    in a pass — forward order is fixed — expands every member; the others reuse their
    buffer.  Valid because weights only change between passes (optimizer step); a
    ``w_big`` saved for backward is rebuilt by the NEXT forward, i.e. after that backward.
    """

    MAX_EXPAND = 24  # csrc/ndp_kernels.h kMaxExpand

    def __init__(self):
        self.members: list = []  # [(layer, geom, w_big)]
        self._index: dict = {}

    def get(self, layer, weight: torch.Tensor, geom: tuple, n: int, k: int) -> torch.Tensor:
        key = id(layer)
        i = self._index.get(key)
        if i is None or self.members[i][1] != geom or self.members[i][2].device != weight.device:
            assert not torch.cuda.is_current_stream_capturing(), "Toeplitz bank grows during capture"
            w_big = torch.empty(n, k, device=weight.device, dtype=torch.float32)
            ext().toeplitz_expand(weight.contiguous(), w_big, list(geom))
            if i is None:
                self._index[key] = len(self.members)
                self.members.append((layer, geom, w_big))
            else:
                self.members[i] = (layer, geom, w_big)
            return w_big
        if i == 0:  # <= MAX_EXPAND layers per launch (kernel-argument table)
            batch = [(m.weight, wb, list(g)) for m, g, wb in self.members]
            for j in range(0, len(batch), self.MAX_EXPAND):
                ext().toeplitz_expand_many(batch[j: j + self.MAX_EXPAND])
        return self.members[i][2]


class _ToeplitzConv(torch.autograd.Function):
    """Device tensors: W_big built / grad-W folded by csrc/conv.hip (index arithmetic, one
    launch each, or one expand launch for a whole :class:`ToeplitzBank`); CPU tensors (fp64
    tests): the same maps as index tensors."""

    @staticmethod
    def forward(ctx, x, weight, src, dst, oh, ow, geom=None, bank=None, layer=None, link=None, branch=None):
        B = x.shape[0]
        co = weight.shape[0]
        X = x.reshape(B, -1)
        if x.is_cuda and geom is not None:  # device: W_big^T [N, K], built by one kernel
            C, H, W = x.shape[1:]
            if bank is not None:
                w_big = bank.get(layer, weight, tuple(geom), co * oh * ow, C * H * W)
            else:
                w_big = torch.empty(co * oh * ow, C * H * W, device=x.device, dtype=x.dtype)
                ext().toeplitz_expand(weight.contiguous(), w_big, list(geom))
            out = X @ w_big.t()
        else:
            w_ext = torch.cat([weight.reshape(-1), weight.new_zeros(1)])
            w_big = w_ext[src]                                    # [K, N]
            out = X @ w_big
        ctx.save_for_backward(X, w_big, dst)
        ctx.geom = geom
        ctx.weight = weight  # the Parameter: a deferred fold writes its adopted .grad
        ctx.link = link      # ops/gradlink.py: residual-branch gradient, folded in by addmm
        ctx.branch = branch if (branch is not None and x.is_cuda and geom is not None) else None
        if ctx.branch is not None:
            ctx.branch.join()  # ops/gradlink.BranchLink: grad-x shared with a sibling conv
        ctx.x_shape = x.shape
        ctx.w_shape = weight.shape
        return out.view(B, co, oh, ow)

    @staticmethod
    def backward(ctx, g):
        X, w_big, dst = ctx.saved_tensors
        G = g.reshape(g.shape[0], -1)
        dev = G.is_cuda and ctx.geom is not None
        dx = dw = None
        if dev:  # grad-W: GEMM now, the fold in gradfinish's one batched launch
            if ctx.needs_input_grad[1]:
                dw = grad_buffer(ctx.weight)  # the dense arm's arena slice when registered
                dwt = torch.empty(w_big.shape, device=G.device, dtype=G.dtype)
                torch.mm(G.t(), X, out=dwt)                       # [N, K]
                if gradfinish.can_defer(ctx.weight):
                    gradfinish.defer_fold(dwt, dw, ctx.geom)
                else:
                    ext().toeplitz_fold(dwt, dw, list(ctx.geom))
            if ctx.needs_input_grad[0]:
                addend = ctx.link.take() if ctx.link is not None else None
                br = ctx.branch if ctx.branch is not None and ctx.branch.active() else None
                if br is not None:
                    other = br.take()
                    if addend is None:
                        addend = other
                    elif other is not None:
                        addend = addend + other
                if addend is not None:  # dx = addend + G @ W_big in one GEMM (beta = 1), in place:
                    # the addend is a gradient buffer nothing else reads (no copy of it into dx)
                    dx = addend.reshape(G.shape[0], -1).addmm_(G, w_big).view(ctx.x_shape)
                else:
                    dx = (G @ w_big).view(ctx.x_shape)
                    if br is not None and other is None:  # first of the two: the sibling adds onto it
                        br.put(dx)
                        dx = None
            return dx, dw, None, None, None, None, None, None, None, None, None
        if ctx.needs_input_grad[0]:
            dx = (G @ w_big.t()).view(ctx.x_shape)
        if ctx.needs_input_grad[1]:
            dw_big = X.t() @ G                                    # [K, N]
            ext_ = torch.cat([dw_big.reshape(-1), dw_big.new_zeros(1)])
            dw = ext_[dst].sum(-1).view(ctx.w_shape)              # fixed-order, deterministic
        return dx, dw, None, None, None, None, None, None, None, None, None


class GemmConv2d(nn.Conv2d):
    """``nn.Conv2d`` that runs small-spatial cases as exact hipBLASLt GEMMs."""

    def __init__(self, *a, gemm: bool = True, direct: bool = True, **kw):
        super().__init__(*a, **kw)
        self.gemm = gemm
        self.direct = direct
        self._maps: Dict[Tuple, tuple] = {}
        self.bank: "ToeplitzBank | None" = None  # set by the owning model (one expand launch per pass)
        self.wbank = None  # ops/conv.WinoBank, set by the owning model (one Winograd transform launch per pass)

    def _plan(self, x):
        C, H, W = x.shape[1:]
        kh, kw = self.kernel_size
        s, p = self.stride[0], self.padding[0]
        sub = 1
        # 1x1 strided on CPU: subsample, then stride 1.  On device the stride stays inside
        # W_big (the expand kernel handles it): no slice + contiguous forward, no
        # zero-fill + strided-copy pairs in backward (4 ATen launches per downsample).
        if kh == 1 and kw == 1 and p == 0 and s > 1 and not x.is_cuda:
            sub, s = s, 1
            H, W = (H + sub - 1) // sub, (W + sub - 1) // sub
        key = (C, H, W, x.device, sub)
        if key not in self._maps:
            geom = (C, H, W, self.out_channels, kh, kw, s, p)
            oh = (H + 2 * p - kh) // s + 1
            ow = (W + 2 * p - kw) // s + 1
            if x.is_cuda:  # native expand / fold: no index maps needed
                self._maps[key] = (None, None, oh, ow, sub, geom)
            else:
                src, dst, _ = toeplitz_maps(C, H, W, self.out_channels, kh, kw, s, p)
                self._maps[key] = (src, dst, oh, ow, sub, None)
        return self._maps[key]

    def forward(self, x, link=None, slab_out=None, grad_slab=None, branch=None):
        """``link`` (ops/gradlink.GradLink): a residual-branch gradient to add into this
        conv's grad-x (fused into the kernel / GEMM where the path allows).
        ``slab_out`` / ``grad_slab`` (ops/slablink.SlabLink, direct kernels only): the
        forward / grad-x split-K slabs go to the neighbouring fused BN instead of a sum
        launch (other paths leave the links empty).  ``branch`` (ops/gradlink.BranchLink):
        grad-x shared with a sibling conv of the same input."""
        if not (self.gemm and x.is_cuda and self.groups == 1 and self.dilation == (1, 1) and self.bias is None
                and self.stride[0] == self.stride[1] and self.padding[0] == self.padding[1]
                and self.padding_mode == "zeros" and x.dtype == torch.float32):
            return super().forward(InjectGrad.apply(x, link) if link is not None else x)
        H, W = x.shape[2:]
        kh, kw = self.kernel_size
        s, p = self.stride[0], self.padding[0]
        if self.direct:
            plan = direct_plan(x, self.weight, s, p)
            if plan is not None:
                return DirectConvFn.apply(x, self.weight, plan, link, slab_out, grad_slab, branch, self.wbank)
            padded = direct_plan_padded(x, self.weight, s, p)
            if padded is not None:  # ragged batch: zero-padded images, same kernels (links left empty)
                plan, Bp = padded
                B = x.shape[0]
                xi = InjectGrad.apply(x, link) if link is not None else x
                xp = torch.cat([xi, xi.new_zeros((Bp - B,) + tuple(x.shape[1:]))])
                return DirectConvFn.apply(xp, self.weight, plan, None, None, None)[:B]
            tplan = tg_plan(x, self.weight, s, p)
            if tplan is not None:  # pointwise 1x1 / small-map tabled GEMM (csrc/tgemm.hip)
                return TgConvFn.apply(x, self.weight, tplan, link, branch, slab_out, grad_slab)
        oh = (H + 2 * p - kh) // s + 1
        ow = (W + 2 * p - kw) // s + 1
        if not eligible(H, W, oh, ow):
            return super().forward(InjectGrad.apply(x, link) if link is not None else x)
        src, dst, oh2, ow2, sub, geom = self._plan(x)
        if sub > 1:
            x = x[:, :, ::sub, ::sub]
        if link is not None and geom is None:  # CPU index-map path: plain add in backward
            x, link = InjectGrad.apply(x, link), None
        return _ToeplitzConv.apply(x.contiguous(), self.weight, src, dst, oh2, ow2, geom, self.bank, self, link,
                                   branch)
