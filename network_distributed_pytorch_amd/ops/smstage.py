"""ResNet layer3 + layer4 (2x2 / 1x1 maps) as ONE autograd node with BatchNorm fused into the
small-map convolutions (csrc/smallconv.hip ``SmOps``).

The reference trains torchvision ResNets (ddp_guide_cifar10/ddp_init.py:108,
ddp_powersgd_guide_cifar10/ddp_init.py:111); on 32x32 inputs their last two stages run on 2x2
and 1x1 maps, where every BatchNorm pass is a latency-bound launch of its own.  Here no
BatchNorm kernel runs between the convolutions of the stage:

forward, per BasicBlock k (c = raw conv outputs, O = block outputs):
  conv1   operand = O_{k-1} computed while it is staged (relu(bn2(c2) + residual), the
          residual itself bn_d(c_d) after a downsample block) and written once (n-tile 0)
          as the materialised block output; epilogue: per-row-tile sum / sum-of-squares of c1
  [ds]    operand = O_{k-1}; epilogue: statistics of c_d
  conv2   operand = relu(bn1(c1)) (bn1 finalized in the prologue from conv1's partial sums);
          epilogue: statistics of c2
  the last block's output: one apply kernel (the stage's only BN pass)
backward, given dO:
  conv2 grad-x / grad-W   operand dc2 = BN2-backward(dO) computed while staged (its dz / dz*xhat
          sums come from the epilogue of the kernel that produced dO); grad-x epilogue: the
          sums of BN1's backward (relu mask recomputed from c1)
  [ds grad-x / grad-W]    operand = BN_d-backward(dO) (same dz, its own x-hat)
  conv1 grad-x / grad-W   operand dc1 = BN1-backward(dh); grad-x epilogue: + the residual
          gradient (dz2 of this block, or the downsample grad-x), then the sums of the previous
          block's BN2 (+ BN_d) backward
so the stage is 2-3 kernels per block in each direction instead of ~2 per conv plus ~2 per BN.
Running statistics, saved mean / invstd, dgamma / dbeta are written by the kernels (the
workgroup at grid origin); parameters / buffers / state_dict are the modules' own.
``NDP_SM_STAGE=0`` keeps the per-module path (still on the small-map convs).  The stage only
runs with the small-map convs on (``NDP_SM=1``, off by default): the fused operand transforms
and epilogue statistics cost more than the BatchNorm launches they replace at these kernel
speeds (profiles/r4/smallconv.md: batch 512 2.51 ms with the stage vs 2.16 without).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from . import gradfinish
from ._ext import ext
from .gradarena import grad_buffer

__all__ = ["stage_blocks", "run_stage", "enabled"]

_ON = os.environ.get("NDP_SM_STAGE", "1") != "0"


def enabled() -> bool:
    return _ON


def _geom(conv, x_shape):
    C, H, W = x_shape[1:]
    kh, kw = conv.kernel_size
    return [C, H, W, conv.out_channels, kh, kw, conv.stride[0], conv.padding[0]]


def _out_hw(g):
    C, H, W, Co, kh, kw, s, p = g
    return (H + 2 * p - kh) // s + 1, (W + 2 * p - kw) // s + 1


def stage_blocks(model, x: torch.Tensor) -> Optional[list]:
    """The BasicBlocks of layer3 + layer4 if the fused stage covers them for input ``x``
    (layer2's output), else None."""
    from . import smconv

    if not (_ON and smconv.enabled() and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and torch.is_grad_enabled()):
        return None
    from ..models.resnet import BasicBlock
    from .batchnorm import BatchNormAct2d

    blocks = list(model.layer3) + list(model.layer4)
    shape = tuple(x.shape)
    X = ext()
    for b in blocks:
        if not isinstance(b, BasicBlock) or not b.fused:
            return None
        convs = [b.conv1, b.conv2] + ([b.downsample[0]] if b.downsample is not None else [])
        bns = [b.bn1, b.bn2] + ([b.downsample[1]] if b.downsample is not None else [])
        if b.downsample is not None and len(b.downsample) != 2:
            return None
        for bn in bns:
            if not (isinstance(bn, BatchNormAct2d) and bn.training and bn.track_running_stats
                    and bn.momentum is not None and bn.affine):
                return None
        for cv in convs:
            if cv.bias is not None or cv.groups != 1 or cv.dilation != (1, 1) or cv.padding_mode != "zeros":
                return None
        g1 = _geom(b.conv1, shape)
        if X.sm_plan(g1, shape[0])[0] < 0:
            return None
        oh, ow = _out_hw(g1)
        mid = (shape[0], b.conv1.out_channels, oh, ow)
        g2 = _geom(b.conv2, mid)
        if X.sm_plan(g2, shape[0])[0] < 0:
            return None
        if b.downsample is not None:
            gd = _geom(b.downsample[0], shape)
            if X.sm_plan(gd, shape[0])[0] < 0 or tuple(_out_hw(gd)) != tuple(_out_hw(g2)):
                return None
        elif tuple(_out_hw(g2)) != shape[2:] or b.conv2.out_channels != shape[1]:
            return None
        shape = (shape[0], b.conv2.out_channels) + tuple(_out_hw(g2))
        if shape[1] % 16:
            return None
    return blocks


def _bn_params(bn):
    return [bn.weight, bn.bias]


def run_stage(blocks, x: torch.Tensor) -> torch.Tensor:
    params: List[torch.Tensor] = []
    for b in blocks:
        params += [b.conv1.weight] + _bn_params(b.bn1) + [b.conv2.weight] + _bn_params(b.bn2)
        if b.downsample is not None:
            params += [b.downsample[0].weight] + _bn_params(b.downsample[1])
    return _StageFn.apply(x, blocks, *params)


def _bnf(bn, part, R, count, sm, si, write_running: bool):
    """Forward BN descriptor: from partial sums (part) or the saved statistics (part None)."""
    d = {"part": part, "R": R, "count": float(count), "gamma": bn.weight.detach(), "beta": bn.bias.detach(),
         "eps": float(bn.eps), "momentum": float(bn.momentum), "save_mean": sm, "save_invstd": si}
    if write_running:
        d.update(rmean=bn.running_mean, rvar=bn.running_var, nbt=bn.num_batches_tracked)
    return d


class _Blk:
    """Per-block saved state of one forward."""
    __slots__ = ("g1", "g2", "gd", "c1", "c2", "cd", "inp", "out", "s1", "s2", "sd", "p1", "p2", "pd", "R1", "R2",
                 "Rd", "count1", "count2")


class _StageFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, blocks, *params):
        X = ext()
        x = x.contiguous()
        B = x.shape[0]
        dev = x.device
        f32 = dict(device=dev, dtype=torch.float32)
        st: List[_Blk] = []
        inp = x          # materialised input of the current block (None until a consumer writes it)
        prev = None      # the previous block's state (its output still virtual)
        for k, b in enumerate(blocks):
            s = _Blk()
            s.g1 = _geom(b.conv1, x.shape if prev is None else prev.c2.shape)
            oh, ow = _out_hw(s.g1)
            C1 = b.conv1.out_channels
            s.c1 = torch.empty(B, C1, oh, ow, **f32)
            s.R1 = int(X.sm_rowtile(s.g1, B, 0))
            s.R1 = (B + s.R1 - 1) // s.R1
            s.p1 = torch.empty(s.R1 * C1 * 2, device=dev, dtype=torch.float64)
            ops = {"emode": 1, "epart": s.p1}
            if prev is not None:  # operand = O_{k-1} = relu(bn2(c2) + residual), written to `mat`
                inp = torch.empty_like(prev.c2)
                ops.update(_fwd_out_ops(prev, blocks[k - 1]))
                ops["mat"] = inp
                act = prev.c2
                prev.out = inp
            else:
                act = inp
            s.inp = inp
            X.sm_fwd_ops(act, b.conv1.weight.detach().contiguous(), s.c1, s.g1, ops)
            s.count1 = B * oh * ow
            s.s1 = (torch.empty(C1, **f32), torch.empty(C1, **f32))
            if b.downsample is not None:
                cvd, bnd = b.downsample[0], b.downsample[1]
                s.gd = _geom(cvd, inp.shape)
                dh, dw = _out_hw(s.gd)
                s.cd = torch.empty(B, cvd.out_channels, dh, dw, **f32)
                rt = int(X.sm_rowtile(s.gd, B, 0))
                s.Rd = (B + rt - 1) // rt
                s.pd = torch.empty(s.Rd * cvd.out_channels * 2, device=dev, dtype=torch.float64)
                X.sm_fwd_ops(inp, cvd.weight.detach().contiguous(), s.cd, s.gd, {"emode": 1, "epart": s.pd})
                s.sd = (torch.empty(cvd.out_channels, **f32), torch.empty(cvd.out_channels, **f32))
            else:
                s.gd = s.cd = s.pd = s.sd = None
                s.Rd = 0
            s.g2 = _geom(b.conv2, s.c1.shape)
            oh2, ow2 = _out_hw(s.g2)
            C2 = b.conv2.out_channels
            s.c2 = torch.empty(B, C2, oh2, ow2, **f32)
            rt = int(X.sm_rowtile(s.g2, B, 0))
            s.R2 = (B + rt - 1) // rt
            s.p2 = torch.empty(s.R2 * C2 * 2, device=dev, dtype=torch.float64)
            ops2 = {"amode": 1, "af": _bnf(b.bn1, s.p1, s.R1, s.count1, s.s1[0], s.s1[1], True),
                    "emode": 1, "epart": s.p2}
            X.sm_fwd_ops(s.c1, b.conv2.weight.detach().contiguous(), s.c2, s.g2, ops2)
            s.count2 = B * oh2 * ow2
            s.s2 = (torch.empty(C2, **f32), torch.empty(C2, **f32))
            s.out = None
            st.append(s)
            prev = s
        # the stage output: the last block's relu(bn2(c2) + residual)
        out = torch.empty_like(prev.c2)
        X.sm_bn_apply(prev.c2, out, _fwd_out_ops(prev, blocks[-1]))
        prev.out = out
        ctx.blocks = blocks
        ctx.st = st
        ctx.save_for_backward(x, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        X = ext()
        blocks, st = ctx.blocks, ctx.st
        saved = ctx.saved_tensors
        params = saved[1:]
        dout = dout.contiguous()
        B = dout.shape[0]
        dev = dout.device
        grads = []  # per block: [dW1, dg1, db1, dW2, dg2, db2, (dWd, dgd, dbd)]
        # BN2 (+ BN_d) backward sums of the last block, from dO
        last, lb = st[-1], blocks[-1]
        Rb = int(X.sm_bstats_rows(B))
        bpart = torch.empty(Rb * last.c2.shape[1] * 4, device=dev, dtype=torch.float64)
        ops = {"epart": bpart, "emask": 1, "emtensor": last.out, "ec": last.c2,
               "ef": _bnf(lb.bn2, None, 0, last.count2, last.s2[0], last.s2[1], False)}
        if last.cd is not None:
            ops.update(eds=1, ecd=last.cd, efd=_bnf(lb.downsample[1], None, 0, last.count2, last.sd[0], last.sd[1],
                                                    False))
        X.sm_bn_bstats(dout, ops)
        bR = Rb
        dO = dout
        per_block = [None] * len(blocks)
        for k in range(len(blocks) - 1, -1, -1):
            b, s = blocks[k], st[k]
            bn1, bn2 = b.bn1, b.bn2
            w1 = b.conv1.weight.detach().contiguous()
            w2 = b.conv2.weight.detach().contiguous()
            dg2, db2 = grad_buffer(bn2.weight), grad_buffer(bn2.bias)
            # ---- conv2: operand dc2 = BN2-backward(dO) ------------------------------------
            g2ops = {"amode": 4, "amask": 1, "mtensor": s.out, "c": s.c2,
                     "ab": {"part": bpart, "R": bR, "j": 1, "count": float(s.count2), "gamma": bn2.weight.detach(),
                            "mean": s.s2[0], "invstd": s.s2[1], "dgamma": dg2, "dbeta": db2}}
            dh = torch.empty_like(s.c1)
            rt = int(X.sm_rowtile(s.g2, B, 1))
            R1b = (B + rt - 1) // rt
            bpart1 = torch.empty(R1b * s.c1.shape[1] * 4, device=dev, dtype=torch.float64)
            f1 = _bnf(bn1, None, 0, s.count1, s.s1[0], s.s1[1], False)
            d2 = dict(g2ops, emode=2, epart=bpart1, emask=2, ec=s.c1, ef=f1)
            X.sm_dgrad_ops(dO, w2, dh, s.g2, d2)
            g2w = dict(g2ops)
            g2w["ab"] = dict(g2ops["ab"], dgamma=None, dbeta=None)
            dW2 = _wgrad(X, s.c1, dO, b.conv2.weight, s.g2, {"amode": 1, "af": f1}, g2w)
            # ---- downsample: operand = BN_d-backward(dO) (dz of BN2, its own x-hat) ------
            dxd = None
            if s.cd is not None:
                bnd = b.downsample[1]
                dgd, dbd = grad_buffer(bnd.weight), grad_buffer(bnd.bias)
                gdops = {"amode": 4, "amask": 1, "mtensor": s.out, "c": s.cd,
                         "ab": {"part": bpart, "R": bR, "j": 2, "count": float(s.count2), "gamma": bnd.weight.detach(),
                                "mean": s.sd[0], "invstd": s.sd[1], "dgamma": dgd, "dbeta": dbd}}
                dxd = torch.empty_like(s.inp)
                X.sm_dgrad_ops(dO, b.downsample[0].weight.detach().contiguous(), dxd, s.gd, gdops)
                gdw = dict(gdops)
                gdw["ab"] = dict(gdops["ab"], dgamma=None, dbeta=None)
                dWd = _wgrad(X, s.inp, dO, b.downsample[0].weight, s.gd, {}, gdw)
            # ---- conv1: operand dc1 = BN1-backward(dh) -------------------------------------
            dg1, db1 = grad_buffer(bn1.weight), grad_buffer(bn1.bias)
            g1ops = {"amode": 4, "amask": 2, "af": f1, "c": s.c1,
                     "ab": {"part": bpart1, "R": R1b, "j": 1, "count": float(s.count1), "gamma": bn1.weight.detach(),
                            "mean": s.s1[0], "invstd": s.s1[1], "dgamma": dg1, "dbeta": db1}}
            dI = torch.empty_like(s.inp)
            d1 = dict(g1ops)
            if dxd is not None:
                d1.update(eadd=1, addend=dxd)
            else:  # identity residual: + dz2 = dO * (O > 0)
                d1.update(eadd=2, addend=dO, addmask=s.out)
            nbpart, nR = None, 0
            if k > 0:  # the previous block's BN2 (+ BN_d) backward sums, from the final dI
                ps, pb = st[k - 1], blocks[k - 1]
                rt = int(X.sm_rowtile(s.g1, B, 1))
                nR = (B + rt - 1) // rt
                nbpart = torch.empty(nR * ps.c2.shape[1] * 4, device=dev, dtype=torch.float64)
                d1.update(emode=2, epart=nbpart, emask=1, emtensor=ps.out, ec=ps.c2,
                          ef=_bnf(pb.bn2, None, 0, ps.count2, ps.s2[0], ps.s2[1], False))
                if ps.cd is not None:
                    d1.update(eds=1, ecd=ps.cd, efd=_bnf(pb.downsample[1], None, 0, ps.count2, ps.sd[0], ps.sd[1],
                                                         False))
            X.sm_dgrad_ops(dh, w1, dI, s.g1, d1)
            g1w = dict(g1ops)
            g1w["ab"] = dict(g1ops["ab"], dgamma=None, dbeta=None)
            dW1 = _wgrad(X, s.inp, dh, b.conv1.weight, s.g1, {}, g1w)
            g = [dW1, dg1, db1, dW2, dg2, db2]
            if s.cd is not None:
                g += [dWd, dgd, dbd]
            per_block[k] = g
            dO, bpart, bR = dI, nbpart, nR
        for g in per_block:
            grads += g
        del params
        return (dO, None) + tuple(grads)


def _fwd_out_ops(s, b):
    """Operand transform computing block s's output relu(bn2(c2) + residual) (amode 2 / 3);
    the consumer finalizes (and records) bn2 / bn_d from the conv epilogues' partial sums."""
    ops = {"af": _bnf(b.bn2, s.p2, s.R2, s.count2, s.s2[0], s.s2[1], True)}
    if s.cd is not None:
        ops.update(amode=3, res=s.cd, afd=_bnf(b.downsample[1], s.pd, s.Rd, s.count2, s.sd[0], s.sd[1], True))
    else:
        ops.update(amode=2, res=s.inp)
    return ops


def _wgrad(X, x, dy, weight, geom, xops, gops):
    """grad-W of one conv into the parameter's gradient buffer (batch-split slabs summed later,
    batched, when the backward pass ends: ops/gradfinish.py)."""
    dw = grad_buffer(weight)
    z = int(X.sm_plan(geom, x.shape[0])[3])
    if z > 1:
        part = torch.empty(z * weight.numel(), device=x.device, dtype=x.dtype)
        X.sm_wgrad_ops(x, dy, part, geom, xops, gops)
        if gradfinish.can_defer(weight):
            gradfinish.defer_slab(part, dw, z)
        else:
            X.slab_sum(part, dw.view(-1), z)
    else:
        X.sm_wgrad_ops(x, dy, dw, geom, xops, gops)
    return dw
