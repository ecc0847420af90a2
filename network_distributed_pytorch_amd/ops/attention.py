"""Fused fp32 self-attention (csrc/attention.hip) with an explicit-math fallback.

Semantics are HF DistilBERT's ``MultiHeadSelfAttention`` core (the reference model,
ddp_powersgd_distillBERT_IMDb/ddp_init.py:150): ``softmax(mask(q k^T / sqrt(dh))) v``
with ``masked_fill(finfo.min)`` for padded keys and dropout on the probabilities.

``attention(q, k, v, mask, p_drop)`` takes q/k/v as ``[B, S, H, 64]`` (a free view of the
``[B, S, H*64]`` projections — no transposes) and returns ``[B, S, H, 64]``.  On a GPU with
fp32 inputs it runs the flash-style HIP kernels (scores never touch HBM); elsewhere the
explicit math below runs (and is the numerics oracle for the tests).

Dropout keep-decisions come from a counter hash of (seed, b*H+h, query, key); the seed
is a device int32 drawn from torch's CUDA generator each call, so hipGraph replays see
fresh masks and backward regenerates exactly the forward's mask.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ._ext import ext

__all__ = ["attention", "attention_qkv", "attention_reference", "dropout_keep_mask", "fused_ok"]

_M32 = 0xFFFFFFFF


def fused_ok(q: torch.Tensor) -> bool:
    return q.is_cuda and q.dtype == torch.float32 and q.dim() == 4 and q.shape[-1] == 64


def _u32(x):
    return x & _M32


def dropout_keep_mask(seed: int, B: int, H: int, S: int, p: float, device="cpu") -> torch.Tensor:
    """Host re-implementation of the kernels' keep mask, [B, H, S(query), S(key)] bool."""
    thr = min(int(p * 4294967296.0), _M32)
    bh = torch.arange(B * H, dtype=torch.int64, device=device).view(-1, 1, 1)
    q = torch.arange(S, dtype=torch.int64, device=device).view(1, -1, 1)
    k = torch.arange(S, dtype=torch.int64, device=device).view(1, 1, -1)
    a = seed & _M32
    h = _u32(_u32(a * 0x9E3779B1) ^ _u32(_u32(bh + 0x7F4A7C15) * 0x85EBCA77))
    h = h ^ _u32(_u32(q + 0x165667B1) * 0xC2B2AE3D)
    h = _u32((h ^ (h >> 15)) * 0x2C1B3C6D)
    h = h ^ _u32(_u32(k + 0x27D4EB2F) * 0x9E3779B1)
    h = _u32((h ^ (h >> 13)) * 0x297A2D39)
    h = h ^ (h >> 16)
    return (h >= thr).view(B, H, S, S)


def attention_reference(q, k, v, mask: Optional[torch.Tensor] = None, p_drop: float = 0.0,
                        keep: Optional[torch.Tensor] = None, dropout=None):
    """Explicit math, [B, S, H, D] in / out.  ``keep`` pins the dropout mask (tests);
    otherwise ``dropout`` (an ``nn.Dropout``) or ``F.dropout`` is applied."""
    B, S, H, D = q.shape
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    scores = torch.matmul(qt / math.sqrt(D), kt.transpose(-1, -2))
    if mask is not None:
        scores = scores.masked_fill((mask == 0).view(B, 1, 1, S), torch.finfo(scores.dtype).min)
    w = torch.softmax(scores, dim=-1)
    if keep is not None:
        w = w * keep.to(w.dtype) / (1.0 - p_drop)
    elif dropout is not None:
        w = dropout(w)
    elif p_drop > 0:
        w = torch.nn.functional.dropout(w, p_drop)
    return torch.matmul(w, vt).transpose(1, 2)


class _FusedAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, mask, seed, p_drop):
        B, S, H, _ = q.shape
        o = torch.empty(q.shape, device=q.device, dtype=q.dtype)
        lse = torch.empty(2, B, H, S, device=q.device, dtype=torch.float32)   # row max, log(sum)
        scale = 1.0 / math.sqrt(q.shape[-1])
        ext().attn_fwd(q, k, v, mask, o, lse, scale, seed, p_drop)
        ctx.save_for_backward(q, k, v, mask, o, lse, seed)
        ctx.has_mask = mask is not None
        ctx.p_drop = p_drop
        ctx.scale = scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, mask, o, lse, seed = ctx.saved_tensors
        do = do.contiguous()
        B, S, H, _ = q.shape
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty(B, H, S, device=q.device, dtype=torch.float32)
        ext().attn_bwd(q, k, v, mask if ctx.has_mask else None, o, do, lse, delta, dq, dk, dv, ctx.scale,
                       seed if ctx.p_drop > 0 else None, ctx.p_drop)
        return dq, dk, dv, None, None, None


def attention(q, k, v, mask: Optional[torch.Tensor] = None, p_drop: float = 0.0,
              seed: Optional[torch.Tensor] = None, dropout=None):
    """[B, S, H, 64] fp32 -> [B, S, H, 64].  ``mask``: [B, S] (nonzero = attend)."""
    if not fused_ok(q):
        return attention_reference(q, k, v, mask, p_drop, dropout=dropout)
    q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
    if mask is not None:
        mask = mask.to(torch.int32).contiguous()
    if p_drop > 0 and seed is None:
        seed = torch.randint(0, 2 ** 31 - 1, (1,), device=q.device, dtype=torch.int32)
    return _FusedAttention.apply(q, k, v, mask, seed, float(p_drop))


class _FusedAttentionQKV(torch.autograd.Function):
    """Attention straight off a packed QKV projection [B, S, 3 * H * 64] (one GEMM for the
    three projections): the kernels read q / k / v in place with a 3*H*64 token stride and
    the backward writes dq / dk / dv into ONE packed gradient — the projection's backward is
    then one grad-x GEMM, one grad-W GEMM and one bias column sum instead of three each plus
    two autograd adds of the three grad-x tensors."""

    @staticmethod
    def forward(ctx, qkv, H, mask, seed, p_drop):
        B, S, D3 = qkv.shape
        v5 = qkv.view(B, S, 3, H, 64)
        q, k, v = v5[:, :, 0], v5[:, :, 1], v5[:, :, 2]
        o = torch.empty(B, S, H, 64, device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty(2, B, H, S, device=qkv.device, dtype=torch.float32)
        scale = 1.0 / 8.0  # 1 / sqrt(64)
        ext().attn_fwd(q, k, v, mask, o, lse, scale, seed, p_drop)
        ctx.save_for_backward(qkv, mask, o, lse, seed)
        ctx.has_mask = mask is not None
        ctx.p_drop = p_drop
        ctx.scale = scale
        ctx.H = H
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, mask, o, lse, seed = ctx.saved_tensors
        do = do.contiguous()
        B, S, D3 = qkv.shape
        H = ctx.H
        v5 = qkv.view(B, S, 3, H, 64)
        dqkv = torch.empty_like(qkv)
        d5 = dqkv.view(B, S, 3, H, 64)
        delta = torch.empty(B, H, S, device=qkv.device, dtype=torch.float32)
        ext().attn_bwd(v5[:, :, 0], v5[:, :, 1], v5[:, :, 2], mask if ctx.has_mask else None, o, do, lse, delta,
                       d5[:, :, 0], d5[:, :, 1], d5[:, :, 2], ctx.scale, seed if ctx.p_drop > 0 else None,
                       ctx.p_drop)
        return dqkv, None, None, None, None


def attention_qkv(qkv, n_heads: int, mask: Optional[torch.Tensor] = None, p_drop: float = 0.0,
                  seed: Optional[torch.Tensor] = None):
    """Fused attention on a packed projection ``qkv`` [B, S, 3 * n_heads * 64] (q | k | v
    along the last dim) -> [B, S, n_heads, 64]."""
    B, S, D3 = qkv.shape
    assert D3 == 3 * n_heads * 64, "attention_qkv: packed q | k | v of 64-wide heads"
    qkv = qkv.contiguous()
    if mask is not None:
        mask = mask.to(torch.int32).contiguous()
    if p_drop > 0 and seed is None:
        seed = torch.randint(0, 2 ** 31 - 1, (1,), device=qkv.device, dtype=torch.int32)
    return _FusedAttentionQKV.apply(qkv, n_heads, mask, seed, float(p_drop))
