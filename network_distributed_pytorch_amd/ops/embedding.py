"""``nn.Embedding`` with a native deterministic, hipGraph-replayable backward.

Forward is the ordinary row gather (``F.embedding``).  On device the weight gradient is
built by csrc/embedding.hip (rank-by-comparison permutation + fixed-order row sums, no sort
library, no atomics, no temporary allocation) instead of PyTorch-ROCm's
``embedding_dense_backward``, whose rocPRIM sort path (> 3072 ids per call) faulted the GPU
when replayed inside a captured training step.  Same parameters and ``state_dict`` as
``nn.Embedding``; ``padding_idx`` rows get a zero gradient as there.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._ext import ext

__all__ = ["Embedding"]


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, pad, mod):
        ctx.save_for_backward(ids)
        ctx.pad, ctx.mod, ctx.shape = pad, mod, weight.shape
        return F.embedding(ids, weight, pad)

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        gw = torch.empty(ctx.shape, device=g.device, dtype=torch.float32)
        perm, start, cnt = ctx.mod._scratch(ids.numel(), g.device)
        ext().embedding_backward(ids.reshape(-1).contiguous(), g.reshape(-1, ctx.shape[1]).contiguous(), gw,
                                 -1 if ctx.pad is None else int(ctx.pad), perm, start, cnt)
        return None, gw, None, None


class Embedding(nn.Embedding):
    """Drop-in ``nn.Embedding`` (dense gradient, no max_norm / scale_grad_by_freq)."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self._perm = None
        self._rows = None  # [2, V] int32: row start, row count (count re-armed by the kernel)

    def _scratch(self, n_ids: int, device):
        if self._rows is None or self._rows.device != device:
            assert not torch.cuda.is_current_stream_capturing(), "embedding scratch allocated during capture"
            self._rows = torch.zeros(2, self.num_embeddings, dtype=torch.int32, device=device)
        if self._perm is None or self._perm.numel() < n_ids or self._perm.device != device:
            assert not torch.cuda.is_current_stream_capturing(), "embedding scratch grows during capture"
            self._perm = torch.empty(max(n_ids, 1), dtype=torch.int32, device=device)
        return self._perm, self._rows[0], self._rows[1]

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        if (ids.is_cuda and self.weight.dtype == torch.float32 and self.max_norm is None
                and not self.scale_grad_by_freq and not self.sparse and self.embedding_dim % 4 == 0
                and torch.is_grad_enabled() and self.weight.requires_grad):
            self._scratch(ids.numel(), ids.device)  # first (eager) call sizes the scratch
            return _EmbeddingFn.apply(ids.long(), self.weight, self.padding_idx, self)
        return super().forward(ids)
