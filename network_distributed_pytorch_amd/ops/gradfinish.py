"""Deferred, batched weight-gradient finishing for the native convolutions.

Each direct-conv grad-W ends with a split-slab sum and each Toeplitz conv grad-W with a
fold of grad-W_big into the weight shape: ~20 small launches per ResNet-18 backward that
are latency-bound (4-7 µs each).  Instead, the conv backward functions record them here
and ONE ``gradw_finish`` launch (csrc/conv.hip: slab-sum blocks then fold blocks) finishes
them all when autograd's backward pass ends (``queue_callback`` on the execution engine: the
gradients are complete when ``backward()`` returns, exactly as without deferral), or
earlier when a consumer needs them mid-backward (:func:`flush`: the overlapped gradient
sync calls it before handing a group's gradients to the side stream).  Same summation
order per element as the per-layer kernels: results are bitwise identical.

Capture-safe (kernel arguments only, no table uploads).  ``NDP_FUSION_OFF=defer_gradw`` restores
per-layer launches.
"""
from __future__ import annotations

import warnings

import torch

from ._ext import ext
from ..knobs import fusion_on

__all__ = ["enabled", "can_defer", "defer_slab", "defer_fold", "flush", "pending"]

_MAX = 24  # csrc/ndp_kernels.h kMaxExpand
_ENABLED = fusion_on("defer_gradw")
_slabs: list = []
_folds: list = []
_queued = [False]
_keep: list = []


def enabled() -> bool:
    return _ENABLED


def pending() -> int:
    return len(_slabs) + len(_folds)


def _queue():
    if not _queued[0]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
            _queued[0] = True
        except RuntimeError:  # not inside a backward pass: finish right away
            flush()


def _end_of_backward():
    _queued[0] = False
    _CLAIMED.clear()  # claims live for one graph task (ids of dead params may be reused)
    flush()


def _task_id():
    """The running autograd graph task's id, or None when this torch exposes none."""
    try:
        return int(torch._C._current_graph_task_id())
    except Exception:  # pragma: no cover - older torch: no task ids
        return None


_NO_TASK_WARNED = [False]


# id(param) -> autograd graph task in which a gradient of the param was deferred
_CLAIMED: dict = {}


def can_defer(param: torch.Tensor) -> bool:
    """Deferral needs the returned buffer to BE the final gradient: ``param.grad is None``
    (AccumulateGrad adopts the buffer, or ``autograd.grad`` returns it) and no
    double-backward graph.

    A parameter used twice in one forward (shared / tied module) gets a second gradient in
    the SAME graph task before AccumulateGrad adopted the first; autograd then adds the two
    buffers as soon as the second arrives.  So the first claim of a task defers, and a
    second one finishes every pending sum right now (stream-ordered before autograd's add
    reads the first buffer) and is computed immediately."""
    if not (_ENABLED and param.grad is None and not torch.is_grad_enabled()):
        return False
    task = _task_id()
    if task is None:
        # without task ids a shared parameter's second gradient cannot be told from the next
        # backward's first: defer nothing, say so once
        if not _NO_TASK_WARNED[0]:
            _NO_TASK_WARNED[0] = True
            warnings.warn("torch exposes no autograd graph-task id: deferred grad-W finishing is off")
        return False
    if _CLAIMED.get(id(param)) == task:
        flush()
        return False
    _CLAIMED[id(param)] = task
    return True


def _alias(t: torch.Tensor) -> torch.Tensor:
    """A tensor on ``t``'s storage that is NOT a reference to ``t``'s TensorImpl: holding it
    keeps the memory alive without raising ``t``'s use count (with a second reference
    AccumulateGrad would copy the still-unfinished buffer instead of adopting it)."""
    return torch.empty(0, dtype=t.dtype, device=t.device).set_(t.untyped_storage(), t.storage_offset(), t.shape,
                                                               t.stride())


def defer_slab(part: torch.Tensor, dw: torch.Tensor, slices: int, keep=()) -> None:
    """``dw`` (the buffer the backward returns) = sum over ``slices`` slabs of ``part``, later.
    ``keep``: tensors a held-back grad-W launch still reads (csrc/conv.hip conv_flush_pending:
    the grad-W waits for its conv's grad-x to share one launch), kept alive until the flush."""
    _slabs.append((part, _alias(dw), int(slices)))
    _keep.extend(keep)
    _queue()


def defer_fold(dwt: torch.Tensor, dw: torch.Tensor, geom) -> None:
    """``dw`` = fold(dw_big) (csrc/conv.hip toeplitz_fold), later."""
    _folds.append((dwt, _alias(dw), list(geom)))
    _queue()


def flush() -> None:
    """Finish every pending weight gradient (one launch per kind, per 24 entries)."""
    if not _slabs and not _folds:
        return
    X = ext()
    X.conv_flush_pending()  # a grad-W still held back for a grad-x that never came: its slabs first
    _keep.clear()
    slabs, folds = list(_slabs), list(_folds)
    _slabs.clear()
    _folds.clear()
    if len(slabs) <= _MAX and len(folds) <= _MAX:
        X.gradw_finish(slabs, folds)  # both kinds in one launch (ResNet-18: 1 instead of 2)
        return
    for i in range(0, len(slabs), _MAX):
        X.slab_sum_many(slabs[i: i + _MAX])
    for i in range(0, len(folds), _MAX):
        X.toeplitz_fold_many(folds[i: i + _MAX])
