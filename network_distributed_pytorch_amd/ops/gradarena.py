"""Gradient buffers that ARE slices of a gradient-sync arena.

The dense arm (parallel/ddp.py) all-reduces gradients as contiguous buckets of one flat
arena.  Without help, autograd puts every parameter's gradient in a fresh buffer and each
bucket needs a flatten launch (+ a read and a write of every gradient) before its
collective.  A backward function that produces a parameter's gradient asks
:func:`grad_buffer` for its output buffer instead of ``torch.empty_like``: for a registered
parameter it gets the parameter's arena slice, writes the gradient there directly, and
autograd's AccumulateGrad adopts that tensor as ``param.grad`` (it is the only reference,
with the parameter's layout).  The bucket flatten then skips every parameter whose
``.grad`` already lives in the arena.  Only when ``param.grad is None`` (set_to_none
zero_grad; with an existing ``.grad`` autograd accumulates, and handing out the arena slice
would alias it).  Used by the native conv (direct / tgemm / Toeplitz) and BN backwards.
"""
from __future__ import annotations

import os
import weakref
from typing import Iterable

import torch
from ..knobs import fusion_on

__all__ = ["register", "unregister", "grad_buffer", "registered", "release"]

_VIEWS: dict = {}
# id(param) -> autograd graph task that received the param's arena slice.  A parameter used
# twice in one forward (tied / shared weights) gets a second gradient in the SAME backward
# before AccumulateGrad adopted the first: that one must not alias the slice (autograd would
# add the two aliased tensors, 2 x g2 instead of g1 + g2).  ADVICE r3.
_HANDED: dict = {}


def _task_id() -> int:
    try:
        return int(torch._C._current_graph_task_id())
    except Exception:  # pragma: no cover - older torch: no task ids, one handout per release
        return -2
_ON = fusion_on("grad_arena")


def register(param: torch.Tensor, arena: torch.Tensor, offset: int) -> None:
    _VIEWS[id(param)] = (weakref.ref(param), arena, int(offset))


def unregister(params: Iterable[torch.Tensor]) -> None:
    for p in params:
        _VIEWS.pop(id(p), None)
        _HANDED.pop(id(p), None)


def release(params: Iterable[torch.Tensor]) -> None:
    """The parameters' ``.grad`` were dropped (zero_grad): their slices may be handed out again."""
    for p in params:
        _HANDED.pop(id(p), None)


def registered(param: torch.Tensor) -> bool:
    e = _VIEWS.get(id(param))
    return e is not None and e[0]() is param


def grad_buffer(param: torch.Tensor, like: torch.Tensor = None) -> torch.Tensor:
    """Output buffer for ``param``'s gradient: its arena slice when registered and adoptable,
    else a fresh tensor like ``like`` (default ``param``)."""
    e = _VIEWS.get(id(param)) if _ON else None
    if e is not None and param.grad is None and not torch.is_grad_enabled():
        ref, arena, off = e
        task = _task_id()
        if ref() is param and _HANDED.get(id(param)) != task:
            _HANDED[id(param)] = task
            return arena[off: off + param.numel()].view_as(param)
    return torch.empty_like(param if like is None else like)
