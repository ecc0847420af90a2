"""Native ops: flat-arena / multi-tensor kernels with device dispatch.

Device tensors -> hand-written gfx950 HIP kernels (``_C``); CPU tensors -> pure torch.
The PowerSGD grouped kernels are driven from
:mod:`network_distributed_pytorch_amd.parallel.powersgd` through the plan tables.
"""
from __future__ import annotations

import contextlib

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
    "capturing",
    "upload",
    "SegPlan",
    "upload_epoch",
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


class _PinnedPool:
    """Bump allocator over one pinned host buffer, reserved before any graph capture.

    Pinned allocation is not permitted while a stream is capturing, so capture-time table
    uploads take never-reused slices of this pool (the graph's memcpy nodes read them on
    every replay).
    """

    def __init__(self):
        self.buf = None
        self.off = 0

    def reserve(self, nbytes: int = 16 << 20):
        if self.buf is None and torch.cuda.is_available():
            self.buf = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)

    def take(self, nbytes: int) -> torch.Tensor:
        assert self.buf is not None, "pinned pool not reserved before capture"
        start = (self.off + 255) // 256 * 256
        assert start + nbytes <= self.buf.numel(), "pinned upload pool exhausted"
        self.off = start + nbytes
        return self.buf[start: start + nbytes]


_PINNED = _PinnedPool()


def capturing() -> bool:
    """True while the current HIP stream is being captured into a graph."""
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def upload(dev: torch.Tensor, host: torch.Tensor) -> None:
    """Copy a small host table into a preallocated device buffer, hipGraph-capture safe.

    Outside capture: an ordinary (synchronous) copy.  Inside capture: the bytes go to a
    never-reused slice of a pre-reserved pinned pool and the copy becomes an async memcpy
    node, so every replay re-uploads exactly the capture-time table.
    """
    n = host.numel()
    assert dev.numel() >= n and dev.dtype == host.dtype
    if n == 0:
        return
    if dev.is_cuda and capturing() and _UPLOADS.defer:
        _UPLOADS.record(dev[:n], host.reshape(-1).clone())
        return
    if dev.is_cuda and capturing():
        nbytes = n * host.element_size()
        pinned = _PINNED.take(nbytes).view(host.dtype)
        pinned.copy_(host.reshape(-1))
        dev[:n].copy_(pinned, non_blocking=True)
    else:
        if dev.is_cuda:
            _PINNED.reserve()
            _UPLOADS.generation += 1
        dev[:n].copy_(host)


class _DeferredUploads:
    """Capture-time table uploads applied ONCE after capture instead of as memcpy nodes.

    A graph captured by :class:`utils.graph.StepRunner` always replays the capture-time
    tables, so re-uploading them on every replay (one ~5 µs copy node per table, 5 per
    PowerSGD step) is wasted.  Inside :meth:`capture_scope` uploads are recorded and, when
    the scope ends, copied synchronously.  ``generation`` counts eager uploads: if an eager
    step re-bound a table after capture, :meth:`ensure` restores the capture-time contents
    before the next replay.

    ``epoch`` counts :meth:`apply` calls.  Every Python-side table cache (``SegPlan``,
    ``_PlanBuffers``, the optimizers' pointer tables) puts the epoch into its cache key:
    after the capture-time tables were (re)applied, the next eager bind always re-uploads
    instead of trusting an address key that no longer describes the device table.
    """

    def __init__(self):
        self.defer = False
        self.generation = 0
        self.epoch = 0
        self._pending = []

    def record(self, dev: torch.Tensor, host: torch.Tensor):
        for d, h in self._pending:
            if d.data_ptr() == dev.data_ptr() and not (h.numel() == host.numel() and torch.equal(h, host)):
                raise RuntimeError("table uploaded twice with different contents inside one capture; "
                                   "capture without deferred uploads")
        self._pending.append((dev, host))

    @contextlib.contextmanager
    def capture_scope(self):
        """Yields the list that receives the recorded uploads (applied on exit)."""
        self.defer, self._pending = True, []
        try:
            yield self._pending
        finally:
            self.defer = False
        self.apply(self._pending)

    def apply(self, uploads):
        for d, h in uploads:
            d.copy_(h)
        if uploads:
            torch.cuda.synchronize()
        self.generation += 1  # the tables now hold the capture-time contents
        self.epoch += 1       # ... so every eager-side cache key is stale

    def ensure(self, uploads, generation: int) -> int:
        """Re-apply ``uploads`` if any eager upload happened since ``generation``."""
        if generation != self.generation:
            self.apply(uploads)
        return self.generation


_UPLOADS = _DeferredUploads()


def upload_epoch() -> int:
    """Current table-restore epoch (include it in any device-table cache key)."""
    return _UPLOADS.epoch


class SegPlan:
    """One-launch multi-tensor reduce-copy: ``dst_i = (sum_c src_i[c*stride_i:]) / div_i``.

    ``specs`` = list of (src_tensor, dst_tensor, chunks, stride, div); src/dst are flat
    float32 tensors (views are fine).  On device the table lives in a device buffer and the
    whole list is ONE kernel launch.  :meth:`set` re-targets the plan at new tensors (the
    table is only re-uploaded when an address changed; capture-safe via :func:`upload`).
    """

    def __init__(self, specs: Sequence[tuple] = (), device: torch.device = "cpu", capacity: int = 0):
        self.device = torch.device(device)
        self.specs: list = []
        self._key = None
        self._ent = None
        self._prefix = None
        self._n_ent = 0
        self._n_blocks = 0
        self._cap = 0
        if self.device.type == "cuda":
            self._reserve(max(capacity, len(specs), 1))
        self.set(specs)

    def _reserve(self, n_entries: int):
        X = ext()
        self._cap = n_entries
        self._ent = torch.empty(n_entries * X.SIZEOF_SEGENTRY, dtype=torch.uint8, device=self.device)
        self._prefix = torch.empty(n_entries, dtype=torch.int64, device=self.device)

    def set(self, specs: Sequence[tuple]) -> None:
        specs = list(specs)
        key = (_UPLOADS.epoch,) + tuple((s.data_ptr(), d.data_ptr(), d.numel(), int(c), int(st), float(dv))
                                        for s, d, c, st, dv in specs)
        self.specs = specs
        if key == self._key:
            return
        self._key = key
        if self.device.type != "cuda" or not specs:
            return
        rows = [(a, b, n, st, c, dv) for a, b, n, c, st, dv in key[1:]]
        ent, prefix, n_ent, n_blocks = ext().make_seg_table(rows)
        if n_ent > self._cap:
            assert not capturing(), "SegPlan must be sized before graph capture"
            self._reserve(max(n_ent, 2 * self._cap))
        upload(self._ent, ent.to(self._ent.dtype) if ent.dtype != torch.uint8 else ent)
        upload(self._prefix, prefix)
        self._n_ent, self._n_blocks = int(n_ent), int(n_blocks)

    def table(self):
        """(entries, prefix, n_entries, n_blocks) of the device table, for a kernel that runs the
        plan in its own launch (the PowerSGD P pass's rank-1 pack); None when there is nothing to do."""
        if not self.specs or self.device.type != "cuda" or not self._n_ent:
            return None
        return self._ent, self._prefix, self._n_ent, self._n_blocks

    def run(self) -> None:
        if not self.specs:
            return
        if self.device.type == "cuda":
            if self._n_ent:
                ext().seg_reduce(self._ent, self._prefix, self._n_ent, self._n_blocks)
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
