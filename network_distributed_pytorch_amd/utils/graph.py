"""hipGraph step runner (HIP graphs instead of a tracing compiler).

ResNet-18 on 32x32 inputs launches ~300 small kernels per training step; eager launch
overhead leaves the GPU idle for ~25 % of the step (profiles/).  :class:`StepRunner`
warms a training step up on a side stream (MIOpen find, RCCL communicator init, the
native table uploads), then captures it and replays it every step:

* ``full``      — forward + backward + the fused PowerSGD / SGD update (and, for N > 1,
                  the collectives) in ONE graph;
* ``piecewise`` — the compute phases are captured, the collectives run eagerly between
                  graph replays (``sync.phases()``): robust for RCCL at N > 1 while still
                  removing every compute-kernel launch from the host path;
* ``none``      — plain eager execution.

``auto`` = ``full`` at world size 1, ``piecewise`` otherwise.  The step must read its
inputs from static tensors (copy each batch into them before calling the runner).
Requirements: all ops capture-safe (the native kernels and ``ops.upload`` are); PowerSGD
needs ``reuse_query=True`` (the reference default) because the query re-draw is host-side.
"""
from __future__ import annotations

import contextlib
import os
from typing import Callable, List, Optional, Tuple

import torch

from ..ops import _UPLOADS
from ..parallel.comm import world_size

# NDP_DEFER_UPLOADS=0: capture-time table uploads stay memcpy nodes re-run on every replay
_DEFER_UPLOADS = os.environ.get("NDP_DEFER_UPLOADS", "1") != "0"

__all__ = ["StepRunner", "GraphedStep"]


class StepRunner:
    def __init__(self, pre: Callable[[], None], sync, mode: str = "auto", warmup: int = 3,
                 post: Optional[Callable[[], None]] = None):
        self.pre = pre
        self.sync = sync
        self.post = post or (lambda: None)
        if mode == "auto":
            mode = "full" if world_size() <= 1 else "piecewise"
        if not torch.cuda.is_available():
            mode = "none"
        self.mode = mode
        self.warmup = warmup
        self.segments: List[Tuple[Callable[[], None], bool]] = self._segments()
        self.graphs: Optional[list] = None
        self._uploads: list = []
        self._upload_gen = 0
        self.replays = 0

    def _segments(self):
        if self.mode in ("none", "full"):
            def whole():
                self.pre()
                self.sync.step()
                self.post()
            return [(whole, self.mode == "full")]
        phases = list(self.sync.phases())
        segs: List[Tuple[List[Callable], bool]] = [([self.pre], True)]
        for fn, is_comm in phases:
            if is_comm:
                segs.append(([fn], False))
            elif segs[-1][1]:
                segs[-1][0].append(fn)
            else:
                segs.append(([fn], True))
        segs[-1][0].append(self.post) if segs[-1][1] else segs.append(([self.post], True))

        def chain(fns):
            def run():
                for f in fns:
                    f()
            return run
        return [(chain(f), cap) for f, cap in segs]

    def _run_eager(self):
        for fn, _ in self.segments:
            fn()

    def capture(self):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self._run_eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        graphs = []
        scope = _UPLOADS.capture_scope() if _DEFER_UPLOADS else contextlib.nullcontext([])
        with scope as uploads:  # table uploads: applied once after capture, not per replay
            for fn, cap in self.segments:
                if cap:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=pool):
                        fn()
                    graphs.append(g)
                else:
                    graphs.append(None)
        torch.cuda.synchronize()
        self._uploads = uploads
        self._upload_gen = _UPLOADS.generation
        self.graphs = graphs
        # the first replay below is the first real step after capture

    def __call__(self):
        if self.mode == "none":
            self._run_eager()
            return
        if self.graphs is None:
            self.capture()
        # an eager step since capture may have re-bound a table the graph reads
        self._upload_gen = _UPLOADS.ensure(self._uploads, self._upload_gen)
        for (fn, _), g in zip(self.segments, self.graphs):
            if g is None:
                fn()
            else:
                g.replay()
        self.replays += 1
        count = getattr(self.sync, "count_step", None)
        if count is not None:  # host bookkeeping skipped by the replayed Python
            count()


class GraphedStep(StepRunner):
    """Back-compat: capture one closure (full mode)."""

    def __init__(self, fn: Callable[[], None], warmup: int = 3, enabled: bool = True):
        class _NoSync:
            def step(self):
                pass

            def phases(self):
                return []
        super().__init__(fn, _NoSync(), mode="full" if enabled else "none", warmup=warmup)
