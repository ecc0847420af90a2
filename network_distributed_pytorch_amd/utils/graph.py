"""hipGraph step runner (HIP graphs instead of a tracing compiler).

ResNet-18 on 32x32 inputs launches ~200 small kernels per training step; eager launch
overhead leaves the GPU idle for ~25 % of the step (profiles/).  :class:`StepRunner`
warms a training step up on a side stream (MIOpen find, RCCL communicator init, the
native table uploads), then captures it and replays it every step:

* ``full``      — the whole step (forward + backward + gradient sync + update) captured.
                  With a stream-ordered data plane (native RCCL communicator, or world
                  size 1) the sync's post-accumulate-grad hooks hand bucket / PowerSGD-group
                  work (kernels AND collectives) to the communicator's side stream
                  (``Communicator.side_launch``).  The step is then captured as TWO linear
                  graphs: the compute graph (forward + backward) with a one-lane
                  "flag signal" kernel at every hook point, and the comm graph with a
                  matching "flag wait" kernel before each piece of side work.  Replay
                  launches the compute graph on the current stream and the comm graph on
                  the side stream; the comm graph ends by signalling a DONE flag that the
                  next compute graph waits on first.  Measured reasons for this shape
                  (profiles/overlap_r2.md): one graph with a parallel branch is executed by
                  the HIP runtime node by node across internal streams (2.50 vs 2.13 ms per
                  step), and hipEvent waits between the two graphs were re-evaluated only
                  after the producing queue drained its kernel train (the comm work started
                  after the whole backward).  The device flags react within microseconds.
                  ``runner.join()`` orders the current stream after the last comm graph.
* ``piecewise`` — the compute phases are captured, the collectives run eagerly between
                  graph replays (``sync.phases()``): the c10d data plane (``NDP_NATIVE_COMM=0``).
* ``none``      — plain eager execution (gloo: its host thread blocks on collectives).

``auto`` = ``full`` when the sync's communicator is stream-ordered, ``piecewise`` for a
c10d-nccl group, ``none`` for gloo / CPU.

Warm-up does not change training: the sync's training state (parameters, error memory,
momentum, warm-start Q, step counter — ``sync.snapshot()``) and any ``state_tensors``
(e.g. BatchNorm running statistics) are saved before the warm-up steps and restored after
capture, so the first replay is the first real step (graph mode used to apply
``warmup`` extra optimizer updates to batch 0).

The step must read its inputs from static tensors (copy each batch into them before
calling the runner).  Requirements: all ops capture-safe (the native kernels and
``ops.upload`` are); PowerSGD needs ``reuse_query=True`` (the reference default) because
the query re-draw is host-side.
"""
from __future__ import annotations

import contextlib
import gc
import os
import time
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops import _UPLOADS, ext
from ..parallel.comm import world_size
from ..knobs import fusion_on

# NDP_FUSION_OFF=defer_uploads: capture-time table uploads stay memcpy nodes re-run on every replay
_DEFER_UPLOADS = fusion_on("defer_uploads")

__all__ = ["StepRunner", "GraphedStep", "auto_mode"]


def auto_mode(sync) -> str:
    """Pick the capture mode for a gradient-sync object (see module docstring)."""
    if not torch.cuda.is_available():
        return "none"
    comm = getattr(sync, "comm", None)
    if comm is None:
        return "full" if world_size() <= 1 else "piecewise"
    if getattr(comm, "stream_ordered", False):
        return "full"
    try:
        backend = dist.get_backend(comm.group)
    except Exception:
        backend = "gloo"
    return "piecewise" if backend == "nccl" else "none"


class StepRunner:
    def __init__(self, pre: Callable[[], None], sync, mode: str = "auto", warmup: int = 3,
                 post: Optional[Callable[[], None]] = None, state_tensors: Sequence[torch.Tensor] = ()):
        self.pre = pre
        self.sync = sync
        self.post = post or (lambda: None)
        if mode == "auto":
            mode = auto_mode(sync)
        if not torch.cuda.is_available():
            mode = "none"
        self.mode = mode
        self.warmup = warmup
        self.state_tensors = [t for t in state_tensors if t is not None]
        self.segments: List[Tuple[Callable[[], None], bool]] = self._segments()
        self.graphs: Optional[list] = None
        self._uploads: list = []
        self._upload_gen = 0
        self.replays = 0
        self.side_graphs = []
        self._comm = None
        self.host_launch_s = [0.0, 0.0]  # host time inside replay() of compute / comm graphs
        self._joined = True

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
        self.join()  # an eager step after a replay reads what the comm graph writes
        for fn, _ in self.segments:
            fn()

    def _snapshot(self):
        snap = self.sync.snapshot() if hasattr(self.sync, "snapshot") else None
        return snap, [t.clone() for t in self.state_tensors]

    def _restore(self, saved):
        snap, tensors = saved
        if snap is not None:
            self.sync.restore(snap)
        for t, s in zip(self.state_tensors, tensors):
            t.copy_(s)

    def capture(self):
        if hasattr(self.sync, "prepare"):
            self.sync.prepare()  # e.g. draw PowerSGD's initial queries BEFORE the snapshot
        saved = self._snapshot()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        comm = getattr(self.sync, "comm", None)
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                n0 = getattr(comm, "side_launches", 0)
                self._run_eager()
        # split compute / comm graphs only if the step hands work to the side stream (the
        # compute graph's DONE wait would otherwise have no signaller)
        self._uses_side = getattr(comm, "side_launches", 0) > n0 if self.warmup > 0 else True
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # no cyclic GC while capturing: a collected graph / stream / event of an earlier
        # runner would call a HIP API that is illegal during capture (abort in a destructor)
        gc.collect()
        gc_was_enabled = gc.isenabled()
        gc.disable()
        try:
            self._capture_graphs()
        finally:
            if gc_was_enabled:
                gc.enable()
        self._restore(saved)  # warm-up steps leave no trace: the first replay is step 1
        torch.cuda.synchronize()

    def _capture_graphs(self):
        pool = torch.cuda.graph_pool_handle()
        graphs = []
        comm = getattr(self.sync, "comm", None)
        segmented = (self.mode == "full" and comm is not None and hasattr(comm, "defer_side")
                     and getattr(self, "_uses_side", True))
        self.side_graphs = []
        scope = _UPLOADS.capture_scope() if _DEFER_UPLOADS else contextlib.nullcontext([])
        with scope as uploads:  # table uploads: applied once after capture, not per replay
            if segmented:
                # compute graph: wait(DONE) + forward + backward, one flag-signal kernel at
                # every side launch; comm graph: flag-wait + side work per signal, then
                # signal(DONE) for the next step's compute graph
                (fn, _), = self.segments
                with comm.defer_side() as items:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=pool):
                        comm.graph_prologue()
                        fn()
                    graphs.append(g)
                if not items:
                    raise RuntimeError("captured compute graph waits for a comm graph, but the step "
                                       "launched no side work during capture (it did during warm-up)")
                if items:
                    gs = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gs, pool=torch.cuda.graph_pool_handle(), stream=torch.cuda.Stream()):
                        for i, item in enumerate(items):
                            comm.graph_wait(i)
                            for f in item:
                                f()
                        comm.graph_epilogue()
                    self.side_graphs.append(gs)
                    self._comm = comm
                    comm.reset_flags()
            else:
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

    def join(self):
        """Make the current stream wait for the last replay's comm graph (call before
        reading parameters / sync state on the host side: checkpoint, eval, checks)."""
        if self.side_graphs and not self._joined:
            self._comm.join()
            self._joined = True

    def __call__(self):
        if self.mode == "none":
            self._run_eager()
            return
        if self.graphs is None:
            self.capture()
        # an eager step since capture may have re-bound a table the graph reads
        self._upload_gen = _UPLOADS.ensure(self._uploads, self._upload_gen)
        if self.side_graphs:
            if self._comm.host_flag_error():  # a wait of an earlier replay timed out: stop now
                self._comm.raise_flag_error()
            # comm graph FIRST: the command processor serves the queues roughly in doorbell
            # order, so a comm graph submitted after the compute graph is dispatched only
            # when the compute queue's kernel train has (nearly) drained — measured with
            # tools/probe_queue.py (profiles/r2/queue_probe.md).  Submitted first, its
            # flag-wait kernel is resident before the compute graph starts.
            t0 = time.perf_counter()
            with self._comm.on_side():
                self.side_graphs[0].replay()  # each piece waits for its compute-graph signal
            t1 = time.perf_counter()
            self.graphs[0].replay()          # waits (device flag) for the previous comm graph
            self.host_launch_s[1] += t1 - t0
            self.host_launch_s[0] += time.perf_counter() - t1
            self._joined = False
        else:
            t0 = time.perf_counter()
            for (fn, _), g in zip(self.segments, self.graphs):
                if g is None:
                    fn()
                else:
                    g.replay()
            self.host_launch_s[0] += time.perf_counter() - t0
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
