"""Dense data parallelism: the reference's blocking per-parameter arm and a bucketed,
backward-overlapped MI355X arm.

* :func:`average_gradients` — reference semantics (ddp_guide_cifar10/ddp_init.py:57-62):
  one blocking SUM all-reduce per parameter followed by ``grad /= world_size``.
* :class:`BucketedDataParallel` — gradients live in ONE arena laid out in reverse
  parameter order (≈ backward production order) and cut into contiguous buckets.  The
  native conv / BN backwards write their parameters' gradients straight into the arena
  slices (ops/gradarena.py, adopted by autograd as ``.grad``); only gradients produced
  elsewhere (ATen Linear, MIOpen) are copied in by the bucket's flatten launch.
  A post-accumulate-grad hook launches each bucket as soon as its last gradient lands, in
  bucket order on every rank:
    - stream-ordered data plane (native RCCL communicator, csrc/comm.cpp; or world size
      1): the flatten kernel and the bucket all-reduce go on the communicator's side
      stream, forked from the compute stream with a hipEvent, so they run concurrently
      with the rest of backward — also inside a captured hipGraph (the fork/join events are
      capture-legal).  ``step()`` joins the side stream and runs ONE fused gfx950
      SGD-momentum kernel over the arena with the ``/N`` mean folded in (the reference's
      ``grad /= N`` + ``optim.SGD.step``).
    - c10d data plane (gloo CPU tests, ``NDP_NATIVE_COMM=0``): flatten on the compute
      stream + async c10d all-reduce; ``step()`` waits on the work handles.
  Bucket size (default ``DEFAULT_BUCKET_MB``): on MI355X each GPU has 7 xGMI links of
  ≈153 GB/s (one ring uses one link per direction); RCCL reaches its large-message ring
  bandwidth from a few MB per message while per-collective latency is tens of µs, so a
  bucket of ~8 MB keeps the launch count low (ResNet-18: 6 buckets; DistilBERT: 33)
  and the first bucket starts after the classifier + last block instead of after half of
  backward.  Modelled, not measured at N > 1 (no multi-GPU box in the build loop); the
  knob is ``bucket_mb`` / ``-bucket_mb`` / ``--bucket-mb``.
  Parameters are broadcast from rank 0 at construction (quirk Q4 fixed).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from ..ops import SegPlan, capturing, gradarena, gradfinish, sgd_momentum_
from .comm import Communicator, all_reduce, world_size

__all__ = ["average_gradients", "BucketedDataParallel", "DEFAULT_BUCKET_MB"]

DEFAULT_BUCKET_MB = 8.0


def average_gradients(model: torch.nn.Module, comm: Optional[Communicator] = None) -> int:
    """Blocking per-parameter SUM all-reduce then ``/= N`` (ddp_init.py:57-62). Returns bits."""
    bits = 0
    size = float(comm.world_size if comm is not None else world_size())
    for p in model.parameters():
        if p.grad is None:
            continue
        if comm is not None:
            comm.all_reduce(p.grad.data)
        else:
            all_reduce(p.grad.data)
        p.grad.data /= size
        bits += 8 * p.grad.numel() * p.grad.element_size()
    return bits


class BucketedDataParallel:
    def __init__(self, model: torch.nn.Module, comm: Optional[Communicator] = None, lr: float = 1e-3,
                 momentum: float = 0.9, bucket_mb: Optional[float] = None, broadcast_params: bool = True,
                 overlap: Optional[bool] = None):
        bucket_mb = DEFAULT_BUCKET_MB if bucket_mb is None else float(bucket_mb)
        self.model = model
        self.comm = comm if comm is not None else Communicator()
        self.lr = float(lr)
        self.momentum = float(momentum)
        self.params: List[torch.nn.Parameter] = [p for p in model.parameters() if p.requires_grad]
        self.device = self.params[0].device
        order = list(reversed(self.params))
        offs, o = {}, 0
        for p in order:
            offs[id(p)] = o
            o += (p.numel() + 15) // 16 * 16
        self.numel = o
        self.offsets = offs
        f32 = dict(dtype=torch.float32, device=self.device)
        self.x = torch.zeros(o, **f32)
        self.g = torch.zeros(o, **f32)
        self.buf = torch.zeros(o, **f32)
        with torch.no_grad():
            for p in self.params:
                s = offs[id(p)]
                v = self.x[s: s + p.numel()].view_as(p)
                v.copy_(p.data)
                p.data = v
                p.grad = None
        if broadcast_params:
            self.comm.broadcast(self.x, src=0)
        # the native backwards write these parameters' gradients straight into their arena
        # slices (ops/gradarena.py): no flatten copy for them
        if self.device.type == "cuda":
            for p in self.params:
                gradarena.register(p, self.g, offs[id(p)])
        # buckets: contiguous arena ranges in backward order
        cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        self.buckets = []  # [start, end, [params]]
        self.bucket_of = {}
        cur, start, cur_end = [], 0, 0
        for p in order:
            s = offs[id(p)]
            e = s + (p.numel() + 15) // 16 * 16
            if cur and e - start > cap:
                self.buckets.append([start, cur_end, cur])
                start, cur = s, []
            self.bucket_of[id(p)] = len(self.buckets)
            cur.append(p)
            cur_end = e
        if cur:
            self.buckets.append([start, cur_end, cur])
        self._segs = [SegPlan([], self.device, capacity=len(b[2])) for b in self.buckets]
        self._copies = [True] * len(self.buckets)
        self._ready = [0] * len(self.buckets)
        self._works = [None] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._next = 0
        if overlap is None:  # default: overlap only when a step has wire time to hide
            overlap = self.comm.has_traffic
        # stream mode (overlap on a stream-ordered data plane: native RCCL / IPC / world 1):
        # flatten + collective + SGD on the side stream.  Without overlap everything stays on
        # the compute stream — at N = 1 the captured step is ONE serial graph, no side stream,
        # no device-flag waits
        self.stream_mode = self.device.type == "cuda" and self.comm.stream_ordered and bool(overlap)
        self.overlap = overlap and (self.comm.active or self.stream_mode)
        self._hooks = []
        if overlap:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self.step_count = 0

    @property
    def bytes_per_step(self) -> int:
        return 4 * sum(p.numel() for p in self.params)

    @property
    def collectives_per_step(self) -> int:
        return len(self.buckets) if self.comm.active else 0

    def collective_payloads(self):
        """Bytes of every bucket all-reduce of one step (link-model input)."""
        return [4 * (e - s) for s, e, _ in self.buckets]

    def _bind(self, b: int) -> bool:
        """Copy table of bucket b's gradients that are NOT already in the arena; False if
        every gradient was written in place (no flatten launch)."""
        _, _, ps = self.buckets[b]
        specs = []
        for p in ps:
            o = self.offsets[id(p)]
            dst = self.g[o: o + p.numel()]
            if p.grad is None:  # unused parameter: zero gradient, in place
                p.grad = dst.view_as(p)
                p.grad.zero_()
            if p.grad.data_ptr() == dst.data_ptr():
                continue
            specs.append((p.grad.reshape(-1), dst, 1, 0, 1.0))
        self._segs[b].set(specs)
        self._copies[b] = bool(specs)
        return self._copies[b]

    def _flatten(self, b: int):
        if self._bind(b):
            self._segs[b].run()        # one flatten launch per bucket (only copied gradients)

    def _allreduce(self, b: int):
        s, e, _ = self.buckets[b]
        if self.comm.has_traffic:  # N > 1, or a 1-GPU link emulation (pacing only, no data)
            self._works[b] = self.comm.all_reduce(self.g[s:e], async_op=True)

    def _launch(self, b: int):
        gradfinish.flush()  # deferred conv grad-W sums / folds (launches on the compute stream)
        if self.stream_mode:
            copies = self._bind(b)     # table upload on the compute stream, before the fork

            def flatten_reduce():
                if copies:
                    self._segs[b].run()
                self._allreduce(b)     # ddp_guide_cifar10/ddp_init.py:61, one per bucket
            self.comm.side_launch(flatten_reduce)
        else:
            self._flatten(b)
            self._allreduce(b)
        self._launched[b] = True

    def _on_grad(self, p):
        if not self.overlap:
            return
        b = self.bucket_of[id(p)]
        self._ready[b] += 1
        # launch in bucket order on every rank (identical collective sequence everywhere)
        while self._next < len(self.buckets) and not self._launched[self._next] and \
                self._ready[self._next] == len(self.buckets[self._next][2]):
            self._launch(self._next)
            self._next += 1

    # -- piecewise-graph phases (collectives run eagerly between captured phases) -----------
    @torch.no_grad()
    def phase_flatten(self):
        for b in range(len(self.buckets)):
            self._flatten(b)

    @torch.no_grad()
    def comm_buckets(self):
        for b in range(len(self.buckets)):
            self._allreduce(b)
        for b, w in enumerate(self._works):
            if w is not None:
                w.wait()
            self._works[b] = None

    @torch.no_grad()
    def phase_sgd(self):
        sgd_momentum_(self.x, self.g, self.buf, self.lr, self.momentum, float(self.comm.world_size))
        self.count_step()

    def phases(self):
        self.overlap = False  # piecewise capture: collectives run eagerly between segments
        self.stream_mode = False
        return [(self.phase_flatten, False), (self.comm_buckets, True), (self.phase_sgd, False)]

    def _reset(self):
        self._ready = [0] * len(self.buckets)
        self._works = [None] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._next = 0

    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            p.grad = None
        gradarena.release(self.params)
        self._reset()

    @torch.no_grad()
    def step(self) -> int:
        n = self.comm.world_size
        for b in range(len(self.buckets)):
            if not self._launched[b]:  # overlap disabled / unused params
                self._launch(b)
        if self.stream_mode:
            # the fused SGD runs on the side stream too (it needs every bucket), then join
            lr, mu = self.lr, self.momentum
            self.comm.side_launch(lambda: sgd_momentum_(self.x, self.g, self.buf, lr, mu, float(n)))
            self.comm.side_join()
        else:
            for w in self._works:
                if w is not None:
                    w.wait()
            sgd_momentum_(self.x, self.g, self.buf, self.lr, self.momentum, float(n))
        self._reset()
        self.count_step()
        return 8 * self.bytes_per_step

    def snapshot(self):
        return {"x": self.x.clone(), "buf": self.buf.clone(), "step_count": self.step_count}

    def restore(self, snap):
        self.x.copy_(snap["x"])
        self.buf.copy_(snap["buf"])
        self.step_count = snap["step_count"]

    def count_step(self):
        if not capturing():
            self.step_count += 1

    def state_dict(self):
        return {"momentum_buffer": self.buf.detach().cpu().clone(), "lr": self.lr, "momentum": self.momentum}

    def load_state_dict(self, sd):
        self.buf.copy_(sd["momentum_buffer"])
        self.lr = float(sd["lr"])
        self.momentum = float(sd["momentum"])
