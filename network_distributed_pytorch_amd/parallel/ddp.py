"""Dense data parallelism: the reference's blocking per-parameter arm and a bucketed,
backward-overlapped MI355X arm.

* :func:`average_gradients` — reference semantics (ddp_guide_cifar10/ddp_init.py:57-62):
  one blocking SUM all-reduce per parameter followed by ``grad /= world_size``.
* :class:`BucketedDataParallel` — gradients live in ONE flat arena laid out in reverse
  parameter order (≈ backward production order) and cut into contiguous buckets
  (default 25 MB: few, large RCCL all-reduces that saturate a ring over the 7 xGMI
  links).  A post-accumulate-grad hook launches each bucket's async all-reduce as soon
  as its last gradient lands, so communication overlaps the rest of backward; ``step()``
  waits and runs ONE fused gfx950 SGD-momentum kernel over the arena with the ``/N``
  mean folded in (the reference's ``grad /= N`` + ``optim.SGD.step``).
  Parameters are broadcast from rank 0 at construction (quirk Q4 fixed).
"""
from __future__ import annotations

from typing import List, Optional

import torch

from ..ops import SegPlan, capturing, sgd_momentum_
from .comm import Communicator, all_reduce, world_size

__all__ = ["average_gradients", "BucketedDataParallel"]


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
                 momentum: float = 0.9, bucket_mb: float = 25.0, broadcast_params: bool = True,
                 overlap: bool = True):
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
        self._ready = [0] * len(self.buckets)
        self._works = [None] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self.overlap = overlap and self.comm.active
        self._hooks = []
        if self.overlap:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self.step_count = 0

    @property
    def bytes_per_step(self) -> int:
        return 4 * sum(p.numel() for p in self.params)

    @property
    def collectives_per_step(self) -> int:
        return len(self.buckets) if self.comm.active else 0

    def _flatten(self, b: int):
        _, _, ps = self.buckets[b]
        specs = []
        for p in ps:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            o = self.offsets[id(p)]
            specs.append((p.grad.reshape(-1), self.g[o: o + p.numel()], 1, 0, 1.0))
        seg = self._segs[b]
        seg.set(specs)
        seg.run()                      # one flatten launch per bucket

    def _allreduce(self, b: int):
        s, e, _ = self.buckets[b]
        if self.comm.active:
            self._works[b] = self.comm.all_reduce(self.g[s:e], async_op=True)

    def _launch(self, b: int):
        self._flatten(b)
        self._allreduce(b)
        self._launched[b] = True

    def _on_grad(self, p):
        if not self.overlap:
            return
        b = self.bucket_of[id(p)]
        self._ready[b] += 1
        if self._ready[b] == len(self.buckets[b][2]) and not self._launched[b]:
            self._launch(b)

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
        self.overlap = False  # hooks must not launch collectives inside a captured backward
        return [(self.phase_flatten, False), (self.comm_buckets, True), (self.phase_sgd, False)]

    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            p.grad = None
        self._ready = [0] * len(self.buckets)
        self._works = [None] * len(self.buckets)
        self._launched = [False] * len(self.buckets)

    @torch.no_grad()
    def step(self) -> int:
        n = self.comm.world_size
        for b in range(len(self.buckets)):
            if not self._launched[b]:  # overlap disabled / unused params
                self._launch(b)
        for w in self._works:
            if w is not None:
                w.wait()
        sgd_momentum_(self.x, self.g, self.buf, self.lr, self.momentum, float(n))
        self.count_step()
        return 8 * self.bytes_per_step

    def count_step(self):
        if not capturing():
            self.step_count += 1

    def state_dict(self):
        return {"momentum_buffer": self.buf.detach().cpu().clone(), "lr": self.lr, "momentum": self.momentum}

    def load_state_dict(self, sd):
        self.buf.copy_(sd["momentum_buffer"])
        self.lr = float(sd["lr"])
        self.momentum = float(sd["momentum"])
