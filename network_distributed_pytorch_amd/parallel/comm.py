"""Collective layer: world-size-guarded collectives, byte accounting, link emulation.

Reference behaviour kept:
  * ``all_reduce`` / ``all_gather`` are no-ops at world size 1
    (ddp_powersgd_guide_cifar10/reducer.py:193-195, tensor_buffer.py:59-69);
  * ``n_bits(t) = 8 * numel * element_size`` (reducer.py:197-198).

MI355X additions:
  * every collective is accounted (calls, payload bytes, modelled ring wire bytes
    2(N-1)/N * S) so the bytes/step metric is measured, not only derived;
  * :class:`LinkModel` paces each collective to an emulated 1/10/100 Gb link
    (``alpha + wire_bits / bandwidth``) by stalling the HIP stream with a wall-clock
    spin kernel (no root / ``tc`` on the GPU box) — the reference's README.md:2
    bandwidth experiments;
  * collectives run on RCCL (``backend="nccl"`` is RCCL on ROCm) over xGMI; gloo for CPU;
  * ``NDP_FORCE_COLLECTIVES=1`` issues the collectives even in a 1-rank process group
    (:attr:`Communicator.active`): a one-GPU rehearsal of the N > 1 RCCL path (async work
    handles, bucket overlap hooks, eager collectives between graph segments) whose sums
    are the identity, so results match the world-size-1 no-op path.
"""
from __future__ import annotations

import dataclasses
import os
import time
from typing import List, Optional

import torch
import torch.distributed as dist

__all__ = [
    "n_bits",
    "all_reduce",
    "all_gather",
    "world_size",
    "get_rank",
    "LinkModel",
    "CommStats",
    "Communicator",
    "LINK_PRESETS",
]


def n_bits(tensor: torch.Tensor) -> int:
    """Bits in a tensor payload (reducer.py:197-198)."""
    return 8 * tensor.nelement() * tensor.element_size()


def world_size(group=None) -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


def get_rank(group=None) -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group)
    return 0


def all_reduce(*args, **kwargs):
    """``dist.all_reduce`` guarded for world size 1 (reducer.py:193-195)."""
    if world_size(kwargs.get("group")) > 1:
        return dist.all_reduce(*args, **kwargs)
    return None


def all_gather(out_list: List[torch.Tensor], in_tensor: torch.Tensor, **kwargs):
    """``dist.all_gather`` with the single-worker aliasing fallback (tensor_buffer.py:64-69)."""
    if world_size(kwargs.get("group")) > 1:
        return dist.all_gather(out_list, in_tensor, **kwargs)
    assert len(out_list) == 1
    out_list[0].data = in_tensor
    return None


@dataclasses.dataclass
class LinkModel:
    """Emulated point-to-point link: time(S) = alpha + 8*wire(S)/bandwidth_bps."""

    bandwidth_bps: float
    alpha_s: float = 25e-6
    name: str = "custom"

    def wire_bytes(self, payload: int, n: int) -> float:
        return 0.0 if n <= 1 else 2.0 * (n - 1) / n * payload

    def seconds(self, payload: int, n: int) -> float:
        if n <= 1:
            return 0.0
        return self.alpha_s + 8.0 * self.wire_bytes(payload, n) / self.bandwidth_bps


LINK_PRESETS = {
    "1g": LinkModel(1e9, 50e-6, "1Gb"),
    "10g": LinkModel(10e9, 30e-6, "10Gb"),
    "100g": LinkModel(100e9, 10e-6, "100Gb"),
}


@dataclasses.dataclass
class CommStats:
    calls: int = 0
    payload_bytes: int = 0
    wire_bytes: float = 0.0
    emulated_seconds: float = 0.0

    def reset(self):
        self.calls = 0
        self.payload_bytes = 0
        self.wire_bytes = 0.0
        self.emulated_seconds = 0.0

    def as_dict(self):
        return dataclasses.asdict(self)


class _PacedWork:
    """Async handle that applies link pacing when waited on."""

    def __init__(self, work, comm: "Communicator", seconds: float, device_tensor: bool):
        self._work = work
        self._comm = comm
        self._seconds = seconds
        self._device = device_tensor

    def wait(self):
        if self._work is not None:
            self._work.wait()
        self._comm._pace(self._seconds, self._device)
        return True

    def is_completed(self):
        return self._work is None or self._work.is_completed()


class Communicator:
    """Accounting + pacing front-end over a c10d process group (RCCL or gloo)."""

    def __init__(self, group=None, link: Optional[LinkModel] = None):
        self.group = group
        self.link = link
        self.stats = CommStats()

    @property
    def world_size(self) -> int:
        return world_size(self.group)

    @property
    def rank(self) -> int:
        return get_rank(self.group)

    @property
    def active(self) -> bool:
        """Whether collectives are issued (world > 1, or forced for a 1-rank rehearsal)."""
        if self.world_size > 1:
            return True
        return os.environ.get("NDP_FORCE_COLLECTIVES") == "1" and dist.is_available() and dist.is_initialized()

    def _pace(self, seconds: float, device_tensor: bool):
        if seconds <= 0:
            return
        if device_tensor:
            from ..ops import delay_ns

            delay_ns(int(seconds * 1e9))
        else:
            time.sleep(seconds)

    def _account(self, t: torch.Tensor) -> float:
        n = self.world_size
        payload = t.nelement() * t.element_size()
        self.stats.calls += 1
        self.stats.payload_bytes += payload
        self.stats.wire_bytes += 0.0 if n <= 1 else 2.0 * (n - 1) / n * payload
        secs = self.link.seconds(payload, n) if self.link is not None else 0.0
        self.stats.emulated_seconds += secs
        return secs

    def all_reduce(self, t: torch.Tensor, async_op: bool = False, op=None):
        secs = self._account(t)
        if not self.active:
            return _PacedWork(None, self, 0.0, t.is_cuda) if async_op else None
        kw = {"group": self.group}
        if op is not None:
            kw["op"] = op
        if async_op:
            work = dist.all_reduce(t, async_op=True, **kw)
            return _PacedWork(work, self, secs, t.is_cuda)
        dist.all_reduce(t, **kw)
        self._pace(secs, t.is_cuda)
        return None

    def all_gather(self, out_list: List[torch.Tensor], t: torch.Tensor, async_op: bool = False):
        self._account(t)
        if not self.active:
            assert len(out_list) == 1
            out_list[0].copy_(t)
            return None
        return dist.all_gather(out_list, t, group=self.group, async_op=async_op)

    def broadcast(self, t: torch.Tensor, src: int = 0):
        if not self.active:
            return None
        return dist.broadcast(t, src=src, group=self.group)

    def barrier(self):
        if self.active:
            dist.barrier(group=self.group)
