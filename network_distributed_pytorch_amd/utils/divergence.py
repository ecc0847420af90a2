"""Replica-divergence detection and fault injection.

Data parallelism is only correct while every rank holds bitwise-identical parameters.
The reference never checks it (and its HF head is seeded per rank, quirk Q3).

* :class:`ReplicaChecker` — every ``every`` steps, a deterministic fp64 checksum of the
  flat parameter arena (one gfx950 kernel) is all-gathered; any mismatch is reported
  with the offending ranks (and raises when ``strict``).
* :class:`FaultInjector` — a :class:`Communicator` wrapper that corrupts one rank's copy
  of a chosen collective's result (silent divergence), delays it (straggler / timeout
  testing) or, at world size 1, drops it — used by tests to prove the checker catches a
  diverged replica and that timeouts surface.
"""
from __future__ import annotations

import time
from typing import List, Optional

import torch

from ..ops import checksum
from ..parallel.comm import Communicator

__all__ = ["ReplicaChecker", "ReplicaDivergence", "FaultInjector"]


class ReplicaDivergence(RuntimeError):
    pass


class ReplicaChecker:
    def __init__(self, comm: Communicator, flat_params: torch.Tensor, every: int = 100, strict: bool = True):
        self.comm = comm
        self.flat = flat_params
        self.every = max(1, every)
        self.strict = strict
        self.history: List[dict] = []

    def check(self, step: int, force: bool = False) -> bool:
        if not force and step % self.every:
            return True
        on_dev = self.comm.world_size > 1 and self.flat.is_cuda
        if on_dev:
            import torch.distributed as dist
            on_dev = dist.get_backend(self.comm.group) != "gloo"  # gloo gathers host tensors only
        local = torch.tensor([checksum(self.flat)], dtype=torch.float64, device=self.flat.device if on_dev else "cpu")
        outs = [torch.zeros_like(local) for _ in range(self.comm.world_size)]
        if self.comm.world_size > 1:
            import torch.distributed as dist
            dist.all_gather(outs, local, group=self.comm.group)
        else:
            outs = [local]
        vals = [float(o.item()) for o in outs]
        ok = all(v == vals[0] for v in vals)
        self.history.append({"step": step, "ok": ok, "checksums": vals})
        if not ok and self.strict:
            bad = [r for r, v in enumerate(vals) if v != vals[0]]
            raise ReplicaDivergence(f"replicas diverged at step {step}: ranks {bad} differ from rank 0 ({vals})")
        return ok


class FaultInjector(Communicator):
    """Communicator that skips or delays the ``call_index``-th collective on ``rank``."""

    def __init__(self, base: Communicator, mode: str = "drop", rank: int = 0, call_index: int = 0,
                 delay_s: float = 0.0):
        super().__init__(base.group, base.link)
        self.stats = base.stats
        self.mode = mode
        self.target_rank = rank
        self.call_index = call_index
        self.delay_s = delay_s
        self._calls = 0
        self.fired = False

    def all_reduce(self, t, async_op: bool = False, op=None):
        idx = self._calls
        self._calls += 1
        hit = idx == self.call_index and self.rank == self.target_rank
        if hit and self.mode == "delay":
            self.fired = True
            time.sleep(self.delay_s)
        if hit and self.mode == "drop" and self.world_size == 1:
            self.fired = True
            return None
        work = super().all_reduce(t, async_op=async_op, op=op)
        if hit and self.mode == "corrupt":
            # the collective happened, but this rank's copy of the result is perturbed:
            # a silent replica divergence (bit flip / bad link) the checker must catch
            self.fired = True
            if work is not None:
                work.wait()
                work = None if not async_op else _Done()
            t.view(-1)[:1].add_(1e-3)
        return work


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True
