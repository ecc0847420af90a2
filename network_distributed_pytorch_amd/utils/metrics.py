"""Metrics and tracing (SURVEY.md §5.1 / §5.5 — the reference only prints epoch losses).

* :class:`JsonlLogger` — structured per-step / per-epoch records (loss, samples/s,
  bytes all-reduced: payload and modelled ring wire bytes, phase timings).
* :class:`PhaseTimer` — HIP-event timers around named phases (forward, backward,
  compress, all-reduce, update ...).  Events are recorded on the stream and resolved
  lazily, so timing adds no host synchronisation inside the step.
* :func:`print_epoch` — the reference's "Rank r, epoch e: mean loss" line
  (ddp_powersgd_guide_cifar10/ddp_init.py:183-184).
"""
from __future__ import annotations

import collections
import contextlib
import json
import os
import time
from typing import Dict, List, Optional

import torch

__all__ = ["JsonlLogger", "PhaseTimer", "print_epoch"]


class JsonlLogger:
    def __init__(self, path: Optional[str], rank: int = 0, all_ranks: bool = False):
        self.path = path
        self.enabled = path is not None and (all_ranks or rank == 0)
        self.rank = rank
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
            self._f = open(path, "a")

    def log(self, **rec):
        if not self.enabled:
            return
        rec.setdefault("time", time.time())
        rec.setdefault("rank", self.rank)
        self._f.write(json.dumps(rec) + "\n")
        self._f.flush()

    def close(self):
        if self.enabled:
            self._f.close()


class PhaseTimer:
    """Accumulate device time per named phase with HIP events (CPU: perf_counter)."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled
        self.cuda = torch.cuda.is_available()
        self._pending: List = []
        self.totals: Dict[str, float] = collections.defaultdict(float)
        self.counts: Dict[str, int] = collections.defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if self.cuda:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self._pending.append((name, a, b))
        else:
            t0 = time.perf_counter()
            yield
            self.totals[name] += (time.perf_counter() - t0) * 1e3
            self.counts[name] += 1

    def resolve(self):
        if self._pending:
            torch.cuda.synchronize()
            for name, a, b in self._pending:
                self.totals[name] += a.elapsed_time(b)
                self.counts[name] += 1
            self._pending.clear()

    def summary(self) -> Dict[str, float]:
        """Mean milliseconds per occurrence of each phase."""
        self.resolve()
        return {k: self.totals[k] / max(1, self.counts[k]) for k in self.totals}

    def reset(self):
        self.resolve()
        self.totals.clear()
        self.counts.clear()


def print_epoch(rank: int, epoch: int, mean_loss: float):
    print("     Rank ", rank, ", epoch ", epoch, ": ", mean_loss, flush=True)
