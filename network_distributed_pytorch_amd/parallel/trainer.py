"""Gradient-synchronisation strategies behind one interface (zero_grad / step).

``build_grad_sync(kind, model, comm, ...)``:

=================  ===========================================================================
``powersgd``       fused native engine (:class:`PowerSGDOptimizer`): EF + PowerSGD + momentum
                   + SGD over flat arenas; on a device the per-group pipelines (6 gfx950
                   launches + 2 collectives each) overlap backward on the side stream.
``powersgd-ref``   reference semantics, eager per-tensor loops (ddp_init.py:149-178 with the
                   reducer's torch path) — the "eager reference" comparison arm.
``dense``          bucketed all-reduce overlapped with backward + fused SGD-momentum kernel.
``dense-ref``      reference dense arm: blocking per-parameter all-reduce + torch.optim.SGD
                   (ddp_guide_cifar10/ddp_init.py:57-62,111,124-125).
=================  ===========================================================================
"""
from __future__ import annotations

from typing import Optional

import torch

from .comm import Communicator
from .ddp import BucketedDataParallel, average_gradients
from .powersgd import PowerSGDOptimizer, PowerSGDReducer, powersgd_bytes_per_step

__all__ = ["build_grad_sync", "ReferencePowerSGDLoop", "ReferenceDenseLoop", "PowerSGDSync"]


class PowerSGDSync:
    def __init__(self, model, comm, lr, momentum, rank, seed=714, **kw):
        self.opt = PowerSGDOptimizer(model.parameters(), lr=lr, momentum=momentum, rank=rank,
                                     random_seed=seed, comm=comm, **kw)
        b = powersgd_bytes_per_step(list(model.parameters()), rank)
        self.bytes_per_step = b["total"]

    @property
    def collectives_per_step(self):
        return self.opt.collectives_per_step

    @property
    def comm(self):
        return self.opt.comm

    def collective_payloads(self):
        return self.opt.collective_payloads()

    def zero_grad(self):
        self.opt.zero_grad()

    def step(self):
        return self.opt.step()

    def phases(self):
        return self.opt.phases()

    def count_step(self):
        self.opt.count_step()

    def prepare(self):
        self.opt.prepare()

    def snapshot(self):
        return self.opt.snapshot()

    def restore(self, snap):
        self.opt.restore(snap)

    def check_errors(self):
        self.opt.check_errors()

    def state_dict(self):
        return self.opt.state_dict()

    def load_state_dict(self, sd):
        self.opt.load_state_dict(sd)


class ReferencePowerSGDLoop:
    """Algorithm 2 exactly as the reference loop writes it (ddp_init.py:130-178)."""

    def __init__(self, model, comm, lr, momentum, rank, seed=714, native_reducer=False):
        self.model = model
        self.params = list(model.parameters())
        self.lr, self.lam = lr, momentum
        self.reducer = PowerSGDReducer(seed, self.params[0].device, 0, True, rank=rank, comm=comm)
        self.native_reducer = native_reducer
        self.memories = [torch.zeros_like(p) for p in self.params]
        self.send_buffers = [torch.zeros_like(p) for p in self.params]
        self.momenta = [torch.empty_like(p) for p in self.params]
        self.first = True
        self.bits = 0
        b = powersgd_bytes_per_step(self.params, rank)
        self.bytes_per_step = b["total"]
        self._payloads = [b["p"], b["rank1"], b["q"]]  # reducer.py:126, :132, :145
        self.collectives_per_step = 3 if comm.active else 0

    def collective_payloads(self):
        return list(self._payloads)

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    @torch.no_grad()
    def step(self):
        grads = [p.grad for p in self.params]
        for g, e, s in zip(grads, self.memories, self.send_buffers):
            s.data[:] = g + e
        if self.native_reducer:
            self.bits += self.reducer.reduce(self.send_buffers, grads, self.memories)
        else:
            self.bits += self.reducer.reduce_torch(self.send_buffers, grads, self.memories)
        for g, m in zip(grads, self.momenta):
            if self.first:
                m.data = g.clone().detach()
            else:
                m.mul_(self.lam).add_(g)
            g.data[:] += m
        self.first = False
        for p, g in zip(self.params, grads):
            p.data.add_(g, alpha=-self.lr)
        return self.bytes_per_step * 8


class ReferenceDenseLoop:
    def __init__(self, model, comm, lr, momentum):
        self.model = model
        self.comm = comm
        self.opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=momentum)
        self.bytes_per_step = 4 * sum(p.numel() for p in model.parameters())
        self._payloads = [4 * p.numel() for p in model.parameters()]  # ddp_init.py:61, one per param
        self.collectives_per_step = len(list(model.parameters())) if comm.active else 0

    def collective_payloads(self):
        return list(self._payloads)

    def zero_grad(self):
        self.opt.zero_grad()

    def step(self):
        bits = average_gradients(self.model, self.comm)
        self.opt.step()
        return bits


class _DenseSync:
    def __init__(self, model, comm, lr, momentum, bucket_mb, overlap=None):
        self.ddp = BucketedDataParallel(model, comm, lr=lr, momentum=momentum, bucket_mb=bucket_mb, overlap=overlap)
        self.bytes_per_step = self.ddp.bytes_per_step

    @property
    def collectives_per_step(self):
        return self.ddp.collectives_per_step

    @property
    def comm(self):
        return self.ddp.comm

    def collective_payloads(self):
        return self.ddp.collective_payloads()

    def snapshot(self):
        return self.ddp.snapshot()

    def restore(self, snap):
        self.ddp.restore(snap)

    def check_errors(self):
        self.ddp.comm.check()

    def zero_grad(self):
        self.ddp.zero_grad()

    def step(self):
        return self.ddp.step()

    def phases(self):
        return self.ddp.phases()

    def count_step(self):
        self.ddp.count_step()

    def state_dict(self):
        return self.ddp.state_dict()

    def load_state_dict(self, sd):
        self.ddp.load_state_dict(sd)


def build_grad_sync(kind: str, model: torch.nn.Module, comm: Optional[Communicator] = None, lr: float = 1e-3,
                    momentum: float = 0.9, rank: int = 4, bucket_mb: Optional[float] = None, seed: int = 714,
                    **kw):
    comm = comm if comm is not None else Communicator()
    if kind == "powersgd":
        return PowerSGDSync(model, comm, lr, momentum, rank, seed=seed, **kw)
    if kind == "powersgd-ref":
        return ReferencePowerSGDLoop(model, comm, lr, momentum, rank, seed=seed)
    if kind == "powersgd-api":
        return ReferencePowerSGDLoop(model, comm, lr, momentum, rank, seed=seed, native_reducer=True)
    if kind == "dense":
        return _DenseSync(model, comm, lr, momentum, bucket_mb, overlap=kw.get("overlap"))
    if kind == "dense-ref":
        return ReferenceDenseLoop(model, comm, lr, momentum)
    if kind in ("local-sgd-nesterov", "local-adamw"):
        return LocalOptimizer(model, kind, lr, momentum)
    raise ValueError(f"unknown grad sync {kind!r}")


class LocalOptimizer:
    """Single-GPU baselines, no communication (reference C17):
    ``local-sgd-nesterov`` = SGD(lr, momentum=0.9, nesterov=True)
    (ddp_powersgd_distillBERT_IMDb/IMDb_distillBERT_example.py:57);
    ``local-adamw`` = AdamW(lr) (IMDb_dataset_distributer.py:55)."""

    def __init__(self, model, kind, lr, momentum):
        if kind == "local-adamw":
            self.opt = torch.optim.AdamW(model.parameters(), lr=lr)
        else:
            self.opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=momentum, nesterov=True)
        self.bytes_per_step = 0
        self.collectives_per_step = 0

    def zero_grad(self):
        self.opt.zero_grad()

    def step(self):
        self.opt.step()
        return 0

    def state_dict(self):
        return self.opt.state_dict()

    def load_state_dict(self, sd):
        self.opt.load_state_dict(sd)
