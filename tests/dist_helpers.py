"""Rank bodies for multi-process gloo tests (module-level so ``spawn`` can pickle them)."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def _init(rank, world):
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)


def _dev():
    if os.environ.get("NDP_TEST_DEVICE") == "cuda" and torch.cuda.is_available():
        return torch.device("cuda", 0)
    return torch.device("cpu")


def reducer_rank_body(rank, world, out_dir, R):
    """Each rank reduces different send buffers; dump outs / mems / Q for the parent."""
    from network_distributed_pytorch_amd.parallel.comm import Communicator
    from network_distributed_pytorch_amd.parallel.powersgd import PowerSGDReducer

    _init(rank, world)
    dev = _dev()
    shapes = [(16, 3, 3, 3), (16,), (10, 32), (10,), (7, 5)]
    g = torch.Generator().manual_seed(100 + rank)
    Ms = [torch.randn(s, generator=g) for s in shapes]
    red = PowerSGDReducer(714, dev, 0, True, rank=R, comm=Communicator())
    outs = [torch.zeros(s, device=dev) for s in shapes]
    mems = [torch.zeros(s, device=dev) for s in shapes]
    q0 = None
    rec = []
    for call in range(2):
        bits = red.reduce([m.to(dev) for m in Ms], outs, mems)
        if q0 is None:
            q0 = red._buf.q_warm.clone().cpu()
        rec.append({"outs": [o.cpu().clone() for o in outs], "mems": [m.cpu().clone() for m in mems],
                    "q": red._buf.q_warm.cpu().clone(), "bits": bits})
    torch.save({"Ms": Ms, "rec": rec}, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def train_rank_body(rank, world, out_dir, kind, steps, native):
    """Train a small CNN with a grad-sync strategy; dump final params + checksums."""
    _init(rank, world)
    _train(rank, world, out_dir, kind, steps, native)
    dist.destroy_process_group()


def _train(rank, world, out_dir, kind, steps, native, comm=None, tag=None):
    from network_distributed_pytorch_amd.parallel.comm import Communicator
    from network_distributed_pytorch_amd.parallel.trainer import build_grad_sync

    dev = _dev()
    torch.manual_seed(1000 + rank)  # different init per rank: the sync must broadcast
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8), torch.nn.ReLU(),
                                torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 5)).to(dev)
    if kind in ("dense-ref", "powersgd-ref"):
        for p in model.parameters():  # reference has no broadcast: seed identically instead
            dist.broadcast(p.data, 0)
    kw = {"native": native} if kind == "powersgd" else {}
    sync = build_grad_sync(kind, model, comm or Communicator(), lr=0.05, momentum=0.9, rank=2, **kw)
    g = torch.Generator().manual_seed(7 + rank)
    losses = []
    for _ in range(steps):
        x = torch.randn(16, 3, 8, 8, generator=g).to(dev)
        y = torch.randint(0, 5, (16,), generator=g).to(dev)
        sync.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        sync.step()
        losses.append(float(loss))
    params = [p.detach().cpu().clone() for p in model.parameters()]
    torch.save({"params": params, "losses": losses}, os.path.join(out_dir, f"{tag or kind}_rank{rank}.pt"))


def checker_rank_body(rank, world, out_dir):
    """ReplicaChecker must catch a corrupted collective result on one rank."""
    from network_distributed_pytorch_amd.parallel.comm import Communicator
    from network_distributed_pytorch_amd.parallel.trainer import build_grad_sync
    from network_distributed_pytorch_amd.utils.divergence import FaultInjector, ReplicaChecker, ReplicaDivergence

    _init(rank, world)
    torch.manual_seed(0)
    model = torch.nn.Linear(6, 3)
    comm = FaultInjector(Communicator(), mode="corrupt", rank=1, call_index=3)
    sync = build_grad_sync("powersgd", model, comm, lr=0.1, momentum=0.9, rank=2)
    checker = ReplicaChecker(comm, sync.opt.x, every=1, strict=True)
    caught = None
    for step in range(4):
        sync.zero_grad()
        model(torch.randn(4, 6)).sum().backward()
        sync.step()
        try:
            checker.check(step)
        except ReplicaDivergence as e:
            caught = step
            break
    torch.save({"caught": caught, "fired": comm.fired}, os.path.join(out_dir, f"chk{rank}.pt"))
    dist.destroy_process_group()


def forced_rank_body(rank, world, out_dir, kind, force):
    """1-rank group: collectives issued (NDP_FORCE_COLLECTIVES=1) vs skipped."""
    os.environ["NDP_FORCE_COLLECTIVES"] = "1" if force else "0"
    from network_distributed_pytorch_amd.parallel.comm import Communicator

    _init(rank, world)
    comm = Communicator()
    calls = []
    orig = dist.all_reduce

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    dist.all_reduce = counting
    try:
        _train(rank, world, out_dir, kind, 3, False, comm=comm, tag=f"{kind}_f{int(force)}")
    finally:
        dist.all_reduce = orig
    torch.save({"calls": len(calls), "active": comm.active},
               os.path.join(out_dir, f"{kind}_f{int(force)}_meta.pt"))
    dist.destroy_process_group()
