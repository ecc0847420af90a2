"""Checkpoint / resume (absent from the reference).

Layout of a checkpoint ``<path>``:

* ``<path>`` — written by rank 0: the model ``state_dict`` with torchvision / HF key names
  (compatible with the reference's model definitions), rank 0's gradient-sync state, the
  epoch / step counters, the world size and rank 0's torch RNG.
* ``<path>.rank<r>`` — written by EVERY rank r: that rank's gradient-sync state and RNG
  streams.  PowerSGD's error memory ``e = (g + e) - P Q^T`` is rank-local (M is the local
  gradient), and ranks are seeded ``seed + rank``, so a resume at N > 1 must give each
  rank its own EF residual and RNG back (a single rank-0 file replaced every
  rank's residual with rank 0's).

Loading: the model from ``<path>``; the sync state and RNG from ``<path>.rank<r>`` when it
exists (same world size), else from ``<path>`` (a world-size-1 checkpoint, or a resume
at a different world size: the EF residual then restarts from rank 0's, with a warning).
Both files carry the epoch / step counters; a per-rank file from a different save than the
rank-0 file (a crash between the ranks' writes) raises :class:`CheckpointMismatch`.
Writes are atomic (tmp file + rename).  Files contain only tensors and plain containers
and are read back with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
import warnings
from typing import Any, Dict, Optional

import torch

from ..parallel.comm import get_rank, world_size

__all__ = ["save_checkpoint", "load_checkpoint", "rank_file", "CheckpointMismatch"]


class CheckpointMismatch(RuntimeError):
    """The per-rank file and the rank-0 file of a checkpoint come from different saves."""

FORMAT = "network_distributed_pytorch_amd/ckpt-v2"


def rank_file(path: str, rank: int) -> str:
    return f"{path}.rank{rank}"


def _atomic_save(obj, path: str):
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _rng_state() -> Dict[str, Any]:
    st = {"torch_rng": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda_rng"] = torch.cuda.get_rng_state()
    return st


def _set_rng(state: Dict[str, Any]):
    if "torch_rng" in state:
        torch.set_rng_state(state["torch_rng"])
    if "cuda_rng" in state and torch.cuda.is_available():
        torch.cuda.set_rng_state(state["cuda_rng"])


def save_checkpoint(path: str, model: torch.nn.Module, sync=None, epoch: int = 0, step: int = 0,
                    extra: Optional[Dict[str, Any]] = None, rank: Optional[int] = None,
                    world: Optional[int] = None) -> Optional[str]:
    rank = get_rank() if rank is None else rank
    world = world_size() if world is None else world
    sync_state = sync.state_dict() if sync is not None and hasattr(sync, "state_dict") else None
    _atomic_save({"format": FORMAT, "rank": int(rank), "world": int(world), "sync": sync_state,
                  "epoch": int(epoch), "step": int(step), **_rng_state()}, rank_file(path, rank))
    if rank != 0:
        return None
    state = {
        "format": FORMAT,
        "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "sync": sync_state,
        "epoch": int(epoch),
        "step": int(step),
        "world": int(world),
        "extra": extra or {},
        **_rng_state(),
    }
    _atomic_save(state, path)
    return path


def load_checkpoint(path: str, model: torch.nn.Module, sync=None, strict: bool = True,
                    rank: Optional[int] = None, world: Optional[int] = None) -> Dict[str, Any]:
    rank = get_rank() if rank is None else rank
    world = world_size() if world is None else world
    state = torch.load(path, map_location="cpu", weights_only=True)
    with torch.no_grad():
        model.load_state_dict(state["model"], strict=strict)
    local = state
    rf = rank_file(path, rank)
    if os.path.exists(rf):
        own = torch.load(rf, map_location="cpu", weights_only=True)
        if (own.get("epoch"), own.get("step")) != (state["epoch"], state["step"]):
            # a partial save (crash between the ranks' atomic writes) would otherwise mix
            # epoch-e weights with another epoch's EF residual / momentum / RNG
            raise CheckpointMismatch(
                f"{rf} is from epoch {own.get('epoch')} step {own.get('step')}, {path} from epoch "
                f"{state['epoch']} step {state['step']}: the checkpoint set is from different saves")
        if own.get("world", world) == world:
            local = own
        else:
            warnings.warn(f"checkpoint was written at world size {own.get('world')}, resuming at {world}: "
                          "per-rank error memories restart from rank 0's")
    elif world > 1:
        warnings.warn(f"{rf} missing: rank {rank} resumes with rank 0's gradient-sync state")
    if sync is not None and local.get("sync") is not None and hasattr(sync, "load_state_dict"):
        sync.load_state_dict(local["sync"])
    _set_rng(local)
    return {"epoch": state["epoch"], "step": state["step"], "extra": state.get("extra", {})}
