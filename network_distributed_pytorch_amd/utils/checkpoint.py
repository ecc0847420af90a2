"""Checkpoint / resume (absent from the reference).

A checkpoint holds the model ``state_dict`` with torchvision / HF key names (so it stays
compatible with the reference's model definitions), the gradient-sync state (PowerSGD:
error memories, momenta, the warm-start query ``q_warm`` and the reducer's numpy RNG;
dense: momentum buffer), the epoch / step counters and the torch RNG.  Rank 0 writes
atomically (tmp file + rename); every rank loads.  Files contain only tensors and plain
containers and are read back with ``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch

from ..parallel.comm import get_rank

__all__ = ["save_checkpoint", "load_checkpoint"]


def save_checkpoint(path: str, model: torch.nn.Module, sync=None, epoch: int = 0, step: int = 0,
                    extra: Optional[Dict[str, Any]] = None, rank: Optional[int] = None) -> Optional[str]:
    rank = get_rank() if rank is None else rank
    if rank != 0:
        return None
    state = {
        "format": "network_distributed_pytorch_amd/ckpt-v1",
        "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "sync": sync.state_dict() if sync is not None and hasattr(sync, "state_dict") else None,
        "epoch": int(epoch),
        "step": int(step),
        "torch_rng": torch.get_rng_state(),
        "extra": extra or {},
    }
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str, model: torch.nn.Module, sync=None, strict: bool = True) -> Dict[str, Any]:
    state = torch.load(path, map_location="cpu", weights_only=True)
    with torch.no_grad():
        missing, unexpected = model.load_state_dict(state["model"], strict=strict)
    if sync is not None and state.get("sync") is not None and hasattr(sync, "load_state_dict"):
        sync.load_state_dict(state["sync"])
    if "torch_rng" in state:
        torch.set_rng_state(state["torch_rng"])
    return {"epoch": state["epoch"], "step": state["step"], "extra": state.get("extra", {})}
