"""Toy MLP for the ``ddp_guide`` plumbing config (BASELINE.json config 1: CPU/gloo, world 2).

The reference's ``ddp_guide`` only initialises the process group
(ddp_guide/ddp_init.py:19-47); the driver config adds a tiny model so the plumbing
exercises a real dense-DP step.
"""
from __future__ import annotations

import torch.nn as nn

__all__ = ["ToyMLP"]


class ToyMLP(nn.Module):
    def __init__(self, d_in: int = 32, d_hidden: int = 64, d_out: int = 4):
        super().__init__()
        self.fc1 = nn.Linear(d_in, d_hidden)
        self.act = nn.ReLU()
        self.fc2 = nn.Linear(d_hidden, d_out)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))
