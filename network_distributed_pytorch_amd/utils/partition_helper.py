"""Dataset partitioning, API- and permutation-compatible with the reference.

Reference: ddp_guide_cifar10/partition_helper.py:4-35 (copied verbatim into every
experiment directory).  Semantics kept exactly:
  * one shuffle of ``range(len(data))`` with ``random.Random(seed)`` (seed 1234 by
    default, so every rank computes the SAME permutation and the shards are disjoint);
  * consecutive slices of ``int(frac * len)`` indices; the remainder is dropped;
  * ``Partition`` is an index-remapped view: ``part[i] == data[index[i]]``.

Additions for device-resident data: ``Partition.index_tensor()`` (the shard as an int64
tensor for on-device gathers) and ``DataPartitioner.shard(rank, world)``.
"""
from __future__ import annotations

import random
from typing import List, Sequence

import torch

__all__ = ["Partition", "DataPartitioner"]


class Partition:
    def __init__(self, data, index: Sequence[int]):
        self.data = data
        self.index = list(index)

    def __len__(self) -> int:
        return len(self.index)

    def __getitem__(self, i):
        return self.data[self.index[i]]

    def index_tensor(self, device=None) -> torch.Tensor:
        return torch.as_tensor(self.index, dtype=torch.int64, device=device)


class DataPartitioner:
    def __init__(self, data, sizes: Sequence[float] = (0.7, 0.2, 0.1), seed: int = 1234):
        self.data = data
        n = len(data)
        order: List[int] = list(range(n))
        random.Random(seed).shuffle(order)
        self.partitions: List[List[int]] = []
        pos = 0
        for frac in sizes:
            take = int(frac * n)
            self.partitions.append(order[pos: pos + take])
            pos += take

    def use(self, partition: int) -> Partition:
        return Partition(self.data, self.partitions[partition])

    @classmethod
    def shard(cls, data, rank: int, world: int, seed: int = 1234) -> Partition:
        """Equal shards for ``world`` workers (the reference's ``[1/size] * size``)."""
        return cls(data, [1.0 / world] * world, seed).use(rank)
