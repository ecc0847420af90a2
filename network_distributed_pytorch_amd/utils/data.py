"""Synthetic, device-resident datasets with the reference's shapes + an on-device loader.

The reference downloads CIFAR-10 with torchvision (ddp_guide_cifar10/ddp_init.py:37-55)
and tokenizes aclImdb with the HF tokenizer (ddp_powersgd_distillBERT_IMDb/ddp_init.py:
56-94).  Neither torchvision, the datasets nor the network exist on the GPU boxes, so:

* :class:`SyntheticCIFAR10` — 50,000 x (3, 32, 32) float images in [-1, 1] (what
  ``ToTensor + Normalize(0.5, 0.5)`` produces) and 10 labels.  Images carry a
  class-dependent low-frequency pattern under noise so the task is learnable and loss
  curves mean something.
* :class:`SyntheticIMDb` — 25,000 reviews as ``input_ids`` / ``attention_mask`` of length
  512 (the tokenizer's ``truncation=True, padding=True`` output shape), binary labels,
  a label-dependent token distribution, and :func:`train_val_split` with a FIXED seed so
  every rank sees the same split (quirk Q2 fixed: the reference splits per rank with an
  unseeded ``train_test_split``).

Both generate identically on every rank from a seed (so ``DataPartitioner`` shards are
disjoint), and live in HBM: 614 MB for CIFAR is nothing next to 288 GB.
:class:`DeviceLoader` replaces ``DataLoader(partition, batch_size, shuffle=True)``:
per-epoch shuffles and batch gathers happen on the GPU (no host->device copy per step).
"""
from __future__ import annotations

import math
from typing import Dict, Iterator, Optional, Sequence, Union

import torch

from .partition_helper import Partition

__all__ = ["SyntheticCIFAR10", "SyntheticIMDb", "train_val_split", "DeviceLoader", "TensorDictDataset"]


class TensorDictDataset:
    """Columns of equal length; ``ds[i]`` returns a dict (or tuple) of row i."""

    def __init__(self, columns: Dict[str, torch.Tensor], as_tuple: Optional[Sequence[str]] = None):
        n = {len(v) for v in columns.values()}
        assert len(n) == 1, "columns must have equal length"
        self.columns = columns
        self.as_tuple = list(as_tuple) if as_tuple else None

    def __len__(self):
        return len(next(iter(self.columns.values())))

    def __getitem__(self, i):
        if self.as_tuple:
            return tuple(self.columns[k][i] for k in self.as_tuple)
        return {k: v[i] for k, v in self.columns.items()}

    def gather(self, idx: torch.Tensor):
        if self.as_tuple:
            return tuple(self.columns[k].index_select(0, idx) for k in self.as_tuple)
        return {k: v.index_select(0, idx) for k, v in self.columns.items()}

    def to(self, device):
        return TensorDictDataset({k: v.to(device) for k, v in self.columns.items()}, self.as_tuple)


def SyntheticCIFAR10(n: int = 50000, seed: int = 0, device=None, num_classes: int = 10,
                     noise: float = 0.6) -> TensorDictDataset:
    g = torch.Generator(device="cpu").manual_seed(seed)
    labels = torch.randint(0, num_classes, (n,), generator=g)
    patterns = torch.rand(num_classes, 3, 4, 4, generator=g) * 2 - 1
    base = torch.nn.functional.interpolate(patterns, size=(32, 32), mode="bilinear", align_corners=False)
    imgs = torch.empty(n, 3, 32, 32)
    chunk = 8192
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        x = base[labels[s:e]] * (1 - noise) + (torch.rand(e - s, 3, 32, 32, generator=g) * 2 - 1) * noise
        imgs[s:e] = x.clamp_(-1, 1)
    ds = TensorDictDataset({"data": imgs, "target": labels}, as_tuple=("data", "target"))
    return ds.to(device) if device is not None else ds


def SyntheticIMDb(n: int = 25000, seq_len: int = 512, vocab: int = 30522, seed: int = 0, device=None,
                  min_len: int = 64) -> TensorDictDataset:
    g = torch.Generator(device="cpu").manual_seed(seed)
    labels = torch.randint(0, 2, (n,), generator=g)
    min_len = max(2, min(min_len, seq_len // 2))
    lengths = torch.randint(min_len, seq_len + 1, (n,), generator=g)
    ids = torch.randint(1000, vocab, (n, seq_len), generator=g)
    # label-dependent "sentiment" tokens sprinkled through each review
    pos_tok = torch.arange(2000, 2050)
    neg_tok = torch.arange(3000, 3050)
    sprinkle = torch.rand(n, seq_len, generator=g) < 0.08
    choice = torch.randint(0, 50, (n, seq_len), generator=g)
    senti = torch.where(labels[:, None].bool(), pos_tok[choice], neg_tok[choice])
    ids = torch.where(sprinkle, senti, ids)
    ids[:, 0] = 101  # [CLS]
    ar = torch.arange(seq_len)[None, :]
    mask = (ar < lengths[:, None]).long()
    ids = torch.where(mask.bool(), ids, torch.zeros_like(ids))  # [PAD] = 0
    ids[torch.arange(n), lengths - 1] = 102  # [SEP]
    ds = TensorDictDataset({"input_ids": ids, "attention_mask": mask, "labels": labels})
    return ds.to(device) if device is not None else ds


def train_val_split(ds: TensorDictDataset, test_size: float = 0.2, seed: int = 42):
    """Fixed-seed split (the reference's ``train_test_split(test_size=.2)``, made rank-identical)."""
    n = len(ds)
    g = torch.Generator(device="cpu").manual_seed(seed)
    perm = torch.randperm(n, generator=g)
    n_test = int(math.ceil(test_size * n))
    test_idx, train_idx = perm[:n_test], perm[n_test:]
    cols_tr = {k: v.index_select(0, train_idx.to(v.device)) for k, v in ds.columns.items()}
    cols_te = {k: v.index_select(0, test_idx.to(v.device)) for k, v in ds.columns.items()}
    return TensorDictDataset(cols_tr, ds.as_tuple), TensorDictDataset(cols_te, ds.as_tuple)


class DeviceLoader:
    """``DataLoader(partition, batch_size, shuffle)`` with on-device shuffling and gathers.

    ``source`` is a :class:`Partition` over a :class:`TensorDictDataset` (or the dataset
    itself).  Each epoch draws a permutation of the shard from a seeded generator.
    """

    def __init__(self, source: Union[Partition, TensorDictDataset], batch_size: int, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False, device=None):
        if isinstance(source, Partition):
            self.ds = source.data
            self.index = source.index_tensor()
        else:
            self.ds = source
            self.index = torch.arange(len(source))
        first = next(iter(self.ds.columns.values()))
        self.device = torch.device(device) if device is not None else first.device
        if first.device != self.device:
            self.ds = self.ds.to(self.device)
        self.index = self.index.to(self.device)
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        self.dataset = source  # DataLoader-compatible attribute (len(loader.dataset))

    def __len__(self):
        n = len(self.index)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def __iter__(self) -> Iterator:
        n = len(self.index)
        if self.shuffle:
            g = torch.Generator(device="cpu").manual_seed(self.seed * 100003 + self.epoch)
            order = self.index[torch.randperm(n, generator=g).to(self.device)]
        else:
            order = self.index
        self.epoch += 1
        for s in range(0, n, self.batch_size):
            e = s + self.batch_size
            if e > n and self.drop_last:
                break
            yield self.ds.gather(order[s:e])
