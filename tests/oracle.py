"""Test-only semantic oracle for PowerSGD, written from SURVEY.md §2.9 (fp64, per tensor).

Independent of the framework code: used as the golden model for the HIP kernels and for
the end-to-end reducer / fused optimizer.
"""
from __future__ import annotations

from typing import List, Sequence

import torch


def mgs(P: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    P = P.clone()
    for i in range(P.shape[1]):
        P[:, i] = P[:, i] / (torch.sqrt(torch.sum(P[:, i] ** 2)) + eps)
        if i + 1 < P.shape[1]:
            d = (P[:, i: i + 1] * P[:, i + 1:]).sum(0)
            P[:, i + 1:] -= d[None, :] * P[:, i: i + 1]
    return P


def powersgd_round(Ms_per_rank: Sequence[Sequence[torch.Tensor]], Qs: Sequence[torch.Tensor], R: int,
                   eps: float = 1e-8):
    """One reduce() call across N simulated ranks.

    Ms_per_rank[k][i] is rank k's send buffer for tensor i (any shape).
    Qs[i] is the (rank-identical) query of the i-th >1-D tensor.
    Returns (outs, mems_per_rank, new_Qs): outs identical on all ranks.
    """
    N = len(Ms_per_rank)
    T = len(Ms_per_rank[0])
    outs: List[torch.Tensor] = [None] * T
    mems = [[None] * T for _ in range(N)]
    newQ = []
    hi = [i for i in range(T) if Ms_per_rank[0][i].dim() > 1]
    qi = 0
    for i in range(T):
        shape = Ms_per_rank[0][i].shape
        if Ms_per_rank[0][i].dim() <= 1:
            outs[i] = sum(Ms_per_rank[k][i].double() for k in range(N)) / N
            for k in range(N):
                mems[k][i] = None  # never written (stays at its old value)
            continue
        A = [Ms_per_rank[k][i].double().reshape(shape[0], -1) for k in range(N)]
        Q = Qs[qi].double()
        P = sum(a @ Q for a in A) / N
        P = mgs(P, eps)
        Qn = sum(a.t() @ P for a in A) / N
        out = P @ Qn.t()
        outs[i] = out.reshape(shape)
        for k in range(N):
            mems[k][i] = (A[k] - out).reshape(shape)
        newQ.append(Qn)
        qi += 1
    assert qi == len(hi)
    return outs, mems, newQ


def reference_bits(shapes: Sequence[torch.Size], R: int) -> int:
    p = q = r1 = 0
    for s in shapes:
        if len(s) <= 1:
            r1 += int(torch.Size(s).numel())
            continue
        n = s[0]
        m = int(torch.Size(s).numel()) // n
        r = min(n, m, R)
        p += n * r
        q += m * r
    return 32 * (p + q + r1)
