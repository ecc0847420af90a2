"""PowerSGD low-rank gradient compression with error feedback (Vogels et al., Alg. 1 + 2).

Two front-ends share one native execution plan:

* :class:`PowerSGDReducer` — API-compatible with the reference
  (ddp_powersgd_guide_cifar10/reducer.py:25-170):
  ``PowerSGDReducer(random_seed, device, n_power_iterations=0, reuse_query=True, rank=1)``
  and ``reduce(grad_in, grad_out, memory_out) -> bits``.
* :class:`PowerSGDOptimizer` — the reference training loop's whole "Algorithm 2" step
  (EF pack ``g + e``, compression, decompression, error memory, momentum, SGD update;
  ddp_powersgd_guide_cifar10/ddp_init.py:149-178) fused over flat parameter / gradient /
  error / momentum arenas: 6 kernel launches + 2 collectives per step instead of the
  reference's ~1.3k eager ops (SURVEY.md §2.6 launch-count evidence).

Per-step device pipeline (one launch each, all matrices at once):
  psgd_p  (P = (g+e) Q, e <- g+e)  ->  seg_reduce (split-K sum of P | pack rank-1 grads)
  -> all_reduce([P | rank-1])      ->  psgd_orth (/N + batched MGS)
  -> psgd_q (Q = M^T P)            ->  seg_reduce (split-K sum of Q)
  -> all_reduce(Q)                 ->  psgd_update (out = P Q^T/N, e = M - out, momentum,
                                       x -= lr (out + m), warm-start Q)  + rank1_step
The P and rank-1 payloads share ONE collective (the reference issues them separately,
reducer.py:126,132); the byte count per step is unchanged.

Deliberate deviations: Q1 the Q-init RNG is a private generator seeded
exactly like the reference (``torch.manual_seed(rng.randint(1e9))`` per matrix) so the
values match but the global RNG is untouched; Q5 the unused 512 MiB ``precalc_numbers``
is not allocated (``rng_compat=True`` still advances the numpy stream the same way so Q
matches the reference bit-for-bit); Q6 models without <=1-D parameters are fine;
Q8 decompression writes parameter-shaped output directly.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import SegPlan, capturing, ext, gradfinish, upload, upload_epoch
from .comm import Communicator, n_bits
from ..knobs import fusion_on

__all__ = [
    "plan_layout",
    "Reducer",
    "PowerSGDReducer",
    "PowerSGDOptimizer",
    "orthogonalize",
    "powersgd_bytes_per_step",
]

_ALIGN = 16  # floats (64 B) — every high-rank arena slot starts 16-B aligned for float4


def plan_layout(shapes: Sequence[Tuple[int, int]], rank: int):
    """Pure-python P/Q layout (reference order, reducer.py:72-98)."""
    ranks, p_offs, q_offs = [], [], []
    p = q = 0
    for n, m in shapes:
        r = min(n, m, rank)
        ranks.append(r)
        p_offs.append(p)
        q_offs.append(q)
        p += n * r
        q += m * r
    return ranks, p_offs, q_offs, p, q


def powersgd_bytes_per_step(params: Sequence[torch.Tensor], rank: int) -> Dict[str, int]:
    """Bytes all-reduced per step with the reference's accounting."""
    shapes = [(p.shape[0], p.numel() // p.shape[0]) for p in params if p.dim() > 1]
    r1 = sum(p.numel() for p in params if p.dim() <= 1)
    _, _, _, pt, qt = plan_layout(shapes, rank)
    dense = sum(p.numel() for p in params)
    return {"p": 4 * pt, "rank1": 4 * r1, "q": 4 * qt, "total": 4 * (pt + r1 + qt), "dense": 4 * dense}


def orthogonalize(matrix: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    """In-place modified Gram-Schmidt on the columns of ``matrix`` (reducer.py:180-191).

    Device tensors run the batched gfx950 kernel; CPU tensors use torch ops.
    """
    n, m = matrix.shape
    if matrix.is_cuda:
        assert matrix.dtype == torch.float32 and matrix.is_contiguous()
        X = ext()
        geom, items, n_items, max_rank = X.make_orth_geom([(int(n), int(m), 0)])
        scratch = torch.empty(2 * n_items * X.MAX_RANK, dtype=torch.float32, device=matrix.device)
        ctr = torch.zeros(2, dtype=torch.int64, device=matrix.device)
        X.psgd_orth(geom.to(matrix.device), items.to(matrix.device), matrix.view(-1), 1.0, float(eps),
                    int(max_rank), scratch, ctr)
        return matrix
    for i in range(m):
        col = matrix[:, i: i + 1]
        col /= torch.sqrt(torch.sum(col ** 2)) + eps
        if i + 1 < m:
            rest = matrix[:, i + 1:]
            rest -= torch.sum(col * rest, dim=0) * col
    return matrix


class Reducer:
    """Base reducer (reducer.py:6-23): rng, world size, device.

    ``rng_compat=True`` advances the numpy stream past the reference's 128M-sample
    ``precalc_numbers`` draw (without keeping it on the device, quirk Q5) so the Q-init
    seeds equal the reference's.
    """

    def __init__(self, random_seed: int, device, comm: Optional[Communicator] = None,
                 rng_compat: bool = False):
        self.rng = np.random.RandomState(random_seed)
        if rng_compat:
            left = 128 * 1024 * 1024
            while left > 0:
                k = min(left, 1 << 22)
                self.rng.randn(k)
                left -= k
        self.comm = comm if comm is not None else Communicator()
        self.n_workers = self.comm.world_size
        self.worker_rank = self.comm.rank  # quirk Q7: `rank` below means compression rank
        self.device = torch.device(device)

    def reduce(self, grad_in, grad_out, memory_out):
        """Return communicated bits."""
        raise NotImplementedError()


class _PlanBuffers:
    """Device/host buffers + native tables for one list of matrix shapes."""

    def __init__(self, shapes: List[Tuple[int, int]], rank: int, r1_numel: int, device: torch.device,
                 native: bool = True):
        self.shapes = shapes
        self.rank = rank
        self.device = device
        self.ranks, self.p_offs, self.q_offs, self.p_total, self.q_total = plan_layout(shapes, rank)
        self.r1_numel = r1_numel
        self.max_rank = max(self.ranks) if self.ranks else 1
        f32 = dict(dtype=torch.float32, device=device)
        # comm buffer: [ P (sum n_i r_i) | rank-1 group ] -> ONE all-reduce
        self.comm_buf = torch.zeros(self.p_total + r1_numel, **f32)
        self.p_memory = self.comm_buf[: self.p_total]
        self.rank1_buf = self.comm_buf[self.p_total:]
        self.q_memory = torch.zeros(self.q_total, **f32)   # all-reduce payload for Q
        self.q_warm = torch.zeros(self.q_total, **f32)     # averaged Q = next step's query
        self.native = native and device.type == "cuda"
        if self.native:
            X = ext()
            d = X.build_plan([(int(n), int(m)) for n, m in shapes], int(rank))
            assert d["p_total"] == self.p_total and d["q_total"] == self.q_total
            self._geom_host = d["geom"]
            self.p_items = d["p_items"].to(device)
            self.q_items = d["q_items"].to(device)
            self.u_items = d["u_items"].to(device)
            self.p_part = torch.zeros(max(1, d["pp_total"]), **f32)
            self.q_part = torch.zeros(max(1, d["qp_total"]), **f32)
            self.pp_offs, self.qp_offs = d["pp_offs"], d["qp_offs"]
            self.p_chunks, self.q_chunks = d["p_chunks"], d["q_chunks"]
            self.counts = {k: d[k] for k in ("n_p_items", "n_q_items", "n_u_items", "n_orth_items", "pp_total",
                                             "qp_total")}
            self.item_start = {k: d[k + "_item_start"] for k in ("p", "q", "u", "orth")}
            self.orth_items = d["orth_items"].to(device)
            self.orth_scratch = torch.zeros(max(1, 2 * d["n_orth_items"] * X.MAX_RANK), **f32)
            # 64-bit MGS barrier counters (never wrap) + the error word (low half of the last)
            self.orth_ctr = torch.zeros(len(shapes) + 1, dtype=torch.int64, device=device)
            nb = max(1, len(shapes)) * X.SIZEOF_MATGEOM
            self.geom = torch.zeros(nb, dtype=torch.uint8, device=device)
            self.ptrs = torch.zeros(nb, dtype=torch.uint8, device=device)
            self._bind_key = None
            self.q_seg = SegPlan(self.q_seg_specs(0, len(shapes)), device)
            # in-kernel split-K finish of P / Q (csrc/powersgd.hip PFin / QFin): monotonic arrival
            # counters, one per P row block / Q column block (zeroed once, never reset)
            self.p_cols = int(d["p_cols"])  # columns per P item
            self.p_ctr = torch.zeros(max(1, d["n_p_blocks"]), dtype=torch.int64, device=device)
            self.q_ctr = torch.zeros(max(1, d["n_q_blocks"]), dtype=torch.int64, device=device)
            self._q_seg_fused = SegPlan(self.q_seg_specs(0, len(shapes), fused=True), device)
            self.fused = self.max_rank <= _LAZY_MAX_RANK and fusion_on("psgd_fin")

    # -- per-matrix-range views (a PowerSGD overlap group = matrices [lo, hi)) ----------------
    def p_seg_specs(self, lo: int = 0, hi: Optional[int] = None):
        hi = len(self.shapes) if hi is None else hi
        return [(self.p_part[self.pp_offs[i]:], self.p_memory[self.p_offs[i]: self.p_offs[i] + n * r],
                 self.p_chunks[i], n * r, 1.0)
                for i, ((n, m), r) in enumerate(zip(self.shapes, self.ranks)) if lo <= i < hi]

    def q_seg_specs(self, lo: int, hi: int, fused: bool = False):
        """Split-K sums of Q for matrices [lo, hi); ``fused``: only those the Q kernel does not
        finish itself (more than ``Q_FIN_MAX`` row chunks)."""
        return [(self.q_part[self.qp_offs[i]:], self.q_memory[self.q_offs[i]: self.q_offs[i] + m * r],
                 self.q_chunks[i], m * r, 1.0)
                for i, ((n, m), r) in enumerate(zip(self.shapes, self.ranks))
                if lo <= i < hi and (not fused or self.q_chunks[i] > Q_FIN_MAX)]

    def items(self, kind: str, lo: int, hi: int) -> torch.Tensor:
        """Byte slice of a work-item table covering matrices [lo, hi)."""
        size = {"p": 32, "q": 32, "u": 16, "orth": 32}[kind]  # sizeof PItem / QItem / UItem / OrthItem
        table = {"p": self.p_items, "q": self.q_items, "u": self.u_items, "orth": self.orth_items}[kind]
        st = self.item_start[kind]
        return table[st[lo] * size: st[hi] * size]

    def p_range(self, lo: int, hi: int) -> Tuple[int, int]:
        end = self.p_offs[hi - 1] + self.shapes[hi - 1][0] * self.ranks[hi - 1]
        return self.p_offs[lo], end

    def q_range(self, lo: int, hi: int) -> Tuple[int, int]:
        end = self.q_offs[hi - 1] + self.shapes[hi - 1][1] * self.ranks[hi - 1]
        return self.q_offs[lo], end

    def run_p(self, items: torch.Tensor, fuse_ef: bool, p_prev: Optional[torch.Tensor] = None,
              seg: Optional[SegPlan] = None, p_seg: Optional[SegPlan] = None):
        """P = M Q for the matrices of ``items`` (+ the rank-1 pack ``seg``): one launch when the
        split-K sums run in-kernel (``fused``), else the kernel + ``p_seg`` (sums and pack)."""
        X = ext()
        if not self.fused:
            if self.shapes:
                X.psgd_p(self.geom, self.ptrs, items, self.q_warm, self.p_part, fuse_ef, self.max_rank, p_prev,
                         p_cols=self.p_cols)
            if p_seg is not None:
                p_seg.run()
            return
        t = seg.table() if seg is not None else None
        if not self.shapes and t is None:
            return
        kw = dict(seg_entries=t[0], seg_prefix=t[1], seg_n=t[2], seg_blocks=t[3]) if t is not None else {}
        X.psgd_p(self.geom, self.ptrs, items, self.q_warm, self.p_part, fuse_ef, self.max_rank, p_prev,
                 p_out=self.comm_buf, p_ctr=self.p_ctr, p_cols=self.p_cols, **kw)

    def run_q(self, items: torch.Tensor, q_seg: SegPlan, q_seg_fused: Optional[SegPlan] = None):
        """Q = M^T P-hat into q_memory: split-K sums in-kernel when ``fused`` (+ ``q_seg_fused`` for
        the matrices with more than Q_FIN_MAX row chunks), else + ``q_seg``."""
        X = ext()
        if self.fused:
            X.psgd_q(self.geom, self.ptrs, items, self.comm_buf, self.q_part, self.max_rank,
                     q_out=self.q_memory, q_ctr=self.q_ctr, q_fin_max=Q_FIN_MAX)
            (self._q_seg_fused if q_seg_fused is None else q_seg_fused).run()
        else:
            X.psgd_q(self.geom, self.ptrs, items, self.comm_buf, self.q_part, self.max_rank)
            q_seg.run()

    def orth(self, p_div: float, eps: float, items: Optional[torch.Tensor] = None, max_spins: int = -1):
        """P-hat = MGS(P / p_div) for every matrix (or a group's item slice), one launch."""
        ext().psgd_orth(self.geom, self.orth_items if items is None else items, self.comm_buf, p_div, eps,
                        self.max_rank, self.orth_scratch, self.orth_ctr, self.counts["n_orth_items"], max_spins)

    def orth_error(self) -> int:
        """Non-zero if a cross-workgroup barrier of the MGS kernel ever timed out (host sync)."""
        return int(self.orth_ctr[-1].item())

    def check_orth(self):
        if self.native and self.orth_error():
            raise RuntimeError("PowerSGD orthogonalisation: a cross-workgroup barrier timed out; P-hat "
                               "was poisoned with NaN (co-residency violated)")

    def bind(self, rows: List[List[int]], vec: List[int]) -> bool:
        """Point the grouped kernels at new tensors; returns True if the tables changed."""
        key = (upload_epoch(), tuple(map(tuple, rows)), tuple(vec))
        if key == self._bind_key:
            return False
        X = ext()
        upload(self.geom, X.patch_geom_vec(self._geom_host, vec))
        upload(self.ptrs, X.make_mat_ptrs(rows))
        self._bind_key = key
        return True

    def bind_range(self, lo: int, rows: List[List[int]], vec: List[int]):
        """Upload geometry + pointer rows of matrices [lo, lo + len(rows)) only."""
        X = ext()
        sz = X.SIZEOF_MATGEOM
        hi = lo + len(rows)
        geom = self._geom_host[lo * sz: hi * sz].clone()
        gi = geom.view(torch.int32).view(hi - lo, sz // 4)
        gi[:, 3] = torch.tensor(vec, dtype=torch.int32)  # MatGeom.vec
        upload(self.geom[lo * sz: hi * sz], geom)
        upload(self.ptrs[lo * X.SIZEOF_MATPTRS: hi * X.SIZEOF_MATPTRS], X.make_mat_ptrs(rows))

    def p_view(self, i):
        n, _ = self.shapes[i]
        return self.p_memory[self.p_offs[i]: self.p_offs[i] + n * self.ranks[i]].view(n, self.ranks[i])

    def q_view(self, i, buf=None):
        _, m = self.shapes[i]
        buf = self.q_warm if buf is None else buf
        return buf[self.q_offs[i]: self.q_offs[i] + m * self.ranks[i]].view(m, self.ranks[i])


def _vec_ok(m: int, ptrs: Sequence[int]) -> int:
    return int(m % 4 == 0 and all(p % 16 == 0 for p in ptrs if p))


class PowerSGDReducer(Reducer):
    """Rank-r PowerSGD with warm-started Q and error feedback (reducer.py:25-170)."""

    def __init__(self, random_seed, device, n_power_iterations=0, reuse_query=True, rank=1,
                 comm: Optional[Communicator] = None, rng_compat: bool = False, eps: float = 1e-8):
        super().__init__(random_seed, device, comm=comm, rng_compat=rng_compat)
        assert n_power_iterations == 0
        self.rank = rank
        self.reuse_query = reuse_query
        self.eps = eps
        self._buf: Optional[_PlanBuffers] = None
        self.p_memory = None
        self.q_memory = None
        self._bind_key = None
        self._p_seg = None
        self._r1_unpack = None

    def _set_random(self, q: torch.Tensor):
        # reducer.py:36-38 with a private generator (quirk Q1): same seed stream, same values
        seed = int(self.rng.randint(1_000_000_000))
        gen = torch.Generator(device=q.device)
        gen.manual_seed(seed)
        q.copy_(torch.randn(*q.shape, generator=gen, device=q.device, dtype=q.dtype))

    def _init_queries(self, first: bool):
        if self.reuse_query and not first:
            return
        for i in range(len(self._buf.shapes)):
            self._set_random(self._buf.q_view(i))

    # ------------------------------------------------------------------------------------
    def reduce_torch(self, grad_in, grad_out, memory_out):
        """Eager-PyTorch reference-semantics path on any device (comparison arm)."""
        return self.reduce(grad_in, grad_out, memory_out, force_torch=True)

    def reduce(self, grad_in, grad_out, memory_out, force_torch: bool = False):
        rank1 = [(t, o, m) for t, o, m in zip(grad_in, grad_out, memory_out) if t.ndimension() <= 1]
        high = [(t, o, m) for t, o, m in zip(grad_in, grad_out, memory_out) if t.ndimension() > 1]
        first = self._buf is None
        if first:  # sized once, on the first call (quirk Q9 kept)
            shapes = [(t.shape[0], t.numel() // t.shape[0]) for t, _, _ in high]
            self._buf = _PlanBuffers(shapes, self.rank, sum(t.numel() for t, _, _ in rank1), self.device,
                                     native=not force_torch)
            self.p_memory = self._buf.p_memory
            self.q_memory = self._buf.q_memory
        B = self._buf
        self._init_queries(first)
        N = self.n_workers
        if B.native and not force_torch:
            assert all(t.is_cuda for t, _, _ in high + rank1), "mixed host/device tensors"
            self._reduce_native(high, rank1, N)
        else:
            self._reduce_torch(high, rank1, N)
        return n_bits(B.p_memory) + n_bits(B.rank1_buf) + n_bits(B.q_memory)

    # -- device path: 6 launches + 2 collectives ------------------------------------------
    def _bind(self, high, rank1):
        B = self._buf
        key = tuple(x.data_ptr() for trip in high + rank1 for x in trip)
        if key == self._bind_key:
            return
        rows, vec = [], []
        for (t, o, m), (n, mm) in zip(high, B.shapes):
            assert t.is_contiguous() and o.is_contiguous() and m.is_contiguous()
            row = [t.data_ptr(), 0, t.data_ptr(), o.data_ptr(), m.data_ptr(), 0, 0, 0]
            rows.append(row)
            vec.append(_vec_ok(mm, row))
        B.bind(rows, vec)
        specs = [] if B.fused else B.p_seg_specs()  # fused: the P launch sums its slabs itself
        off = 0
        for t, _, _ in rank1:
            specs.append((t.reshape(-1), B.rank1_buf[off: off + t.numel()], 1, 0, 1.0))
            off += t.numel()
        off = 0
        unpack = []
        for _, o, _ in rank1:
            unpack.append((B.rank1_buf[off: off + o.numel()], o.view(-1), 1, 0, float(self.n_workers)))
            off += o.numel()
        if self._p_seg is None:
            self._p_seg = SegPlan(specs, B.device)
            self._r1_unpack = SegPlan(unpack, B.device)
        else:
            self._p_seg.set(specs)
            self._r1_unpack.set(unpack)
        self._bind_key = key

    def _reduce_native(self, high, rank1, N):
        B = self._buf
        X = ext()
        self._bind(high, rank1)
        B.run_p(B.p_items, False, seg=self._p_seg, p_seg=self._p_seg)   # P (+ split-K sum) + rank-1 pack
        self.comm.all_reduce(B.comm_buf)                    # reducer.py:126 + :132 fused
        if B.shapes:
            B.orth(float(N), self.eps)
            B.run_q(B.q_items, B.q_seg)
            self.comm.all_reduce(B.q_memory)                # reducer.py:145
            X.psgd_update(B.geom, B.ptrs, B.u_items, B.comm_buf, B.q_memory, float(N),
                          B.q_warm, 0, 0.0, 0.0, B.max_rank)
        self._r1_unpack.run()                               # reducer.py:166-168

    # -- CPU / reference-semantics path --------------------------------------------------
    def _reduce_torch(self, high, rank1, N):
        B = self._buf
        for i, (t, _, _) in enumerate(high):
            torch.matmul(t.view(t.shape[0], -1), B.q_view(i), out=B.p_view(i))
        off = 0
        for t, _, _ in rank1:
            B.rank1_buf[off: off + t.numel()].copy_(t.reshape(-1))
            off += t.numel()
        self.comm.all_reduce(B.comm_buf)
        B.p_memory.div_(N)
        for i in range(len(high)):
            orthogonalize(B.p_view(i), self.eps)
        for i, (t, _, _) in enumerate(high):
            torch.matmul(t.view(t.shape[0], -1).t(), B.p_view(i), out=B.q_view(i, B.q_memory))
        self.comm.all_reduce(B.q_memory)
        B.q_memory.div_(N)
        B.q_warm.copy_(B.q_memory)
        for i, (t, o, m) in enumerate(high):
            out = torch.matmul(B.p_view(i), B.q_view(i).t())
            o.copy_(out.view_as(o))
            m.copy_(t - o)
        off = 0
        for _, o, _ in rank1:
            o.copy_((B.rank1_buf[off: off + o.numel()] / N).view_as(o))
            off += o.numel()


_LAZY_MAX_RANK = 16  # csrc/ndp_kernels.h kUWideMaxRank: the wide P / update kernels
# Q split-K chunks the Q kernel's last arriver sums itself; taller matrices (DistilBERT's 30522-row
# embedding: 120 chunks) keep a seg_reduce launch, which spreads that sum over the whole device
Q_FIN_MAX = int(os.environ.get("NDP_QFIN_MAX", "32"))


class _Group:
    """One overlap group: high-rank matrices [lo, hi) (contiguous in parameter order, so
    their P / Q payloads are contiguous slices of the reference-order buffers)."""

    def __init__(self, idx: int, lo: int, hi: int, params: List[torch.nn.Parameter]):
        self.idx, self.lo, self.hi = idx, lo, hi
        self.params = params
        self.numel = sum(p.numel() for p in params)
        self.ready = 0
        self.launched = False
        self.key = None
        self.p_seg: Optional[SegPlan] = None
        self.q_seg: Optional[SegPlan] = None
        self.q_seg_fused: Optional[SegPlan] = None


class PowerSGDOptimizer:
    """Fused EF-SGD-with-momentum PowerSGD step (ddp_init.py:121-178) over flat arenas.

    Parameters are re-pointed into a flat parameter arena ``x`` (every high-rank slot 64-B
    aligned, the <=1-D group contiguous at the end) with matching error-memory ``e`` and
    momentum ``m`` arenas.  Gradients stay wherever autograd produced them (no in-place
    accumulation into a preset ``.grad`` — that costs one extra add kernel per parameter);
    the grouped kernels reach them through a device pointer table that is re-uploaded only
    when an address changes (hipGraph-capture safe).  ``step()`` returns the bits
    communicated (reducer.py:170).

    **Overlap with backward** (``overlap=True``, the default on a device with a
    stream-ordered data plane — native RCCL, or nothing to communicate).  The high-rank
    matrices are cut, in backward order, into ``groups`` contiguous groups.  A
    post-accumulate-grad hook launches a group's whole pipeline on the communicator's side
    stream as soon as its last gradient lands, in group order on every rank:

        psgd_p -> split-K sum -> all_reduce(P_g) -> MGS -> psgd_q -> split-K sum
               -> all_reduce(Q_g) -> fused decompress / EF / momentum / SGD update

    so compression, both collectives and the update of the late layers run while backward
    is still computing the early layers.  ``step()`` launches what is left (the rank-1
    group: pack, all-reduce, momentum/SGD) and joins the side stream.  Per-matrix work
    items, split-K slab order and the MGS reduction order are exactly those of the serial
    path, so the result is bitwise identical to ``overlap=False`` (tests/test_overlap_gpu.py);
    the byte count is unchanged, the collective count becomes 2 * groups + 1.

    ``write_grad=True`` also leaves ``p.grad = out + m`` exactly like the reference loop
    (ddp_init.py:172); it costs one extra write pass and is off by default.

    **Lazy error feedback** (native, rank <= 16; ``NDP_FUSION_OFF=lazy_ef`` turns it off): the
    update pass does not store ``e = M - P Q^T`` — it would read ``M`` back only for that
    store, 2 of its 6 arena passes.  The arena keeps ``M`` and ``p_prev`` keeps the step's
    P-hat; the next P pass forms ``e`` element by element with the update kernel's exact
    arithmetic (csrc/powersgd.hip), so every step is bitwise the eager formula's.  :attr:`e`
    (and ``state_dict``) materialise the true error memory first.
    """

    def __init__(self, params, lr: float, momentum: float = 0.9, rank: int = 4,
                 random_seed: int = 714, reuse_query: bool = True,
                 comm: Optional[Communicator] = None, write_grad: bool = False,
                 broadcast_params: bool = True, rng_compat: bool = False, eps: float = 1e-8,
                 native: Optional[bool] = None, overlap: Optional[bool] = None, groups: Optional[int] = None):
        self.params: List[torch.nn.Parameter] = [p for p in params]
        assert self.params, "no parameters"
        self.lr = float(lr)
        self.momentum = float(momentum)
        self.rank = int(rank)
        self.reuse_query = reuse_query
        self.write_grad = write_grad
        self.eps = eps
        self.comm = comm if comm is not None else Communicator()
        self.device = self.params[0].device
        self.rng = np.random.RandomState(random_seed)
        if rng_compat:
            left = 128 * 1024 * 1024
            while left > 0:
                k = min(left, 1 << 22)
                self.rng.randn(k)
                left -= k
        self.step_count = 0
        self.bits_communicated = 0
        self._q_ready = False
        self.orth_max_spins = -1  # < 0: kernel default (debug / tests may lower it)

        hi = [p for p in self.params if p.dim() > 1]
        r1 = [p for p in self.params if p.dim() <= 1]
        self.high, self.rank1 = hi, r1
        offs, o = {}, 0
        for p in hi:
            offs[id(p)] = o
            o += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
        self.r1_start = o
        for p in r1:
            offs[id(p)] = o
            o += p.numel()
        self.arena_numel = o
        f32 = dict(dtype=torch.float32, device=self.device)
        self.x = torch.zeros(o, **f32)
        self._e = torch.zeros(o, **f32)
        self.m = torch.zeros(o, **f32)
        self.offsets = offs
        with torch.no_grad():
            for p in self.params:
                s = offs[id(p)]
                view = self.x[s: s + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
                p.grad = None
        if broadcast_params:  # quirks Q3/Q4: replicas start identical (one flat broadcast)
            self.comm.broadcast(self.x, src=0)

        shapes = [(p.shape[0], p.numel() // p.shape[0]) for p in hi]
        self.r1_numel = o - self.r1_start
        self.r1_upd = torch.zeros(self.r1_numel if write_grad else 0, **f32)
        self.buf = _PlanBuffers(shapes, self.rank, self.r1_numel, self.device, native=native is not False)
        self.native = self.buf.native
        # needs the warm-start Q of the next P pass to BE the update's Qs (reuse_query)
        self.lazy_ef = (self.native and bool(shapes) and self.buf.max_rank <= _LAZY_MAX_RANK and reuse_query
                        and fusion_on("lazy_ef"))
        self._lazy_pending = False  # an update ran since e was last materialised
        # P-hat of the last update (lazy error feedback); zero = no pending correction
        self.p_prev = torch.zeros(self.buf.p_total if self.lazy_ef else 0, **f32)
        self._p_seg = SegPlan([], self.device, capacity=len(shapes) + len(r1) + 1) if self.native else None
        self._r1_out = SegPlan([], self.device, capacity=len(r1) + 1) if self.native else None
        self._r1_pack = SegPlan([], self.device, capacity=len(r1) + 1) if self.native else None
        self._grad_key = None
        self._r1_key = None

        # default: overlap when a step has wire time to hide (N > 1 or link emulation)
        want = overlap if overlap is not None else (os.environ.get("NDP_PSGD_OVERLAP", "1") != "0"
                                                    and self.comm.has_traffic)
        self.overlap = bool(want) and self.native and self.comm.stream_ordered and bool(hi)
        if overlap and not self.overlap:
            raise ValueError("overlap=True needs device tensors, the native extension and a stream-ordered "
                             "communicator (native RCCL or world size 1)")
        self.groups: List[_Group] = []
        self._group_of = {}
        self._hooks = []
        self._next_group = 0
        if self.overlap:
            n_groups = groups if groups is not None else int(os.environ.get("NDP_PSGD_GROUPS", "4"))
            self._build_groups(max(1, n_groups))
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    # -- overlap groups ------------------------------------------------------------------------
    def _build_groups(self, n_groups: int):
        """Cut the high-rank matrices, in backward (reverse parameter) order, into groups of
        about total/n_groups elements; the last group to be produced (the first layers) is
        whatever is left, so the exposed post-backward tail stays small."""
        total = sum(p.numel() for p in self.high)
        target = total / n_groups
        bounds = []  # (lo, hi) in forward index space, built from the back
        hi_idx = len(self.high)
        acc = 0
        for i in range(len(self.high) - 1, -1, -1):
            acc += self.high[i].numel()
            if acc >= target and len(bounds) < n_groups - 1 and i > 0:
                bounds.append((i, hi_idx))
                hi_idx, acc = i, 0
        bounds.append((0, hi_idx))
        for gi, (lo, hi) in enumerate(bounds):
            g = _Group(gi, lo, hi, self.high[lo:hi])
            g.p_seg = SegPlan([], self.device, capacity=hi - lo + 1)
            g.q_seg = SegPlan(self.buf.q_seg_specs(lo, hi), self.device)
            if self.buf.native:
                g.q_seg_fused = SegPlan(self.buf.q_seg_specs(lo, hi, fused=True), self.device)
            self.groups.append(g)
            for p in g.params:
                self._group_of[id(p)] = g

    def _on_grad(self, p):
        if not self.overlap:
            return
        g = self._group_of.get(id(p))
        if g is None:
            return  # rank-1 parameters are handled in step()
        g.ready += 1
        # launch in group order on every rank (identical collective sequence everywhere)
        while self._next_group < len(self.groups):
            nxt = self.groups[self._next_group]
            if nxt.launched or nxt.ready < len(nxt.params):
                break
            self._launch_group(nxt)
            self._next_group += 1

    def _bind_group(self, g: _Group):
        B = self.buf
        grads = [p.grad for p in g.params]
        key = (upload_epoch(),) + tuple(t.data_ptr() for t in grads)
        if key == g.key:
            return
        rows, vec = [], []
        for p, gr, (n, m) in zip(g.params, grads, B.shapes[g.lo:g.hi]):
            assert gr.is_contiguous() and gr.dtype == torch.float32, "PowerSGD needs dense fp32 grads"
            s = self.offsets[id(p)]
            e, mo, x = (t[s:].data_ptr() for t in (self._e, self.m, self.x))
            row = [gr.data_ptr(), e, e, 0, 0, mo, x, gr.data_ptr()]
            rows.append(row)
            vec.append(_vec_ok(m, row))
        B.bind_range(g.lo, rows, vec)
        g.p_seg.set(B.p_seg_specs(g.lo, g.hi))
        g.key = key

    @torch.no_grad()
    def _launch_group(self, g: _Group):
        gradfinish.flush()  # deferred conv grad-W sums / folds of the layers done so far
        B = self.buf
        X = ext()
        N = self.comm.world_size
        self._ensure_queries()
        for p in g.params:
            if p.grad is None:  # parameter unused this step: zero gradient
                p.grad = torch.zeros_like(p)
        self._bind_group(g)  # table uploads on the compute stream, before the fork
        p0, p1 = B.p_range(g.lo, g.hi)
        q0, q1 = B.q_range(g.lo, g.hi)
        mode, lr, mom, spins = 2 if self.write_grad else 1, self.lr, self.momentum, self.orth_max_spins

        pp = self.p_prev if self.lazy_ef else None

        def pipeline():
            B.run_p(B.items("p", g.lo, g.hi), True, pp, p_seg=g.p_seg)
            self.comm.all_reduce(B.comm_buf[p0:p1])                       # reducer.py:126 (group g)
            B.orth(float(N), self.eps, B.items("orth", g.lo, g.hi), spins)
            B.run_q(B.items("q", g.lo, g.hi), g.q_seg, g.q_seg_fused)
            self.comm.all_reduce(B.q_memory[q0:q1])                       # reducer.py:145 (group g)
            X.psgd_update(B.geom, B.ptrs, B.items("u", g.lo, g.hi), B.comm_buf, B.q_memory, float(N),
                          B.q_warm, mode, lr, mom, B.max_rank, pp)
        self.comm.side_launch(pipeline)
        g.launched = True

    def _finish_overlapped(self):
        """After backward: launch groups whose hooks did not fire (unused parameters / hooks
        bypassed), run the rank-1 group on the side stream, join."""
        for g in self.groups[self._next_group:]:
            if not g.launched:
                self._launch_group(g)
        self._next_group = len(self.groups)
        B = self.buf
        N = self.comm.world_size
        if self.r1_numel:
            grads = []
            for p in self.rank1:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                grads.append(p.grad)
            key = (upload_epoch(),) + tuple(t.data_ptr() for t in grads)
            if key != self._r1_key:
                specs, outs = [], []
                for p, gr in zip(self.rank1, grads):
                    s = self.offsets[id(p)] - self.r1_start
                    specs.append((gr.view(-1), B.rank1_buf[s: s + p.numel()], 1, 0, 1.0))
                    if self.write_grad:
                        outs.append((self.r1_upd[s: s + p.numel()], gr.view(-1), 1, 0, 1.0))
                self._r1_pack.set(specs)
                self._r1_out.set(outs)
                self._r1_key = key
            r1 = slice(self.r1_start, self.arena_numel)
            lr, mom = self.lr, self.momentum

            def rank1():
                self._r1_pack.run()
                self.comm.all_reduce(B.rank1_buf)                           # reducer.py:132
                ext().rank1_step(B.rank1_buf, float(N), self.m[r1], self.x[r1],
                                 self.r1_upd if self.write_grad else None, lr, mom)
                if self.write_grad:
                    self._r1_out.run()
            self.comm.side_launch(rank1)
        self.comm.side_join()

    # -- helpers -------------------------------------------------------------------------
    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()
        self._reset_groups()

    def _reset_groups(self):
        for g in self.groups:
            g.ready = 0
            g.launched = False
        self._next_group = 0

    def _view(self, t, p):
        s = self.offsets[id(p)]
        return t[s: s + p.numel()]

    def _grads(self):
        gs = []
        for p in self.params:
            if p.grad is None:  # parameter unused this step: zero gradient
                p.grad = torch.zeros_like(p)
            g = p.grad
            assert g.is_contiguous() and g.dtype == torch.float32, "PowerSGD needs dense fp32 grads"
            gs.append(g)
        return gs

    def _bind(self):
        gmap = {id(p): p.grad for p in self.params}
        key = (upload_epoch(),) + tuple(g.data_ptr() for g in gmap.values())
        if key == self._grad_key:
            return
        B = self.buf
        rows, vec = [], []
        for p, (n, m) in zip(self.high, B.shapes):
            s = self.offsets[id(p)]
            g = gmap[id(p)].data_ptr()
            e, mo, x = (t[s:].data_ptr() for t in (self._e, self.m, self.x))
            row = [g, e, e, 0, 0, mo, x, g]
            rows.append(row)
            vec.append(_vec_ok(m, row))
        B.bind(rows, vec)
        pack, outs = [], []
        for p in self.rank1:
            s = self.offsets[id(p)] - self.r1_start
            pack.append((gmap[id(p)].view(-1), B.rank1_buf[s: s + p.numel()], 1, 0, 1.0))
            if self.write_grad:
                outs.append((self.r1_upd[s: s + p.numel()], gmap[id(p)].view(-1), 1, 0, 1.0))
        if B.fused:  # the P launch sums its split-K slabs itself and packs the rank-1 group
            self._r1_pack.set(pack)
        else:
            self._p_seg.set(B.p_seg_specs() + pack)
        self._r1_out.set(outs)
        self._grad_key = key

    def _init_queries(self):
        B = self.buf
        for i in range(len(B.shapes)):
            q = B.q_view(i)
            gen = torch.Generator(device=q.device)
            gen.manual_seed(int(self.rng.randint(1_000_000_000)))
            q.copy_(torch.randn(*q.shape, generator=gen, device=q.device, dtype=q.dtype))

    def _ensure_queries(self):
        """Draw the Q init once (reuse_query=True, reducer.py:101-111) or every step."""
        if self._q_ready:
            return
        assert not capturing(), \
            "run one eager step before capturing; reuse_query=False is not graph-capturable"
        self._init_queries()
        self._q_ready = True

    @property
    def bits_per_step(self) -> int:
        B = self.buf
        return 32 * (B.p_total + B.r1_numel + B.q_total)

    @property
    def collectives_per_step(self) -> int:
        if not self.comm.active:
            return 0
        if self.overlap:
            return 2 * len(self.groups) + (1 if self.r1_numel else 0)
        return 2 if self.buf.shapes else 1

    def collective_payloads(self) -> List[int]:
        """Bytes of every collective of one step, in issue order (link-model input)."""
        B = self.buf
        if self.overlap:
            out = []
            for g in self.groups:
                p0, p1 = B.p_range(g.lo, g.hi)
                q0, q1 = B.q_range(g.lo, g.hi)
                out += [4 * (p1 - p0), 4 * (q1 - q0)]
            if self.r1_numel:
                out.append(4 * self.r1_numel)
            return out
        return [4 * (B.p_total + self.r1_numel)] + ([4 * B.q_total] if B.shapes else [])

    def check_errors(self):
        """Host-synchronising health check (call at a low cadence: epoch / replica check):
        raises on a timed-out MGS barrier or an asynchronous RCCL error."""
        self.buf.check_orth()
        self.comm.check()

    # -- the step --------------------------------------------------------------------------
    # Serial path: step() = phase_p -> comm_p -> phase_q -> comm_q -> phase_update.  The
    # phases are exposed separately so a piecewise hipGraph can capture the compute phases
    # and run the two collectives eagerly in between (utils/graph.py, c10d data plane).
    @torch.no_grad()
    def phase_p(self):
        B = self.buf
        self._ensure_queries()
        self._grads()
        if not self.native:
            return
        self._bind()
        B.run_p(B.p_items, True, self.p_prev if self.lazy_ef else None,   # P (+ split-K sum + rank-1 pack)
                seg=self._r1_pack, p_seg=self._p_seg)

    @torch.no_grad()
    def comm_p(self):
        if self.native:
            self.comm.all_reduce(self.buf.comm_buf)            # [P | rank-1]: one collective

    @torch.no_grad()
    def phase_q(self):
        B = self.buf
        if self.native and B.shapes:
            B.orth(float(self.comm.world_size), self.eps, max_spins=self.orth_max_spins)
            B.run_q(B.q_items, B.q_seg)

    @torch.no_grad()
    def comm_q(self):
        if self.native and self.buf.shapes:
            self.comm.all_reduce(self.buf.q_memory)

    @torch.no_grad()
    def phase_update(self):
        B = self.buf
        N = self.comm.world_size
        if self.native:
            X = ext()
            r1 = slice(self.r1_start, self.arena_numel)
            if B.shapes and B.fused and self.r1_numel:  # the rank-1 step rides in the update launch
                X.psgd_update(B.geom, B.ptrs, B.u_items, B.comm_buf, B.q_memory, float(N), B.q_warm,
                              2 if self.write_grad else 1, self.lr, self.momentum, B.max_rank,
                              self.p_prev if self.lazy_ef else None, r1_buf=B.rank1_buf, r1_div=float(N),
                              r1_mom=self.m[r1], r1_x=self.x[r1], r1_g=self.r1_upd if self.write_grad else None)
                if self.write_grad:
                    self._r1_out.run()
            elif B.shapes:
                X.psgd_update(B.geom, B.ptrs, B.u_items, B.comm_buf, B.q_memory, float(N), B.q_warm,
                              2 if self.write_grad else 1, self.lr, self.momentum, B.max_rank,
                              self.p_prev if self.lazy_ef else None)
            if self.r1_numel and not (B.shapes and B.fused):
                X.rank1_step(B.rank1_buf, float(N), self.m[r1], self.x[r1],
                             self.r1_upd if self.write_grad else None, self.lr, self.momentum)
                if self.write_grad:
                    self._r1_out.run()
        else:
            self._step_torch(N, [p.grad for p in self.params])
        self.count_step()

    def count_step(self):
        """Host-side bookkeeping of one step (graph replays call this explicitly)."""
        if capturing():  # the capture pass is not a real step
            return
        self._lazy_pending = self.lazy_ef
        self.step_count += 1
        self.bits_communicated += self.bits_per_step
        if not self.reuse_query:
            self._q_ready = False

    @torch.no_grad()
    def step(self) -> int:
        if self.overlap:
            self._finish_overlapped()
            self._reset_groups()
            self.count_step()
            return self.bits_per_step
        self.phase_p()
        self.comm_p()
        self.phase_q()
        self.comm_q()
        self.phase_update()
        return self.bits_per_step

    def phases(self):
        """[(fn, is_collective)] in execution order (for piecewise graph capture).  Piecewise
        capture runs the collectives eagerly between segments, so the hooks are disabled."""
        self.set_overlap(False)
        return [(self.phase_p, False), (self.comm_p, True), (self.phase_q, False), (self.comm_q, True),
                (self.phase_update, False)]

    def set_overlap(self, on: bool):
        if on and not self.groups:
            raise ValueError("optimizer was built without overlap groups")
        self.overlap = on
        self._reset_groups()

    def _step_torch(self, N, grads):
        B = self.buf
        lam, lr = self.momentum, self.lr
        gmap = {id(p): g for p, g in zip(self.params, grads)}
        Ms = []
        for i, p in enumerate(self.high):
            n, m = B.shapes[i]
            e = self._view(self._e, p)
            e.add_(gmap[id(p)].reshape(-1))              # M = g + e (stored in e)
            M = e.view(n, m)
            Ms.append(M)
            torch.matmul(M, B.q_view(i), out=B.p_view(i))
        for p in self.rank1:
            s = self.offsets[id(p)] - self.r1_start
            B.rank1_buf[s: s + p.numel()].copy_(gmap[id(p)].reshape(-1))
        self.comm.all_reduce(B.comm_buf)
        B.p_memory.div_(N)
        for i in range(len(self.high)):
            orthogonalize(B.p_view(i), self.eps)
        for i, M in enumerate(Ms):
            torch.matmul(M.t(), B.p_view(i), out=B.q_view(i, B.q_memory))
        self.comm.all_reduce(B.q_memory)
        B.q_memory.div_(N)
        B.q_warm.copy_(B.q_memory)
        for i, (p, M) in enumerate(zip(self.high, Ms)):
            out = torch.matmul(B.p_view(i), B.q_view(i).t()).view(-1)
            self._view(self._e, p).copy_(M.reshape(-1) - out)
            mom = self._view(self.m, p)
            mom.mul_(lam).add_(out)
            upd = out + mom
            self._view(self.x, p).add_(upd, alpha=-lr)
            if self.write_grad:
                gmap[id(p)].copy_(upd.view_as(p))
        if self.r1_numel:
            r1 = slice(self.r1_start, self.arena_numel)
            out = B.rank1_buf / N
            self.m[r1].mul_(lam).add_(out)
            upd = out + self.m[r1]
            self.x[r1].add_(upd, alpha=-lr)
            if self.write_grad:
                for p in self.rank1:
                    s = self.offsets[id(p)] - self.r1_start
                    gmap[id(p)].copy_(upd[s: s + p.numel()].view_as(p))

    # -- lazy error feedback -------------------------------------------------------------------
    @property
    def e(self) -> torch.Tensor:
        """The error-feedback memory (reducer.py ``memories``), materialised: with lazy error
        feedback the arena holds ``M`` and the correction ``- P_prev Qs^T`` is applied here by
        the update kernel's own arithmetic (mode 3), exactly as the next P pass would."""
        self.materialize_error()
        return self._e

    @torch.no_grad()
    def materialize_error(self):
        if not (self.lazy_ef and self._lazy_pending) or capturing():
            return
        B = self.buf
        ext().psgd_update(B.geom, B.ptrs, B.u_items, self.p_prev, B.q_warm, 1.0, None, 3, 0.0, 0.0, B.max_rank)
        self.p_prev.zero_()
        self._lazy_pending = False

    # -- training-state snapshot (graph warm-up must not change training) -------------------
    def prepare(self):
        """Draw the initial queries now (before a graph warm-up snapshot)."""
        with torch.no_grad():
            self._ensure_queries()

    def snapshot(self):
        return {"x": self.x.clone(), "e": self._e.clone(), "p_prev": self.p_prev.clone(),
                "lazy_pending": self._lazy_pending, "m": self.m.clone(), "q": self.buf.q_warm.clone(),
                "step_count": self.step_count, "bits": self.bits_communicated, "q_ready": self._q_ready,
                "rng": self.rng.get_state()}

    def restore(self, snap):
        self.x.copy_(snap["x"])
        self._e.copy_(snap["e"])
        self.p_prev.copy_(snap["p_prev"])
        self._lazy_pending = snap["lazy_pending"]
        self.m.copy_(snap["m"])
        self.buf.q_warm.copy_(snap["q"])
        self.step_count = snap["step_count"]
        self.bits_communicated = snap["bits"]
        self._q_ready = snap["q_ready"]
        self.rng.set_state(snap["rng"])

    # -- checkpoint / resume ---------------------------------------------------------------
    def state_dict(self):
        return {
            "step_count": self.step_count,
            "bits_communicated": self.bits_communicated,
            "error": self.e.detach().cpu().clone(),  # materialised (lazy error feedback)
            "momentum": self.m.detach().cpu().clone(),
            "q_warm": self.buf.q_warm.detach().cpu().clone(),
            "q_ready": self._q_ready,
            "rng_state": _rng_state_to_dict(self.rng.get_state()),
            "lr": self.lr,
            "momentum_coef": self.momentum,
            "rank": self.rank,
        }

    def load_state_dict(self, sd):
        assert sd["rank"] == self.rank, "checkpoint compression rank differs"
        self.step_count = int(sd["step_count"])
        self.bits_communicated = int(sd["bits_communicated"])
        self._e.copy_(sd["error"])
        self.p_prev.zero_()  # e is the true error memory: no pending correction
        self._lazy_pending = False
        self.m.copy_(sd["momentum"])
        self.buf.q_warm.copy_(sd["q_warm"])
        self._q_ready = bool(sd.get("q_ready", self.step_count > 0)) and self.reuse_query
        self.rng.set_state(_rng_state_from_dict(sd["rng_state"]))
        self.lr = float(sd["lr"])
        self.momentum = float(sd["momentum_coef"])


def _rng_state_to_dict(st):
    name, keys, pos, has_gauss, cached = st
    return {"name": name, "keys": torch.from_numpy(np.asarray(keys, dtype=np.int64)), "pos": int(pos),
            "has_gauss": int(has_gauss), "cached": float(cached)}


def _rng_state_from_dict(d):
    return (d["name"], d["keys"].numpy().astype(np.uint32), d["pos"], d["has_gauss"], d["cached"])
