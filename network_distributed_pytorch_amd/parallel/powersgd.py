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
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import SegPlan, capturing, ext, upload
from .comm import Communicator, n_bits

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
        ctr = torch.zeros(2, dtype=torch.int32, device=matrix.device)
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
            self.orth_items = d["orth_items"].to(device)
            self.orth_scratch = torch.zeros(max(1, 2 * d["n_orth_items"] * X.MAX_RANK), **f32)
            self.orth_ctr = torch.zeros(len(shapes) + 1, dtype=torch.int32, device=device)
            nb = max(1, len(shapes)) * X.SIZEOF_MATGEOM
            self.geom = torch.zeros(nb, dtype=torch.uint8, device=device)
            self.ptrs = torch.zeros(nb, dtype=torch.uint8, device=device)
            self._bind_key = None
            self.q_seg = SegPlan(
                [(self.q_part[o:], self.q_memory[qo: qo + m * r], c, m * r, 1.0)
                 for (n, m), r, o, qo, c in zip(shapes, self.ranks, self.qp_offs, self.q_offs, self.q_chunks)],
                device)

    def p_seg_specs(self):
        return [(self.p_part[o:], self.p_memory[po: po + n * r], c, n * r, 1.0)
                for (n, m), r, o, po, c in zip(self.shapes, self.ranks, self.pp_offs, self.p_offs, self.p_chunks)]

    def orth(self, p_div: float, eps: float):
        """P-hat = MGS(P / p_div) for every matrix, one multi-workgroup launch."""
        ext().psgd_orth(self.geom, self.orth_items, self.comm_buf, p_div, eps, self.max_rank,
                        self.orth_scratch, self.orth_ctr)

    def orth_error(self) -> int:
        """Non-zero if a cross-workgroup barrier of the MGS kernel ever timed out."""
        return int(self.orth_ctr[-1].item())

    def bind(self, rows: List[List[int]], vec: List[int]) -> bool:
        """Point the grouped kernels at new tensors; returns True if the tables changed."""
        key = (tuple(map(tuple, rows)), tuple(vec))
        if key == self._bind_key:
            return False
        X = ext()
        upload(self.geom, X.patch_geom_vec(self._geom_host, vec))
        upload(self.ptrs, X.make_mat_ptrs(rows))
        self._bind_key = key
        return True

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
        specs = B.p_seg_specs()
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
        if B.shapes:
            X.psgd_p(B.geom, B.ptrs, B.p_items, B.q_warm, B.p_part, False, B.max_rank)
        self._p_seg.run()                                   # P split-K sum + rank-1 pack
        self.comm.all_reduce(B.comm_buf)                    # reducer.py:126 + :132 fused
        if B.shapes:
            B.orth(float(N), self.eps)
            X.psgd_q(B.geom, B.ptrs, B.q_items, B.comm_buf, B.q_part, B.max_rank)
            B.q_seg.run()
            self.comm.all_reduce(B.q_memory)                # reducer.py:145
            X.psgd_update(B.geom, B.ptrs, B.u_items, B.comm_buf, B.q_memory, float(N),
                          B.q_warm, 0, 0.0, 0.0)
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


class PowerSGDOptimizer:
    """Fused EF-SGD-with-momentum PowerSGD step (ddp_init.py:121-178) over flat arenas.

    Parameters are re-pointed into a flat parameter arena ``x`` (every high-rank slot 64-B
    aligned, the <=1-D group contiguous at the end) with matching error-memory ``e`` and
    momentum ``m`` arenas.  Gradients stay wherever autograd produced them (no in-place
    accumulation into a preset ``.grad`` — that costs one extra add kernel per parameter);
    the grouped kernels reach them through a device pointer table that is re-uploaded only
    when an address changes (hipGraph-capture safe).  ``step()`` returns the bits
    communicated (reducer.py:170).

    ``write_grad=True`` also leaves ``p.grad = out + m`` exactly like the reference loop
    (ddp_init.py:172); it costs one extra write pass and is off by default.
    """

    def __init__(self, params, lr: float, momentum: float = 0.9, rank: int = 4,
                 random_seed: int = 714, reuse_query: bool = True,
                 comm: Optional[Communicator] = None, write_grad: bool = False,
                 broadcast_params: bool = True, rng_compat: bool = False, eps: float = 1e-8,
                 native: Optional[bool] = None):
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
        self.e = torch.zeros(o, **f32)
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
        self._p_seg = SegPlan([], self.device, capacity=len(shapes) + len(r1) + 1) if self.native else None
        self._r1_out = SegPlan([], self.device, capacity=len(r1) + 1) if self.native else None
        self._grad_key = None

    # -- helpers -------------------------------------------------------------------------
    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

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
        key = tuple(g.data_ptr() for g in gmap.values())
        if key == self._grad_key:
            return
        B = self.buf
        rows, vec = [], []
        for p, (n, m) in zip(self.high, B.shapes):
            s = self.offsets[id(p)]
            g = gmap[id(p)].data_ptr()
            e, mo, x = (t[s:].data_ptr() for t in (self.e, self.m, self.x))
            row = [g, e, e, 0, 0, mo, x, g]
            rows.append(row)
            vec.append(_vec_ok(m, row))
        B.bind(rows, vec)
        specs = B.p_seg_specs()
        outs = []
        for p in self.rank1:
            s = self.offsets[id(p)] - self.r1_start
            specs.append((gmap[id(p)].view(-1), B.rank1_buf[s: s + p.numel()], 1, 0, 1.0))
            if self.write_grad:
                outs.append((self.r1_upd[s: s + p.numel()], gmap[id(p)].view(-1), 1, 0, 1.0))
        self._p_seg.set(specs)
        self._r1_out.set(outs)
        self._grad_key = key

    def _init_queries(self):
        B = self.buf
        for i in range(len(B.shapes)):
            q = B.q_view(i)
            gen = torch.Generator(device=q.device)
            gen.manual_seed(int(self.rng.randint(1_000_000_000)))
            q.copy_(torch.randn(*q.shape, generator=gen, device=q.device, dtype=q.dtype))

    @property
    def bits_per_step(self) -> int:
        B = self.buf
        return 32 * (B.p_total + B.r1_numel + B.q_total)

    # -- the step --------------------------------------------------------------------------
    # step() = phase_p -> comm_p -> phase_q -> comm_q -> phase_update.  The phases are
    # exposed separately so a piecewise hipGraph can capture the compute phases and run
    # the two collectives eagerly in between (utils/graph.py).
    @torch.no_grad()
    def phase_p(self):
        B = self.buf
        if self.step_count == 0 or not self.reuse_query:
            assert not capturing(), \
                "run one eager step before capturing; reuse_query=False is not graph-capturable"
            self._init_queries()
        self._grads()
        if not self.native:
            return
        self._bind()
        if B.shapes:
            ext().psgd_p(B.geom, B.ptrs, B.p_items, B.q_warm, B.p_part, True, B.max_rank)
        self._p_seg.run()                                      # P split-K sum + rank-1 pack

    @torch.no_grad()
    def comm_p(self):
        if self.native:
            self.comm.all_reduce(self.buf.comm_buf)            # [P | rank-1]: one collective

    @torch.no_grad()
    def phase_q(self):
        B = self.buf
        if self.native and B.shapes:
            X = ext()
            B.orth(float(self.comm.world_size), self.eps)
            X.psgd_q(B.geom, B.ptrs, B.q_items, B.comm_buf, B.q_part, B.max_rank)
            B.q_seg.run()

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
            if B.shapes:
                X.psgd_update(B.geom, B.ptrs, B.u_items, B.comm_buf, B.q_memory, float(N), B.q_warm,
                              2 if self.write_grad else 1, self.lr, self.momentum)
            if self.r1_numel:
                r1 = slice(self.r1_start, self.arena_numel)
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
        self.step_count += 1
        self.bits_communicated += self.bits_per_step

    def step(self) -> int:
        self.phase_p()
        self.comm_p()
        self.phase_q()
        self.comm_q()
        self.phase_update()
        return self.bits_per_step

    def phases(self):
        """[(fn, is_collective)] in execution order (for piecewise graph capture)."""
        return [(self.phase_p, False), (self.comm_p, True), (self.phase_q, False), (self.comm_q, True),
                (self.phase_update, False)]

    def _step_torch(self, N, grads):
        B = self.buf
        lam, lr = self.momentum, self.lr
        gmap = {id(p): g for p, g in zip(self.params, grads)}
        Ms = []
        for i, p in enumerate(self.high):
            n, m = B.shapes[i]
            e = self._view(self.e, p)
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
            self._view(self.e, p).copy_(M.reshape(-1) - out)
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

    # -- checkpoint / resume ---------------------------------------------------------------
    def state_dict(self):
        return {
            "step_count": self.step_count,
            "bits_communicated": self.bits_communicated,
            "error": self.e.detach().cpu().clone(),
            "momentum": self.m.detach().cpu().clone(),
            "q_warm": self.buf.q_warm.detach().cpu().clone(),
            "rng_state": _rng_state_to_dict(self.rng.get_state()),
            "lr": self.lr,
            "momentum_coef": self.momentum,
            "rank": self.rank,
        }

    def load_state_dict(self, sd):
        assert sd["rank"] == self.rank, "checkpoint compression rank differs"
        self.step_count = int(sd["step_count"])
        self.bits_communicated = int(sd["bits_communicated"])
        self.e.copy_(sd["error"])
        self.m.copy_(sd["momentum"])
        self.buf.q_warm.copy_(sd["q_warm"])
        self.rng.set_state(_rng_state_from_dict(sd["rng_state"]))
        self.lr = float(sd["lr"])
        self.momentum = float(sd["momentum_coef"])


def _rng_state_to_dict(st):
    name, keys, pos, has_gauss, cached = st
    return {"name": name, "keys": torch.from_numpy(np.asarray(keys, dtype=np.int64)), "pos": int(pos),
            "has_gauss": int(has_gauss), "cached": float(cached)}


def _rng_state_from_dict(d):
    return (d["name"], d["keys"].numpy().astype(np.uint32), d["pos"], d["has_gauss"], d["cached"])
