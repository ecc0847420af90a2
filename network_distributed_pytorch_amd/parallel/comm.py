"""Collective layer: world-size-guarded collectives, byte accounting, link emulation, and the
native RCCL data plane.

Reference behaviour kept:
  * ``all_reduce`` / ``all_gather`` are no-ops at world size 1
    (ddp_powersgd_guide_cifar10/reducer.py:193-195, tensor_buffer.py:59-69);
  * ``n_bits(t) = 8 * numel * element_size`` (reducer.py:197-198).

MI355X design:
  * **Data plane = native RCCL** (``csrc/comm.cpp``, :class:`RcclComm`): c10d only
    bootstraps.  Rank 0's ``ncclUniqueId`` goes through the c10d store, every rank calls
    ``ncclCommInitRank``, and collectives are enqueued straight onto a HIP stream: the
    framework-owned high-priority side stream (``csrc/comm.cpp`` SideStream), ordered
    against the compute stream with hipEvents (:meth:`Communicator.side_launch`), so
    bucket / PowerSGD-group work overlaps backward — eagerly, or as the comm graph of a
    captured step, ordered against the compute graph by device flags (utils/graph.py).  c10d (``ProcessGroupNCCL`` = RCCL, or gloo for
    CPU tests) is the fallback data plane.
  * every collective is accounted (calls, payload bytes, modelled ring wire bytes
    2(N-1)/N * S) so the bytes/step metric is measured, not only derived;
  * :class:`LinkModel` paces each collective to an emulated 1/10/100 Gb link
    (``alpha + wire_bits / bandwidth``) by stalling the stream that carries the collective
    with a wall-clock spin kernel (no root / ``tc`` on the GPU box) — the reference's
    README.md:2 bandwidth experiments.  ``emulate_world=N`` charges the N-rank ring time
    even in a 1-GPU run (one-GPU rehearsal of an N-GPU bandwidth curve);
  * ``NDP_FORCE_COLLECTIVES=1`` issues the collectives even in a 1-rank process group
    (:attr:`Communicator.active`): a one-GPU rehearsal of the N > 1 RCCL path whose sums
    are the identity, so results match the world-size-1 no-op path.
  * ``NDP_NATIVE_COMM=0`` forces the c10d data plane.
  * ``NDP_COMM=ipc`` (opt-in) replaces RCCL with :class:`IpcDataPlane`: one-shot all-reduce
    kernels on HIP IPC peer memory (csrc/ipc.hip) — stream-ordered and graph-capturable like
    the RCCL plane, and usable by several ranks sharing ONE GPU (RCCL refuses that), which is
    how the captured, backward-overlapped multi-rank step is exercised on a one-GPU box.
"""
from __future__ import annotations

import contextlib
import dataclasses
import os
import time
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

__all__ = [
    "n_bits",
    "all_reduce",
    "all_gather",
    "world_size",
    "get_rank",
    "LinkModel",
    "CommStats",
    "Communicator",
    "LINK_PRESETS",
    "create_native_comm",
    "FlagTimeout",
]


def n_bits(tensor: torch.Tensor) -> int:
    """Bits in a tensor payload (reducer.py:197-198)."""
    return 8 * tensor.nelement() * tensor.element_size()


def world_size(group=None) -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


def get_rank(group=None) -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group)
    return 0


def all_reduce(*args, **kwargs):
    """``dist.all_reduce`` guarded for world size 1 (reducer.py:193-195)."""
    if world_size(kwargs.get("group")) > 1:
        return dist.all_reduce(*args, **kwargs)
    return None


def all_gather(out_list: List[torch.Tensor], in_tensor: torch.Tensor, **kwargs):
    """``dist.all_gather`` with the single-worker aliasing fallback (tensor_buffer.py:64-69)."""
    if world_size(kwargs.get("group")) > 1:
        return dist.all_gather(out_list, in_tensor, **kwargs)
    assert len(out_list) == 1
    out_list[0].data = in_tensor
    return None


@dataclasses.dataclass
class LinkModel:
    """Emulated point-to-point link: time(S) = alpha + 8*wire(S)/bandwidth_bps (ring)."""

    bandwidth_bps: float
    alpha_s: float = 25e-6
    name: str = "custom"

    def wire_bytes(self, payload: int, n: int) -> float:
        return 0.0 if n <= 1 else 2.0 * (n - 1) / n * payload

    def seconds(self, payload: int, n: int) -> float:
        if n <= 1:
            return 0.0
        return self.alpha_s + 8.0 * self.wire_bytes(payload, n) / self.bandwidth_bps


LINK_PRESETS = {
    "1g": LinkModel(1e9, 50e-6, "1Gb"),
    "10g": LinkModel(10e9, 30e-6, "10Gb"),
    "100g": LinkModel(100e9, 10e-6, "100Gb"),
}


@dataclasses.dataclass
class CommStats:
    calls: int = 0
    payload_bytes: int = 0
    wire_bytes: float = 0.0
    emulated_seconds: float = 0.0

    def reset(self):
        self.calls = 0
        self.payload_bytes = 0
        self.wire_bytes = 0.0
        self.emulated_seconds = 0.0

    def as_dict(self):
        return dataclasses.asdict(self)


class FlagTimeout(RuntimeError):
    """A compute/comm graph ordering wait timed out (see :meth:`Communicator.check`)."""


class _PacedWork:
    """Async handle that applies link pacing when waited on (c10d data plane)."""

    def __init__(self, work, comm: "Communicator", seconds: float, device_tensor: bool):
        self._work = work
        self._comm = comm
        self._seconds = seconds
        self._device = device_tensor

    def wait(self):
        if self._work is not None:
            self._work.wait()
        self._comm._pace(self._seconds, self._device)
        return True

    def is_completed(self):
        return self._work is None or self._work.is_completed()


class _StreamWork:
    """Handle of a stream-ordered (native RCCL) collective: already ordered on its stream."""

    def wait(self):
        return True

    def is_completed(self):
        return True


_MAX_FLAGS = 256
_DONE, _ERR = 2 * _MAX_FLAGS, 2 * _MAX_FLAGS + 2
# A flag wait gives up after this long (device wall clock) instead of hanging the GPU, sets
# the sticky error word and lets the step run unordered; that step's results are never used:
# check() raises on the word (bench health checks, engine logging cadence).  30 s covers rank
# skew (a peer writing a checkpoint, capture skew) and emulated 1 Gb steps (3.75 s for dense
# DistilBERT); NDP_FLAG_WAIT_US lowers it to inject a timeout in tests.
_WAIT_US = int(os.environ.get("NDP_FLAG_WAIT_US", "30000000"))
_SIDE_LINKS = {}
_KEEPALIVE = []


def _side_link(device_index: int):
    """One framework-owned side stream (+ its events) per device and process.  Never
    destroyed: captured graphs hold its events and stream for their whole lifetime, and
    Python's cycle collector frees graphs and streams in no particular order."""
    if device_index not in _SIDE_LINKS:
        from ..ops import ext

        link = ext().SideStream(device_index, os.environ.get("NDP_SIDE_PRIORITY", "high") == "high")
        _SIDE_LINKS[device_index] = (link, torch.cuda.ExternalStream(link.handle,
                                                                      device=torch.device("cuda", device_index)))
    return _SIDE_LINKS[device_index]


def _native_wanted() -> bool:
    return os.environ.get("NDP_NATIVE_COMM", "1") != "0"


def _comm_kind() -> str:
    return os.environ.get("NDP_COMM", "rccl")


class IpcDataPlane:
    """Stream-ordered data plane on HIP IPC peer memory (csrc/ipc.hip): one-shot
    fixed-order all-reduce kernels, graph-capturable, bitwise identical on every rank.
    Opt-in (``NDP_COMM=ipc``) and usable where RCCL is not — several ranks sharing one GPU
    (gloo process group for the bootstrap).  broadcast / all_gather (init-time only) go
    through the c10d group, blocking."""

    def __init__(self, group, device: torch.device, capacity_bytes: int = 8 << 20):
        from ..ops import ext

        X = ext()
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
        self.group = group
        self.rank_in_group = dist.get_rank(group)
        self._c = X.IpcComm(self.rank_in_group, len(ranks), device.index if device.index is not None else 0,
                            int(capacity_bytes))
        store = dist.distributed_c10d._get_default_store()
        IpcDataPlane._n = getattr(IpcDataPlane, "_n", 0) + 1
        key = "ndp_ipc/{}/{}".format("-".join(map(str, ranks)), IpcDataPlane._n)
        # peers on another device need the uncached buffer (csrc/ipc.hip header): every rank
        # publishes its device's PCI bus id and whether its buffer is uncached; a cached
        # buffer is only paired with ranks on the same device (all ranks decide alike)
        store.set(f"{key}/dev/{self.rank_in_group}", f"{self._c.bus_id()}|{int(self._c.uncached)}")
        devs = [store.get(f"{key}/dev/{r}").decode().split("|") for r in range(len(ranks))]
        if len({d for d, _ in devs}) > 1 and not all(u == "1" for _, u in devs):
            self._c.destroy()
            raise RuntimeError("IPC data plane: ranks on different GPUs need the uncached peer buffer, which this "
                               "allocator/IPC export refused; use NDP_COMM=rccl")
        store.set(f"{key}/{self.rank_in_group}", self._c.handle())
        handles = [store.get(f"{key}/{r}") for r in range(len(ranks))]
        self._c.open(handles)
        dist.barrier(group=group)  # every rank mapped every buffer before the first collective

    @property
    def nranks(self) -> int:
        return self._c.nranks

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        self._c.all_reduce(t, op)

    def all_reduce_many(self, ts):
        self._c.all_reduce_many(list(ts))  # one launch (segment table, csrc/ipc.hip)

    @property
    def uncached(self) -> bool:
        return bool(self._c.uncached)

    @property
    def launches(self) -> int:
        return int(self._c.launches)

    def broadcast(self, t: torch.Tensor, src: int = 0):
        torch.cuda.current_stream().synchronize()
        dist.broadcast(t, src=src, group=self.group)

    def all_gather(self, out: torch.Tensor, t: torch.Tensor):
        # through host memory: gloo gathers no device tensors (init-time / check-time only)
        host = [torch.empty(t.numel(), dtype=t.dtype) for _ in range(self.nranks)]
        dist.all_gather(host, t.reshape(-1).cpu(), group=self.group)
        out.copy_(torch.cat(host).to(out.device))

    def check(self):
        self._c.check()

    def destroy(self):
        self._c.destroy()


def create_native_comm(group=None, device: Optional[torch.device] = None):
    """Bootstrap an :class:`RcclComm` over ``group`` (collective: every rank must call it).

    Rank 0 of the group draws the ``ncclUniqueId``; its 128 bytes are exchanged through the
    default c10d store under a per-group, per-call key.  Returns None when the native data
    plane is unavailable (no device, no extension, not an nccl group, or disabled).
    """
    if not (_native_wanted() and dist.is_available() and dist.is_initialized() and torch.cuda.is_available()):
        return None
    from ..ops import native_available, ext

    if not native_available():
        return None
    if _comm_kind() == "ipc":  # opt-in peer-memory data plane (any bootstrap backend)
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        return IpcDataPlane(group, dev)
    try:
        if dist.get_backend(group) != "nccl":
            return None
    except Exception:
        return None
    X = ext()
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    store = dist.distributed_c10d._get_default_store()
    create_native_comm._n = getattr(create_native_comm, "_n", 0) + 1
    ranks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
    key = "ndp_rccl_uid/{}/{}".format("-".join(map(str, ranks)), create_native_comm._n)
    rank = dist.get_rank(group)
    if rank == 0:
        store.set(key, X.rccl_unique_id())
    uid = store.get(key)
    return X.RcclComm(uid, len(ranks), rank, dev.index if dev.index is not None else 0)


class Communicator:
    """Accounting + pacing front-end over the native RCCL communicator or a c10d group.

    Stream-ordered API (device tensors) used by the overlapped gradient-sync engines:
    :meth:`fork` (side stream waits for the compute stream), :meth:`on_side` (context that
    makes the side stream current), :meth:`join` (compute stream waits for the side stream).
    """

    def __init__(self, group=None, link: Optional[LinkModel] = None, native: Optional[bool] = None,
                 emulate_world: Optional[int] = None, device: Optional[torch.device] = None):
        self.group = group
        self.link = link
        self.emulate_world = emulate_world
        self.stats = CommStats()
        self._native = None
        self._side = None
        self._deferred = None
        self._flags = None
        self._captured = False
        self._device = device
        self.side_launches = 0  # eager side launches so far (StepRunner: does a step use the side stream?)
        if native is not False and self.active:
            self._native = create_native_comm(group, device)
            if native is True and self._native is None:
                raise RuntimeError("native RCCL communicator requested but unavailable")

    # -- topology ---------------------------------------------------------------------------
    @property
    def world_size(self) -> int:
        return world_size(self.group)

    @property
    def rank(self) -> int:
        return get_rank(self.group)

    @property
    def active(self) -> bool:
        """Whether collectives are issued (world > 1, or forced for a 1-rank rehearsal)."""
        if self.world_size > 1:
            return True
        return os.environ.get("NDP_FORCE_COLLECTIVES") == "1" and dist.is_available() and dist.is_initialized()

    @property
    def has_traffic(self) -> bool:
        """Whether a step spends time on the wire: real collectives, or link-model pacing of an
        emulated world.  Overlapping the gradient sync with backward only pays when True (at
        one rank the side stream would only add a resident wait kernel)."""
        return self.active or (self.link is not None and self.paced_world > 1)

    @property
    def backend(self) -> str:
        if self._native is not None:
            return "ipc-native" if isinstance(self._native, IpcDataPlane) else "rccl-native"
        if not self.active:
            return "none"
        try:
            return "c10d-" + str(dist.get_backend(self.group))
        except Exception:
            return "c10d"

    @property
    def native(self):
        return self._native

    @property
    def stream_ordered(self) -> bool:
        """True if device collectives are ordered on HIP streams (no host blocking), i.e.
        the overlapped / graph-captured step is possible: native RCCL, or nothing to issue."""
        return self._native is not None or not self.active

    @property
    def paced_world(self) -> int:
        return self.emulate_world if self.emulate_world else self.world_size

    # -- side stream (framework-owned HIP stream, csrc/comm.cpp SideStream) --------------------
    def _link(self):
        if self._side is None:
            dev = self._device or torch.device("cuda", torch.cuda.current_device())
            idx = dev.index if dev.index is not None else torch.cuda.current_device()
            self._side = _side_link(idx)
        return self._side

    def side_stream(self):
        return self._link()[1]

    def fork(self):
        """The side stream waits for all work enqueued so far on the current stream."""
        self._link()[0].fork()

    def join(self):
        """The current stream waits for all work enqueued so far on the side stream."""
        self._link()[0].join()

    @contextlib.contextmanager
    def on_side(self):
        with torch.cuda.stream(self.side_stream()):
            yield

    def side_launch(self, fn):
        """Run ``fn`` (kernels + collectives) on the side stream after the work enqueued so
        far on the current stream.  Eagerly: hipEvent fork + run.  While a step is being
        captured (:meth:`defer_side`): a device-flag signal kernel goes into the compute
        graph and ``fn`` is kept, to be captured into the comm graph behind a matching
        device-flag wait (:meth:`graph_wait`)."""
        if self._deferred is not None:
            i = len(self._deferred)
            assert i < _MAX_FLAGS, "too many side launches in one captured step"
            self._flag_ext().flag_signal(self._flag_buf(), i)
            self._deferred.append([fn])
            return
        self.side_launches += 1
        self.fork()
        with self.on_side():
            fn()

    def side_join(self):
        """Current stream waits for the side stream (skipped while capturing the compute
        graph: the comm graph signals the next step's compute graph through a flag)."""
        if self._deferred is None:
            self.join()

    @contextlib.contextmanager
    def defer_side(self):
        """Capture scope of the compute graph: yields the list that collects the side work
        (one list of callables per signal)."""
        assert self._deferred is None, "nested defer_side"
        self._flag_buf()  # allocate NOW: inside a capture it would come from the graph's pool
        self._deferred = []
        try:
            yield self._deferred
        finally:
            self._deferred = None

    # device-flag protocol between the compute graph (current stream) and the comm graph
    # (side stream); csrc/multitensor.hip flag_signal / flag_wait.  Layout of the int32
    # flag buffer: [0, MAX) signal counters, [MAX, 2 MAX) their "seen" words, then
    # DONE counter, DONE seen, error word.
    def _flag_ext(self):
        from ..ops import ext
        return ext()

    def _flag_buf(self):
        if self._flags is None:
            assert not torch.cuda.is_current_stream_capturing(), "flag buffer must exist before capture"
            dev = self._device or torch.device("cuda", torch.cuda.current_device())
            self._flags = torch.zeros(2 * _MAX_FLAGS + 3, dtype=torch.int32, device=dev)
            # pinned host mirror of the error word (set by a timed-out wait kernel; read by
            # StepRunner before every replay without a device sync)
            self._host_err = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        return self._flags

    def graph_prologue(self):
        """First node of the compute graph: wait until the previous step's comm graph is done."""
        self._flag_ext().flag_wait(self._flag_buf(), _DONE, _DONE + 1, _ERR, _WAIT_US, self._host_err)

    def graph_wait(self, i: int):
        """Comm graph: wait for the compute graph's i-th signal."""
        self._flag_ext().flag_wait(self._flag_buf(), i, _MAX_FLAGS + i, _ERR, _WAIT_US, self._host_err)

    def host_flag_error(self) -> int:
        """The error word as last mirrored to host memory by a wait kernel (no device sync)."""
        h = getattr(self, "_host_err", None)
        return int(h[0]) if h is not None else 0

    def raise_flag_error(self):
        raise FlagTimeout("compute/comm graph ordering: a device-flag wait timed out after "
                          f"{_WAIT_US / 1e6:.3g} s (a stalled peer, or the two streams share a hardware "
                          "queue); the steps since are unordered and must not be used")

    def graph_epilogue(self):
        """Last node of the comm graph: release the next step's compute graph."""
        self._flag_ext().flag_signal(self._flag_buf(), _DONE)

    def reset_flags(self):
        """Before the first replay: counters zero, DONE pre-signalled once."""
        f = self._flag_buf()
        f.zero_()
        f[_DONE] = 1
        self._host_err.zero_()

    def flag_error(self) -> int:
        return int(self._flags[_ERR].item()) if self._flags is not None else 0

    # -- pacing / accounting --------------------------------------------------------------------
    def _pace(self, seconds: float, device_tensor: bool):
        if seconds <= 0:
            return
        if device_tensor:
            from ..ops import delay_ns

            delay_ns(int(seconds * 1e9))
        else:
            time.sleep(seconds)

    def _account(self, t: torch.Tensor) -> float:
        n = self.paced_world
        payload = t.nelement() * t.element_size()
        self.stats.calls += 1
        self.stats.payload_bytes += payload
        self.stats.wire_bytes += 0.0 if n <= 1 else 2.0 * (n - 1) / n * payload
        secs = self.link.seconds(payload, n) if self.link is not None else 0.0
        self.stats.emulated_seconds += secs
        return secs

    def pace_seconds(self, payload_bytes: int) -> float:
        return self.link.seconds(payload_bytes, self.paced_world) if self.link is not None else 0.0

    # -- collectives ----------------------------------------------------------------------------
    def all_reduce(self, t: torch.Tensor, async_op: bool = False, op=None):
        secs = self._account(t)
        if not self.active:
            self._pace(secs, t.is_cuda)  # emulated world on a 1-GPU run: charge the link only
            return _PacedWork(None, self, 0.0, t.is_cuda) if async_op else None
        if self._native is not None and t.is_cuda:
            self._captured |= torch.cuda.is_current_stream_capturing()
            self._native.all_reduce(t, _op_name(op))
            self._pace(secs, True)
            return _StreamWork() if async_op else None
        kw = {"group": self.group}
        if op is not None:
            kw["op"] = op
        if async_op:
            work = dist.all_reduce(t, async_op=True, **kw)
            return _PacedWork(work, self, secs, t.is_cuda)
        dist.all_reduce(t, **kw)
        self._pace(secs, t.is_cuda)
        return None

    def all_reduce_many(self, ts: Sequence[torch.Tensor]):
        """Several SUM all-reduces; ONE fused RCCL launch on the native data plane."""
        ts = [t for t in ts if t.numel()]
        if not ts:
            return
        if self._native is not None and self.active and all(t.is_cuda for t in ts):
            secs = sum(self._account(t) for t in ts)
            self._captured |= torch.cuda.is_current_stream_capturing()
            self._native.all_reduce_many(ts)
            self._pace(secs, True)
            return
        for t in ts:
            self.all_reduce(t)

    def all_gather(self, out_list: List[torch.Tensor], t: torch.Tensor, async_op: bool = False):
        self._account(t)
        if not self.active:
            assert len(out_list) == 1
            out_list[0].copy_(t)  # a copy, not the reference's alias (tensor_buffer.py:69):
            return None           # callers own out_list storage (TensorBuffer.all_gather)
        if self._native is not None and t.is_cuda:
            flat = torch.empty(len(out_list) * t.numel(), dtype=t.dtype, device=t.device)
            self._native.all_gather(flat, t.contiguous())
            for i, o in enumerate(out_list):
                o.copy_(flat[i * t.numel(): (i + 1) * t.numel()].view_as(o))
            return _StreamWork() if async_op else None
        return dist.all_gather(out_list, t, group=self.group, async_op=async_op)

    def broadcast(self, t: torch.Tensor, src: int = 0):
        if not self.active:
            return None
        if self._native is not None and t.is_cuda and t.is_contiguous():
            self._native.broadcast(t, src)
            return None
        return dist.broadcast(t, src=src, group=self.group)

    def barrier(self):
        if self.active:
            dist.barrier(group=self.group)

    def check(self):
        """Raise if the native communicator reported an asynchronous RCCL error, or a
        compute/comm graph flag wait timed out (host sync: call at a low cadence)."""
        if self._native is not None:
            self._native.check()
        if self.flag_error():
            self.raise_flag_error()

    def close(self):
        """Destroy the native communicator — unless a captured graph contains its
        collectives (RCCL ties graph-owned resources to the communicator; destroying it
        before the graph is freed aborts the process), in which case it is kept alive."""
        if self._native is not None:
            if self._captured:
                _KEEPALIVE.append(self._native)
            else:
                self._native.destroy()
            self._native = None


def _op_name(op) -> str:
    if op is None or op == dist.ReduceOp.SUM:
        return "sum"
    if op == dist.ReduceOp.MAX:
        return "max"
    if op == dist.ReduceOp.MIN:
        return "min"
    if op == dist.ReduceOp.PRODUCT:
        return "prod"
    if op == dist.ReduceOp.AVG:
        return "avg"
    raise ValueError(f"unsupported reduce op {op}")
