"""Fail-safe one-process-per-GPU supervisor with configuration fallback (no GPU in this process).

The reference launches every rank by hand and has no failure handling beyond the
``init_process_group`` timeout (ddp_guide/run_script.py:4-23, ddp_guide_cifar10/ddp_init.py:92).
A benchmark of a multi-GPU step must instead end in exactly one of two ways: a number
that was measured on a step whose results are verified, or a non-zero exit.  A rank that
hangs inside a GPU kernel cannot recover in-process, so the supervision lives OUTSIDE the
GPU processes:

* the supervisor never touches the GPU (it may import torch only for a c10d ``TCPStore``);
  it starts the worker processes (``subprocess``, new session — never ``exec``), each of
  which runs ONE configuration ``level`` of an ordered fallback ladder;
* a worker reports progress through a heartbeat file (``<phase> <allowance seconds>``
  written by the worker's MAIN thread at each phase boundary), its failure through
  ``error.<rank>``, success through ``done.<rank>`` and rank 0's result line through
  ``result.json`` — all in a private directory (``NDP_SUP_DIR``);
* a worker that exits non-zero before ``done``, or whose heartbeat is older than the
  allowance it declared, fails the attempt: every worker of the attempt is killed
  (process group SIGTERM, then SIGKILL) and the next level starts on a fresh rendezvous
  port;
* two launch modes share this logic:
  - ``local``: no ``WORLD_SIZE`` in the environment (``python bench.py --gpus N``): the
    supervisor starts all N workers itself (RANK = LOCAL_RANK = i, MASTER_ADDR 127.0.0.1);
  - ``torchrun``: one supervisor per rank (``torchrun ... bench.py --gpus N``); the
    supervisors agree on each attempt through the launcher's store (the agent store when
    ``TORCHELASTIC_USE_AGENT_STORE=True``, else rank 0 hosts one at ``MASTER_PORT``): a
    fresh worker port per attempt, a ``fail`` key any rank can set (every supervisor then
    kills its own worker, which may sit in a collective waiting for the failed peer), and
    a ``finished`` counter so that all ranks decide the attempt's outcome together.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

__all__ = ["Heartbeat", "AttemptResult", "supervise_local", "supervise_torchrun", "worker_env_info"]

ROLE_ENV = "NDP_SUP_ROLE"
DIR_ENV = "NDP_SUP_DIR"
LEVEL_ENV = "NDP_SUP_LEVEL"


def _log(msg: str) -> None:
    print(f"[supervisor] {msg}", file=sys.stderr, flush=True)


# ---- worker side ------------------------------------------------------------------------------
class Heartbeat:
    """Worker-side progress reporting.  ``beat(phase, allow_s)`` promises the supervisor that
    the next beat (or exit) comes within ``allow_s`` seconds.  No-ops outside supervision."""

    def __init__(self, rank: int, directory: Optional[str] = None):
        self.rank = rank
        self.dir = directory if directory is not None else os.environ.get(DIR_ENV)

    @property
    def enabled(self) -> bool:
        return bool(self.dir)

    def _write(self, name: str, text: str) -> None:
        if not self.dir:
            return
        path = os.path.join(self.dir, name)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(text)
        os.replace(tmp, path)

    def beat(self, phase: str, allow_s: float) -> None:
        self._write(f"hb.{self.rank}", f"{phase} {float(allow_s)}")

    def error(self, msg: str) -> None:
        self._write(f"error.{self.rank}", msg)

    def result(self, line: str) -> None:
        self._write("result.json", line)

    def done(self) -> None:
        self._write(f"done.{self.rank}", "ok")


def worker_env_info():
    """(role, level, directory) of this process: role is None outside supervision."""
    return (os.environ.get(ROLE_ENV), int(os.environ.get(LEVEL_ENV, "0")), os.environ.get(DIR_ENV))


# ---- supervisor side ------------------------------------------------------------------------------
@dataclass
class AttemptResult:
    level: int
    ok: bool
    result: Optional[str] = None
    errors: Dict[int, str] = field(default_factory=dict)
    seconds: float = 0.0


class _Worker:
    def __init__(self, rank: int, cmd: Sequence[str], env: dict, directory: str):
        self.rank = rank
        self.dir = directory
        self.started = time.time()
        self.out = open(os.path.join(directory, f"stdout.{rank}"), "w")
        self.proc = subprocess.Popen(list(cmd), env=env, stdout=self.out, stderr=None, start_new_session=True)
        self.status: Optional[str] = None  # None running | "done" | "failed"
        self.reason = ""

    def _read(self, name: str) -> Optional[str]:
        try:
            with open(os.path.join(self.dir, name)) as f:
                return f.read()
        except OSError:
            return None

    def heartbeat(self):
        """(phase, allowance, age seconds) of the last beat, or None before the first."""
        path = os.path.join(self.dir, f"hb.{self.rank}")
        text = self._read(f"hb.{self.rank}")
        if text is None:
            return None
        try:
            phase, allow = text.rsplit(" ", 1)
            return phase, float(allow), time.time() - os.path.getmtime(path)
        except (ValueError, OSError):
            return None

    def poll(self, start_allow_s: float) -> Optional[str]:
        """Update and return the status: None (running), "done" or "failed"."""
        if self.status is not None:
            return self.status
        rc = self.proc.poll()
        if self._read(f"done.{self.rank}") is not None and rc is not None:
            self.status = "done"
            if rc != 0:  # measured and verified, then crashed in teardown: keep, but say so
                self.reason = f"exit code {rc} after completion (teardown)"
            return self.status
        if rc is not None:
            self.status = "failed"
            err = self._read(f"error.{self.rank}")
            self.reason = (err.strip() if err else f"exit code {rc}") + (f" [rc={rc}]" if err else "")
            return self.status
        hb = self.heartbeat()
        if hb is None:
            if time.time() - self.started > start_allow_s:
                self.status, self.reason = "failed", f"no heartbeat within {start_allow_s:.0f} s of start"
        else:
            phase, allow, age = hb
            if age > allow:
                self.status, self.reason = "failed", f"stalled in phase '{phase}' ({age:.0f} s > {allow:.0f} s allowed)"
        return self.status

    def kill(self) -> None:
        if self.proc.poll() is None:
            for sig, grace in ((signal.SIGTERM, 5.0), (signal.SIGKILL, 10.0)):
                try:
                    os.killpg(self.proc.pid, sig)
                except (ProcessLookupError, PermissionError):
                    break
                try:
                    self.proc.wait(timeout=grace)
                    break
                except subprocess.TimeoutExpired:
                    continue
        self.out.close()


def _worker_env(base: dict, rank: int, local_rank: int, world: int, local_world: int, port: int, addr: str,
                level: int, directory: str) -> dict:
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(local_world), "MASTER_ADDR": addr, "MASTER_PORT": str(port),
                ROLE_ENV: "worker", LEVEL_ENV: str(level), DIR_ENV: directory})
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)  # the worker group hosts its own store
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _free_port(host: str = "127.0.0.1") -> int:
    from .launcher import find_free_port

    return find_free_port(host)


def supervise_local(cmd: Sequence[str], world: int, levels: int, start_allow_s: float = 900.0,
                    poll_s: float = 0.2, progress_s: float = 30.0,
                    keep_dirs: bool = False, first_level: int = 0) -> List[AttemptResult]:
    """Run ``cmd`` as ``world`` local ranks at fallback level 0, 1, ... until one attempt
    completes on every rank.  Returns every attempt (the last one is the successful one if any)."""
    attempts: List[AttemptResult] = []
    for level in range(first_level, levels):
        t0 = time.time()
        directory = tempfile.mkdtemp(prefix=f"ndp_sup_l{level}_")
        port = _free_port()
        workers = [_Worker(r, cmd, _worker_env(os.environ, r, r, world, world, port, "127.0.0.1", level, directory),
                           directory) for r in range(world)]
        res = AttemptResult(level=level, ok=False)
        last_note = time.time()
        try:
            while True:
                states = [w.poll(start_allow_s) for w in workers]
                if any(s == "failed" for s in states):
                    break
                if all(s == "done" for s in states):
                    res.ok = True
                    break
                if time.time() - last_note > progress_s:
                    last_note = time.time()
                    _log(f"level {level}: waiting for ranks {[w.rank for w in workers if w.status is None]} "
                         f"({time.time() - t0:.0f} s)")
                time.sleep(poll_s)
        finally:
            for w in workers:
                w.kill()
        res.errors = {w.rank: w.reason for w in workers if w.reason}
        if res.ok:
            try:
                with open(os.path.join(directory, "result.json")) as f:
                    res.result = f.read().strip()
            except OSError:
                res.result = None
        res.seconds = time.time() - t0
        attempts.append(res)
        if not keep_dirs:
            _rmtree(directory)
        if res.ok:
            break
        _log(f"level {level} failed after {res.seconds:.0f} s: {res.errors}")
    return attempts


class _Coordinator:
    """Cross-supervisor agreement through the launcher's c10d store (torchrun mode)."""

    def __init__(self, rank: int, world: int, addr: str, port: int, timeout_s: float):
        import datetime

        from torch.distributed import TCPStore  # CPU-only: no GPU is touched

        agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
        self.store = TCPStore(addr, port, world, is_master=(rank == 0 and not agent),
                              timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False)
        self.prefix = "ndp_sup/{}/{}".format(os.environ.get("TORCHELASTIC_RUN_ID", "run"),
                                            os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        self.rank, self.world = rank, world

    def key(self, level: int, what: str) -> str:
        return f"{self.prefix}/{level}/{what}"

    def port(self, level: int) -> int:
        k = self.key(level, "port")
        if self.rank == 0:
            self.store.set(k, str(_free_port()))
        return int(self.store.get(k).decode())

    def failed(self, level: int) -> bool:
        return self.store.check([self.key(level, "fail")])

    def fail(self, level: int, reason: str) -> None:
        self.store.set(self.key(level, f"err/{self.rank}"), reason[:2000])
        self.store.set(self.key(level, "fail"), str(self.rank))

    def finish(self, level: int, deadline_s: float) -> None:
        self.store.add(self.key(level, "finished"), 1)
        t0 = time.time()
        while int(self.store.add(self.key(level, "finished"), 0)) < self.world:
            if time.time() - t0 > deadline_s:
                raise RuntimeError(f"supervisor: peers did not finish level {level} within {deadline_s:.0f} s")
            time.sleep(0.1)

    def errors(self, level: int) -> Dict[int, str]:
        out = {}
        for r in range(self.world):
            k = self.key(level, f"err/{r}")
            if self.store.check([k]):
                out[r] = self.store.get(k).decode()
        return out


def supervise_torchrun(cmd: Sequence[str], levels: int, start_allow_s: float = 900.0, poll_s: float = 0.2,
                       progress_s: float = 30.0, store_timeout_s: float = 1800.0,
                       first_level: int = 0) -> List[AttemptResult]:
    """One supervisor per rank (under torchrun / any env:// launcher); see the module docstring."""
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    coord = _Coordinator(rank, world, addr, int(os.environ["MASTER_PORT"]), store_timeout_s)
    attempts: List[AttemptResult] = []
    for level in range(first_level, levels):
        t0 = time.time()
        directory = tempfile.mkdtemp(prefix=f"ndp_sup_r{rank}_l{level}_")
        port = coord.port(level)
        w = _Worker(rank, cmd, _worker_env(os.environ, rank, local_rank, world, local_world, port, addr, level,
                                           directory), directory)
        res = AttemptResult(level=level, ok=False)
        last_note = time.time()
        try:
            while True:
                st = w.poll(start_allow_s)
                if st == "failed":
                    coord.fail(level, w.reason)
                    break
                if st == "done":
                    break
                if coord.failed(level):
                    w.status, w.reason = "failed", "peer failure (killed)"
                    break
                if time.time() - last_note > progress_s:
                    last_note = time.time()
                    _log(f"rank {rank} level {level}: running ({time.time() - t0:.0f} s)")
                time.sleep(poll_s)
        finally:
            w.kill()
        coord.finish(level, deadline_s=start_allow_s)
        res.ok = not coord.failed(level)
        res.errors = coord.errors(level)
        if res.ok and rank == 0:
            try:
                with open(os.path.join(directory, "result.json")) as f:
                    res.result = f.read().strip()
            except OSError:
                res.result = None
        res.seconds = time.time() - t0
        attempts.append(res)
        _rmtree(directory)
        if res.ok:
            break
        if rank == 0:
            _log(f"level {level} failed after {res.seconds:.0f} s: {res.errors}")
    return attempts


def _rmtree(path: str) -> None:
    import shutil

    shutil.rmtree(path, ignore_errors=True)


def attach_attempts(line: str, attempts: List[AttemptResult]) -> str:
    """Add the supervisor's record (failed levels and why) to the worker's JSON result line."""
    rec = json.loads(line)
    failed = [{"level": a.level, "errors": {str(k): v[:300] for k, v in a.errors.items()},
               "seconds": round(a.seconds, 1)} for a in attempts if not a.ok]
    rec["supervisor"] = {"level": attempts[-1].level, "attempts": len(attempts), "failed": failed}
    return json.dumps(rec)


def run_supervised(cmd: Sequence[str], world: int, levels: int,
                   describe: Callable[[int], str] = str, **kw) -> int:
    """Pick the launch mode from the environment, supervise, print rank 0's line.  Returns
    the process exit code (0 only if some level completed and verified on every rank)."""
    if os.environ.get("WORLD_SIZE") is not None:
        attempts = supervise_torchrun(cmd, levels, **{k: v for k, v in kw.items() if k != "keep_dirs"})
        is_rank0 = int(os.environ.get("RANK", "0")) == 0
    else:
        attempts = supervise_local(cmd, world, levels, **kw)
        is_rank0 = True
    last = attempts[-1] if attempts else None
    if last is None or not last.ok:
        if is_rank0:
            _log("every configuration failed: " + "; ".join(
                f"level {a.level} ({describe(a.level)}): {a.errors}" for a in attempts))
        return 1
    if is_rank0:
        if not last.result:
            _log("rank 0 completed without a result line")
            return 1
        print(attach_attempts(last.result, attempts), flush=True)
    return 0
