"""Local multi-process launcher and rendezvous helpers.

The reference launches every rank by hand (``python run_script.py -rank R -cuda C`` on
each host; ddp_guide/run_script.py:4-23 documents an mpirun recipe).  Here:

* :func:`spawn` starts ``world_size`` ranks on this node (torch.multiprocessing) with a
  TCP rendezvous on 127.0.0.1 and a free port — used by the CPU/gloo tests and the
  ``-world_size N -spawn`` option of the run scripts;
* :func:`env_rank_info` reads torchrun's RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*;
* :func:`init_method_for` builds ``file://`` / ``tcp://`` init methods (ddp_guide uses a
  shared file, the others a TCP address).
"""
from __future__ import annotations

import os
import socket
from typing import Callable, Optional, Tuple

import torch.multiprocessing as mp

__all__ = ["find_free_port", "spawn", "env_rank_info", "init_method_for"]


def find_free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def _entry(rank: int, fn: Callable, world_size: int, port: int, args: tuple):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world_size)
    fn(rank, world_size, *args)


def spawn(fn: Callable, world_size: int, args: tuple = (), port: Optional[int] = None, join: bool = True):
    """Run ``fn(rank, world_size, *args)`` in ``world_size`` processes."""
    port = port or find_free_port()
    return mp.start_processes(_entry, args=(fn, world_size, port, args), nprocs=world_size, join=join,
                              start_method="spawn")


def env_rank_info() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_method_for(kind: str, output_dir: str = "./output.tmp", addr: str = "127.0.0.1", port: int = 29500) -> str:
    if kind == "file":
        os.makedirs(output_dir, exist_ok=True)
        return "file://" + os.path.abspath(os.path.join(output_dir, "dist_init"))
    if kind == "env":
        return "env://"
    return f"tcp://{addr}:{port}"
