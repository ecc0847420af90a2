"""Shared ``run_script.py`` CLI for every workload (reference: */run_script.py).

Reference flags kept: ``-rank INT -cuda INT`` (all), ``-world_size INT`` and
``-init_method STR`` (ddp_powersgd_distillBERT_IMDb/run_script.py:27-30; here for every
workload — quirk Q12 fixed: the CIFAR scripts hard-code ``n_workers = 4``, which stays the
default).  Additions: ``-spawn`` launches all ranks locally (127.0.0.1 rendezvous),
``-epochs``, ``-steps`` (max steps per epoch), ``-model``, ``-grad_sync``, ``-rank_r``
(PowerSGD rank), ``-batch`` (global batch), ``-graph_mode``, ``-link``, ``-backend``,
``-checkpoint_dir``, ``-resume``, ``-log_file`` (``{rank}`` in the path = one file per rank),
``-log_every``, ``-dataset_size``, ``-check_replicas``, ``-bucket_mb``, ``-reuse_query``,
``-overlap``, ``-psgd_groups``, ``-emulate_world``.
"""
from __future__ import annotations

import argparse
import os
from types import ModuleType
from typing import Optional


def build_parser(default_world: int, world_required: bool = False) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("-rank", type=int, default=None, help="worker id")
    p.add_argument("-cuda", type=int, default=None, help="worker's cuda id")
    p.add_argument("-world_size", type=int, default=None if world_required else default_world)
    p.add_argument("-init_method", type=str, default=None,
                   help="tcp://IP:PORT or file://PATH (default: env/torchrun or file:// under output_dir)")
    p.add_argument("-spawn", action="store_true", help="launch all -world_size ranks on this node")
    p.add_argument("-epochs", type=int, default=None)
    p.add_argument("-steps", type=int, default=None, help="max steps per epoch")
    p.add_argument("-model", type=str, default=None)
    p.add_argument("-num_classes", type=int, default=None)
    p.add_argument("-grad_sync", type=str, default=None,
                   choices=[None, "powersgd", "powersgd-ref", "powersgd-api", "dense", "dense-ref"])
    p.add_argument("-rank_r", type=int, default=None, help="PowerSGD compression rank")
    p.add_argument("-batch", type=int, default=None, help="global batch")
    p.add_argument("-lr", type=float, default=None)
    p.add_argument("-graph_mode", type=str, default=None, choices=[None, "none", "full", "piecewise", "auto"])
    p.add_argument("-link", type=str, default=None, choices=[None, "none", "1g", "10g", "100g"])
    p.add_argument("-backend", type=str, default=None, choices=[None, "nccl", "gloo"])
    p.add_argument("-checkpoint_dir", type=str, default=None)
    p.add_argument("-resume", type=str, default=None)
    p.add_argument("-log_file", type=str, default=None)
    p.add_argument("-dataset_size", type=int, default=None)
    p.add_argument("-check_replicas", type=int, default=None, help="replica checksum every N steps")
    p.add_argument("-toy_steps", type=int, default=None, help="ddp_guide: toy-MLP dense-DP steps")
    p.add_argument("-bucket_mb", type=float, default=None, help="dense arm: all-reduce bucket size (MB)")
    p.add_argument("-reuse_query", type=int, default=None, choices=[None, 0, 1],
                   help="PowerSGD warm-start query (reducer.py reuse_query; 0 redraws Q every step)")
    p.add_argument("-overlap", type=int, default=None, choices=[None, 0, 1],
                   help="launch the gradient sync from grad hooks during backward (default 1 on GPU)")
    p.add_argument("-psgd_groups", type=int, default=None, help="PowerSGD overlap groups")
    p.add_argument("-emulate_world", type=int, default=None, help="link emulation: charge an N-rank ring")
    p.add_argument("-log_every", type=int, default=None, help="per-step JSONL record cadence (0 = off)")
    p.add_argument("-seq_len", type=int, default=None, help="DistilBERT sequence length (reference 512)")
    p.add_argument("-trace", action="store_true", help="per-phase HIP-event timings into the JSONL log")
    p.add_argument("-quiet", action="store_true")
    return p


_MAP = {"epochs": "training_epochs", "steps": "max_steps_per_epoch", "model": "model", "num_classes": "num_classes",
        "grad_sync": "grad_sync", "rank_r": "reducer_rank", "batch": "global_batch", "lr": "learning_rate",
        "graph_mode": "graph_mode", "link": "link", "backend": "distributed_backend",
        "checkpoint_dir": "checkpoint_dir", "resume": "resume", "log_file": "log_file",
        "dataset_size": "dataset_size", "check_replicas": "check_replicas_every", "toy_steps": "toy_mlp_steps",
        "bucket_mb": "bucket_mb", "psgd_groups": "psgd_groups", "emulate_world": "emulate_world",
        "log_every": "log_every", "seq_len": "seq_len"}


def apply_args(ddp_init: ModuleType, args, rank: int, world: int, cuda: Optional[int]):
    c = ddp_init.config
    c["n_workers"] = world
    c["rank"] = rank
    c["cuda_rank"] = rank if cuda is None else cuda
    if args.init_method:
        c["init_method"] = args.init_method
    elif os.environ.get("MASTER_ADDR") and os.environ.get("MASTER_PORT"):
        c["init_method"] = "env://"
    for a, k in _MAP.items():
        v = getattr(args, a)
        if v is not None:
            c[k] = v
    if args.reuse_query is not None:
        c["reuse_query"] = bool(args.reuse_query)
    if args.overlap is not None:
        c["overlap"] = bool(args.overlap)
    if args.quiet:
        c["verbose"] = False
    if args.trace:
        c["trace_phases"] = True


def _spawned(rank, world, module_name, argv):
    import importlib

    mod = importlib.import_module(module_name)
    args = build_parser(world).parse_args(argv)
    args.init_method = None
    apply_args(mod, args, rank, world, None)
    mod.setup()
    mod.run_task()
    mod.cleanup()


def main(ddp_init: ModuleType, default_world: int, world_required: bool = False, argv=None):
    args = build_parser(default_world, world_required).parse_args(argv)
    env_rank = os.environ.get("RANK")
    if args.spawn:
        from ..utils.launcher import spawn

        world = args.world_size or default_world
        import sys

        spawn(_spawned, world, args=(ddp_init.__name__, list(argv if argv is not None else sys.argv[1:])))
        return
    world = args.world_size if args.world_size is not None else int(os.environ.get("WORLD_SIZE", default_world))
    rank = args.rank if args.rank is not None else int(env_rank or 0)
    cuda = args.cuda if args.cuda is not None else (int(os.environ["LOCAL_RANK"]) if "LOCAL_RANK" in os.environ else None)
    apply_args(ddp_init, args, rank, world, cuda)
    ddp_init.setup()
    ddp_init.run_task()
    ddp_init.cleanup()
