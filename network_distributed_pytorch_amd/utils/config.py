"""Typed training configuration.

The reference keeps each experiment's settings in a module-level ``config`` dict
(ddp_powersgd_guide_cifar10/ddp_init.py:24-39); the workloads here keep that dict API.
:class:`TrainConfig` is the typed schema behind it: every key the engine reads, with its
type, default and allowed values.  :func:`validate_config` checks a dict against it (unknown
keys, types, choices, cross-field rules) and returns it with defaults filled in, so a typo
(``-reducer_rnak``) or an impossible combination fails at start-up with a clear message
instead of a KeyError deep in a run.
"""
from __future__ import annotations

import dataclasses
import typing
from typing import Any, Dict, Optional

__all__ = ["TrainConfig", "validate_config", "ConfigError"]


class ConfigError(ValueError):
    pass


GRAD_SYNCS = ("powersgd", "powersgd-ref", "powersgd-api", "dense", "dense-ref", "local-sgd-nesterov", "local-adamw")
TASKS = ("cifar", "imdb", "mlp")
GRAPH_MODES = ("auto", "full", "piecewise", "none")
LINKS = ("none", "1g", "10g", "100g")
BACKENDS = ("nccl", "gloo")


@dataclasses.dataclass
class TrainConfig:
    # reference keys (ddp_init.py config dicts)
    seed: int = 714
    rank: int = 0
    cuda_rank: int = 0
    n_workers: int = 1
    distributed_init_file: Optional[str] = None
    output_dir: str = "./output.tmp"
    distributed_backend: str = "nccl"
    init_method: Optional[str] = None
    timeout_s: float = 600
    learning_rate: float = 1e-3
    momentum: float = 0.9
    nesterov: bool = False
    training_epochs: int = 1
    batch_size: int = 32
    reducer_rank: int = 4
    # additions
    task: str = "cifar"
    model: str = "resnet18"
    num_classes: int = 1000
    global_batch: Optional[int] = 512
    seq_len: int = 512
    grad_sync: str = "powersgd"
    dataset_size: Optional[int] = None
    data_seed: int = 0
    max_steps_per_epoch: Optional[int] = None
    graph_mode: str = "auto"
    link: str = "none"
    emulate_world: Optional[int] = None
    bucket_mb: Optional[float] = None
    reuse_query: bool = True
    overlap: Optional[bool] = None
    psgd_groups: Optional[int] = None
    checkpoint_dir: Optional[str] = None
    resume: Optional[str] = None
    log_file: Optional[str] = None
    log_every: int = 1
    check_replicas_every: int = 0
    check_health_every: int = 50  # host check of flag-wait / MGS / RCCL errors (fatal), 0 = epoch end only
    write_grad: bool = False
    verbose: bool = True
    trace_phases: bool = False
    toy_mlp_steps: int = 0
    deterministic: bool = True  # MIOpen's deterministic solver while the run lasts (engine.setup)


_FIELDS = {f.name: f for f in dataclasses.fields(TrainConfig)}
_HINTS = typing.get_type_hints(TrainConfig)


def _check_type(name: str, value: Any):
    hint = _HINTS[name]
    optional = typing.get_origin(hint) is typing.Union and type(None) in typing.get_args(hint)
    base = [a for a in typing.get_args(hint) if a is not type(None)][0] if optional else hint
    if value is None:
        if optional:
            return None
        raise ConfigError(f"config[{name!r}] must not be None")
    if base is bool:
        if isinstance(value, bool) or value in (0, 1):
            return bool(value)
    elif base is int:
        if isinstance(value, int) and not isinstance(value, bool):
            return value
        if isinstance(value, float) and value.is_integer():
            return int(value)
    elif base is float:
        if isinstance(value, (int, float)) and not isinstance(value, bool):
            return float(value)
    elif base is str:
        if isinstance(value, str):
            return value
    raise ConfigError(f"config[{name!r}] = {value!r}: expected {base.__name__}{' or None' if optional else ''}")


def validate_config(config: Dict[str, Any], strict: bool = True) -> Dict[str, Any]:
    """Type-check ``config`` in place against :class:`TrainConfig` and fill defaults.

    ``strict``: unknown keys raise (set False to only warn via the returned dict's
    ``_unknown_keys``).  Returns the same dict object (the workloads mutate it)."""
    unknown = sorted(k for k in config if k not in _FIELDS and not k.startswith("_"))
    if unknown and strict:
        raise ConfigError(f"unknown config keys {unknown}; known: {sorted(_FIELDS)}")
    for name, f in _FIELDS.items():
        if name not in config:
            config[name] = f.default
        else:
            config[name] = _check_type(name, config[name])
    c = config
    for key, allowed in (("grad_sync", GRAD_SYNCS), ("task", TASKS), ("graph_mode", GRAPH_MODES), ("link", LINKS),
                         ("distributed_backend", BACKENDS)):
        if c[key] not in allowed:
            raise ConfigError(f"config[{key!r}] = {c[key]!r}; allowed: {list(allowed)}")
    if c["n_workers"] < 1 or not 0 <= c["rank"] < c["n_workers"]:
        raise ConfigError(f"rank {c['rank']} / n_workers {c['n_workers']}: need 0 <= rank < n_workers")
    if not 1 <= c["reducer_rank"] <= 64:
        raise ConfigError("reducer_rank must be in [1, 64] (csrc kMaxRank)")
    if c["learning_rate"] <= 0 or not 0 <= c["momentum"] < 1:
        raise ConfigError("learning_rate > 0 and 0 <= momentum < 1 required")
    if c["global_batch"] is not None and c["global_batch"] < c["n_workers"]:
        raise ConfigError(f"global_batch {c['global_batch']} < n_workers {c['n_workers']}: empty per-rank batch")
    if c["emulate_world"] is not None and c["emulate_world"] < 1:
        raise ConfigError("emulate_world must be >= 1")
    if c["bucket_mb"] is not None and c["bucket_mb"] <= 0:
        raise ConfigError("bucket_mb must be > 0")
    if c["psgd_groups"] is not None and c["psgd_groups"] < 1:
        raise ConfigError("psgd_groups must be >= 1")
    if c["graph_mode"] in ("full", "piecewise") and c["grad_sync"] == "powersgd" and not c["reuse_query"]:
        raise ConfigError("graph capture needs reuse_query=True (the per-step query re-draw is host-side)")
    if c["log_every"] < 1 or c["training_epochs"] < 0 or c["timeout_s"] <= 0:
        raise ConfigError("log_every >= 1, training_epochs >= 0, timeout_s > 0 required")
    if unknown:
        config["_unknown_keys"] = unknown
    return config
