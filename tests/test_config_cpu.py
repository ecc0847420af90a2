"""Typed config schema (utils/config.py): every workload's dict validates; bad values fail early."""
import importlib

import pytest

from network_distributed_pytorch_amd import engine
from network_distributed_pytorch_amd.utils.config import ConfigError, TrainConfig, validate_config

WORKLOADS = ["ddp_guide", "ddp_guide_cifar10", "ddp_powersgd_guide_cifar10", "ddp_powersgd_distillBERT_IMDb"]


@pytest.mark.parametrize("name", WORKLOADS)
def test_workload_configs_validate_strictly(name):
    mod = importlib.import_module(f"network_distributed_pytorch_amd.workloads.{name}.ddp_init")
    cfg = dict(mod.config)
    cfg["n_workers"] = max(1, cfg.get("n_workers", 1))
    out = validate_config(cfg, strict=True)
    assert "_unknown_keys" not in out
    assert out["grad_sync"] in ("powersgd", "dense")


def test_engine_default_config_matches_schema():
    cfg = engine.default_config()
    assert set(cfg) <= {f for f in TrainConfig.__dataclass_fields__}
    validate_config(cfg, strict=True)


@pytest.mark.parametrize("bad", [
    {"grad_sync": "powersdg"}, {"reducer_rank": 0}, {"reducer_rank": 65}, {"link": "5g"}, {"rank": 2, "n_workers": 2},
    {"learning_rate": -1.0}, {"momentum": 1.0}, {"graph_mode": "full", "reuse_query": False},
    {"bucket_mb": 0}, {"psgd_groups": 0}, {"training_epochs": "3"}, {"global_batch": 1, "n_workers": 2},
])
def test_bad_values_fail_early(bad):
    cfg = engine.default_config(**bad)
    with pytest.raises(ConfigError):
        validate_config(cfg)


def test_unknown_keys_strict_and_lenient():
    with pytest.raises(ConfigError, match="reducer_rnak"):
        validate_config(engine.default_config(reducer_rnak=4))
    out = validate_config(engine.default_config(reducer_rnak=4), strict=False)
    assert out["_unknown_keys"] == ["reducer_rnak"]


def test_coercion_and_defaults():
    out = validate_config({"learning_rate": 1, "overlap": 1, "training_epochs": 2.0})
    assert out["learning_rate"] == 1.0 and isinstance(out["learning_rate"], float)
    assert out["overlap"] is True and out["training_epochs"] == 2
    assert out["reducer_rank"] == 4 and out["graph_mode"] == "auto"
