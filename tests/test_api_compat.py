"""API compatibility with the reference + the BASELINE bytes/step anchors."""
import importlib

import pytest
import torch

from network_distributed_pytorch_amd.models import build_model
from network_distributed_pytorch_amd.parallel.powersgd import powersgd_bytes_per_step
from network_distributed_pytorch_amd.parallel.tensor_buffer import TensorBuffer
from network_distributed_pytorch_amd.utils.partition_helper import DataPartitioner, Partition
from network_distributed_pytorch_amd.workloads import _cli

W = "network_distributed_pytorch_amd.workloads."
REF_KEYS = {"seed", "rank", "cuda_rank", "n_workers", "distributed_init_file", "output_dir", "distributed_backend"}


@pytest.mark.parametrize("name", ["ddp_guide", "ddp_guide_cifar10", "ddp_powersgd_guide_cifar10",
                                  "ddp_powersgd_distillBERT_IMDb"])
def test_ddp_init_surface(name):
    m = importlib.import_module(W + name + ".ddp_init")
    assert REF_KEYS <= set(m.config)
    for fn in ("setup", "run_task", "cleanup"):
        assert callable(getattr(m, fn))
    if name != "ddp_guide":
        for k in ("learning_rate", "momentum", "nesterov", "training_epochs", "batch_size"):
            assert k in m.config
    if "powersgd" in name:
        assert "reducer_rank" in m.config


def test_reference_defaults():
    c = importlib.import_module(W + "ddp_powersgd_guide_cifar10.ddp_init").config
    assert (c["seed"], c["learning_rate"], c["momentum"], c["reducer_rank"], c["global_batch"]) == (714, 1e-3, 0.9, 4, 512)
    assert c["model"] == "resnet152"
    b = importlib.import_module(W + "ddp_powersgd_distillBERT_IMDb.ddp_init").config
    assert (b["learning_rate"], b["reducer_rank"], b["training_epochs"], b["batch_size"]) == (5e-5, 16, 5, 16)
    d = importlib.import_module(W + "ddp_guide_cifar10.ddp_init").config
    assert (d["model"], d["global_batch"], d["learning_rate"]) == ("resnet50", 256, 1e-3)


def test_reference_module_names():
    red = importlib.import_module(W + "ddp_powersgd_guide_cifar10.reducer")
    assert hasattr(red, "PowerSGDReducer") and hasattr(red, "orthogonalize") and hasattr(red, "n_bits")
    tb = importlib.import_module(W + "ddp_powersgd_distillBERT_IMDb.tensor_buffer")
    assert hasattr(tb, "TensorBuffer")
    ph = importlib.import_module(W + "ddp_guide_cifar10.partition_helper")
    assert hasattr(ph, "DataPartitioner") and hasattr(ph, "Partition")


def test_run_script_flags():
    p = _cli.build_parser(4)
    a = p.parse_args(["-rank", "1", "-cuda", "3", "-world_size", "8", "-init_method", "tcp://127.0.0.1:7392"])
    assert (a.rank, a.cuda, a.world_size, a.init_method) == (1, 3, 8, "tcp://127.0.0.1:7392")
    assert p.parse_args([]).world_size == 4  # reference run_script hard-codes n_workers = 4


def test_tensor_buffer_api_cpu():
    ts = [torch.randn(3), torch.randn(2, 2), torch.randn(5)]
    tb = TensorBuffer(ts)
    assert len(tb) == 3 and tb.nelement() == 12 and tb.element_size() == 4 and tb.bits() == 384
    assert torch.equal(tb[1], ts[1])
    tb.buffer.mul_(2)
    out = [torch.empty_like(t) for t in ts]
    tb.unpack(out)
    assert all(torch.equal(o, 2 * t) for o, t in zip(out, ts))
    tb.pack()
    assert torch.equal(tb.buffer, torch.cat([t.view(-1) for t in ts]))
    assert len(tb.all_gather()) == 1  # world-size-1 fallback
    empty = TensorBuffer([])  # quirk Q6: the reference crashes in torch.cat
    assert empty.nelement() == 0


def test_partitioner_semantics():
    import random
    data = list(range(103))
    dp = DataPartitioner(data, [0.25] * 4)
    order = list(range(103))
    random.Random(1234).shuffle(order)
    parts = [dp.use(i) for i in range(4)]
    assert all(len(p) == 25 for p in parts)  # int(0.25 * 103) = 25, remainder dropped
    assert parts[0].index == order[:25] and parts[3].index == order[75:100]
    flat = [i for p in parts for i in p.index]
    assert len(set(flat)) == 100
    assert parts[2][0] == data[order[50]]
    assert isinstance(DataPartitioner.shard(data, 1, 4), Partition)


# ---- BASELINE.md bytes/step anchors (reference accounting) ----------------
@pytest.mark.parametrize("model,classes,rank,total,dense", [
    ("resnet18", 1000, 4, 641360, 46758048),
    ("resnet18", 10, 4, 621560, 44726568),
    ("resnet152", 1000, 4, 4550992, None),
    ("resnet50", 1000, 4, None, 102228128),
])
def test_bytes_per_step_anchors_resnet(model, classes, rank, total, dense):
    b = powersgd_bytes_per_step(list(build_model(model, classes).parameters()), rank)
    if total is not None:
        assert b["total"] == total
    if dense is not None:
        assert b["dense"] == dense


@pytest.mark.parametrize("rank,total", [(4, 2127800), (8, 4000600), (16, 7746200)])
def test_bytes_per_step_anchors_distilbert(rank, total):
    ps = list(build_model("distilbert").parameters())
    b = powersgd_bytes_per_step(ps, rank)
    assert b["total"] == total
    assert b["dense"] == 267820040
