"""Runtime pieces on CPU: comm accounting + link model, plan builder coverage, checkpoint
resume equivalence, the training engine (all tasks), the orthogonalizer and Q seeding."""
import json
import os

import numpy as np
import pytest
import torch

from network_distributed_pytorch_amd import engine, ops
from network_distributed_pytorch_amd.models import build_model
from network_distributed_pytorch_amd.parallel.comm import LINK_PRESETS, Communicator, LinkModel, n_bits
from network_distributed_pytorch_amd.parallel.powersgd import PowerSGDOptimizer, PowerSGDReducer, orthogonalize, plan_layout
from network_distributed_pytorch_amd.utils.checkpoint import load_checkpoint, save_checkpoint

from .oracle import mgs, powersgd_round


def test_n_bits_and_link_model():
    assert n_bits(torch.zeros(10)) == 320
    lm = LinkModel(10e9, alpha_s=0.0)
    assert lm.wire_bytes(1000, 8) == pytest.approx(1750)
    assert lm.seconds(1000, 8) == pytest.approx(8 * 1750 / 10e9)
    assert lm.seconds(1000, 1) == 0.0
    assert set(LINK_PRESETS) == {"1g", "10g", "100g"}


def test_communicator_world1_accounting():
    c = Communicator(link=LINK_PRESETS["1g"])
    t = torch.ones(100)
    assert c.all_reduce(t) is None and torch.equal(t, torch.ones(100))
    h = c.all_reduce(t, async_op=True)
    assert h.wait()
    assert c.stats.calls == 2 and c.stats.payload_bytes == 800 and c.stats.wire_bytes == 0.0


def test_orthogonalize_cpu_matches_oracle():
    P = torch.randn(50, 6)
    ref = mgs(P.double())
    out = orthogonalize(P.clone())
    assert torch.allclose(out.double(), ref, atol=1e-5)


def test_q_seed_stream_matches_reference_scheme():
    """Q is drawn exactly like reducer.py:36-38 (manual_seed(rng.randint(1e9)); randn)."""
    red = PowerSGDReducer(714, "cpu", 0, True, rank=2)
    M = [torch.randn(6, 4), torch.randn(3, 5)]
    red.reduce(M, [torch.zeros_like(m) for m in M], [torch.zeros_like(m) for m in M])
    rng = np.random.RandomState(714)
    torch.manual_seed(int(rng.randint(1_000_000_000)))
    q0 = torch.randn(4, 2)
    torch.manual_seed(int(rng.randint(1_000_000_000)))
    q1 = torch.randn(5, 2)
    # first-call query reproduced through the oracle
    outs, _, newQ = powersgd_round([M], [q0, q1], 2)
    assert torch.allclose(red._buf.q_warm[:8].view(4, 2).double(), newQ[0], atol=1e-5)


def test_reducer_world1_matches_oracle():
    torch.manual_seed(0)
    shapes = [(8, 3, 3, 3), (8,), (10, 20), (5, 5)]
    Ms = [torch.randn(s) for s in shapes]
    red = PowerSGDReducer(3, "cpu", 0, True, rank=3)
    outs = [torch.zeros(s) for s in shapes]
    mems = [torch.zeros(s) for s in shapes]
    red.reduce(Ms, outs, mems)
    q = red._buf.q_warm.clone()
    red.reduce(Ms, outs, mems)
    ranks, _, q_offs, _, _ = plan_layout([(8, 27), (10, 20), (5, 5)], 3)
    Qs = [q[o: o + m * r].view(m, r) for o, m, r in zip(q_offs, (27, 20, 5), ranks)]
    ref_out, ref_mem, _ = powersgd_round([Ms], Qs, 3)
    for o, r in zip(outs, ref_out):
        assert torch.allclose(o.double(), r, atol=1e-5)
    assert torch.count_nonzero(mems[1]) == 0
    assert torch.equal(mems[0], Ms[0] - outs[0])


@pytest.mark.skipif(not ops.native_available(), reason="extension not built")
@pytest.mark.parametrize("rank", [16, 32])
def test_native_plan_covers_every_element(rank):
    X = ops.ext()
    shapes = [(64, 147), (1000, 512), (7, 5), (30522, 8), (300, 1030)]
    d = X.build_plan(shapes, rank)
    ranks, p_offs, q_offs, pt, qt = plan_layout(shapes, rank)
    assert d["ranks"] == ranks and d["p_offs"] == p_offs and d["q_offs"] == q_offs
    assert d["p_total"] == pt and d["q_total"] == qt
    P = np.frombuffer(d["p_items"].numpy().tobytes(), dtype=np.int32).reshape(-1, 8)
    Q = np.frombuffer(d["q_items"].numpy().tobytes(), dtype=np.int32).reshape(-1, 8)
    U = np.frombuffer(d["u_items"].numpy().tobytes(), dtype=np.int32).reshape(-1, 4)
    wide = max(ranks) <= 16  # plan.cpp: 16 x 1024 P items and 16 x 256 update tiles up to rank 16
    pr, pk = (16, 1024) if wide else (64, 256)
    for i, (n, m) in enumerate(shapes):
        cov = np.zeros((n, m), np.int32)
        for mat, row0, k0, k1, chunk, *_ in P[P[:, 0] == i]:
            cov[row0: row0 + pr, k0:k1] += 1
            assert chunk == k0 // pk
        assert (cov == 1).all()
        cov[:] = 0
        for mat, col0, row0, row1, chunk, *_ in Q[Q[:, 0] == i]:
            assert row1 - row0 <= 256
            cov[row0:row1, col0: col0 + 256] += 1
        assert (cov == 1).all()
        cov[:] = 0
        ur, uc = (16, 256) if wide else (64, 64)
        for mat, row0, col0, _ in U[U[:, 0] == i]:
            cov[row0: row0 + ur, col0: col0 + uc] += 1
        assert (cov == 1).all()
    assert d["q_chunks"][3] <= 128  # the tall embedding's Q slabs are capped


def _tiny_run(steps, ckpt=None, resume=None):
    torch.manual_seed(0)
    model = build_model("resnet18", 10)
    opt = PowerSGDOptimizer(model.parameters(), lr=0.05, rank=2)
    if resume:
        load_checkpoint(resume, model, opt)
    g = torch.Generator().manual_seed(5 + (opt.step_count if resume else 0))
    for s in range(steps):
        x = torch.randn(4, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (4,), generator=g)
        opt.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        opt.step()
        if ckpt and s == 1:
            save_checkpoint(ckpt, model, opt, epoch=0, step=opt.step_count, rank=0)
            g = torch.Generator().manual_seed(5 + opt.step_count)
    return [p.detach().clone() for p in model.parameters()], opt


def test_checkpoint_resume_is_exact(tmp_path):
    ck = str(tmp_path / "ck.pt")
    full, _ = _tiny_run(4, ckpt=ck)
    resumed, opt = _tiny_run(2, resume=ck)
    assert opt.step_count == 4
    for a, b in zip(full, resumed):
        assert torch.equal(a, b)


@pytest.mark.parametrize("task,grad_sync,extra", [
    ("cifar", "powersgd", {"model": "resnet18", "dataset_size": 256, "global_batch": 64}),
    ("cifar", "dense", {"model": "resnet18", "dataset_size": 256, "global_batch": 64}),
    ("cifar", "powersgd-api", {"model": "resnet18", "dataset_size": 128, "global_batch": 64}),
    ("mlp", "dense-ref", {"dataset_size": 512, "global_batch": 64}),
    ("imdb", "powersgd", {"dataset_size": 40, "global_batch": 8, "seq_len": 32, "reducer_rank": 8}),
])
def test_engine_tasks(tmp_path, task, grad_sync, extra):
    cfg = engine.default_config(task=task, grad_sync=grad_sync, training_epochs=2, max_steps_per_epoch=2,
                                verbose=False, log_file=str(tmp_path / "log.jsonl"),
                                checkpoint_dir=str(tmp_path / "ck"), **extra)
    out = engine.run_task(cfg)
    assert len(out["epoch_losses"]) == 2 and all(np.isfinite(out["epoch_losses"]))
    assert os.path.exists(tmp_path / "ck" / "last.pt")
    kinds = [json.loads(ln)["kind"] for ln in (tmp_path / "log.jsonl").read_text().splitlines()]
    assert kinds.count("step") == 4 and kinds.count("epoch") == 2 and kinds[-1] == "summary"


def test_batchnorm_act_cpu_matches_torch():
    from network_distributed_pytorch_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(0)
    ref = torch.nn.BatchNorm2d(6)
    ours = BatchNormAct2d(6)
    ours.load_state_dict(ref.state_dict())
    assert list(ours.state_dict()) == list(ref.state_dict())
    x = torch.randn(4, 6, 5, 5)
    r = torch.randn(4, 6, 5, 5)
    y = ours(x, residual=r, relu=True)
    y_ref = torch.relu(ref(x) + r)
    assert torch.allclose(y, y_ref, atol=1e-6)
    assert torch.equal(ours.running_mean, ref.running_mean) and int(ours.num_batches_tracked) == 1


def test_engine_ragged_last_batch_and_reference_mean(tmp_path):
    """Every sample is trained, the ragged last batch too, and the epoch loss is
    epoch_loss / ceil(len / bsz) like the reference (ddp_powersgd_guide_cifar10/ddp_init.py:118,183)."""
    cfg = engine.default_config(task="mlp", grad_sync="dense-ref", training_epochs=1, dataset_size=100,
                                global_batch=32, verbose=False, log_file=str(tmp_path / "log.jsonl"))
    out = engine.run_task(cfg)
    recs = [json.loads(ln) for ln in (tmp_path / "log.jsonl").read_text().splitlines()]
    ep = [r for r in recs if r["kind"] == "epoch"][0]
    steps = [r for r in recs if r["kind"] == "step"]
    assert ep["steps"] == ep["num_batches"] == 4  # 32 + 32 + 32 + 4
    assert len(steps) == 4 and out["steps"] == 4
    assert out["samples"] == 100  # the ragged batch counts its 4 samples, not 32
    assert abs(ep["mean_loss"] - sum(r["loss"] for r in steps) / 4) < 1e-5


def test_checkpoint_rank_file_from_another_save_is_rejected(tmp_path):
    from network_distributed_pytorch_amd.utils.checkpoint import (CheckpointMismatch, load_checkpoint,
                                                                  save_checkpoint)
    model = torch.nn.Linear(4, 3)
    path = str(tmp_path / "ck.pt")
    save_checkpoint(path, model, epoch=1, step=10, rank=0, world=2)
    save_checkpoint(path, model, epoch=1, step=10, rank=1, world=2)
    info = load_checkpoint(path, model, rank=1, world=2)
    assert info["step"] == 10
    save_checkpoint(path, model, epoch=2, step=20, rank=0, world=2)  # rank 1 "crashed" before its write
    with pytest.raises(CheckpointMismatch, match="different saves"):
        load_checkpoint(path, model, rank=1, world=2)
