"""Multi-rank semantics on CPU with gloo: world sizes 2 and 4.

Checks, against the fp64 oracle of §2.9:
  * Q (warm start) is identical on every rank; the decompressed output is identical;
  * EF identity mem = M - out per rank; <=1-D tensors are exact means, their mem stays 0;
  * bits equal the analytic formula;
  * after k training steps every replica holds bitwise-identical parameters, for the
    fused PowerSGD optimizer, the eager reference loop and the bucketed dense DP;
  * the fused optimizer (torch path) reproduces the reference loop exactly;
  * the bucketed dense DP reproduces the reference's per-parameter all-reduce + SGD;
  * the replica checker catches an injected silent corruption.
"""
import os

import pytest
import torch

from network_distributed_pytorch_amd.utils.launcher import spawn

from . import dist_helpers as H
from .oracle import powersgd_round, reference_bits


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("R", [1, 3])
def test_reducer_multirank_matches_oracle(tmp_path, world, R):
    spawn(H.reducer_rank_body, world, args=(str(tmp_path), R))
    data = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    shapes = [m.shape for m in data[0]["Ms"]]
    for call in range(2):
        recs = [d["rec"][call] for d in data]
        # identical Q / outs on every rank
        for r in range(1, world):
            assert torch.equal(recs[r]["q"], recs[0]["q"])
            for a, b in zip(recs[r]["outs"], recs[0]["outs"]):
                assert torch.equal(a, b)
        assert all(rc["bits"] == reference_bits(shapes, R) for rc in recs)
    # oracle for the first call: Q as drawn by the reducer is reconstructed from call-0 state
    # (the oracle consumes Q_init; the reducer returns the averaged new Q)
    Ms_per_rank = [d["Ms"] for d in data]
    # second call uses the warm-started Q from call 0 -> check via the oracle
    q_prev = data[0]["rec"][0]["q"]
    hi = [i for i, s in enumerate(shapes) if len(s) > 1]
    Qs, off = [], 0
    for i in hi:
        n = shapes[i][0]
        m = int(torch.Size(shapes[i]).numel()) // n
        r = min(n, m, R)
        Qs.append(q_prev[off: off + m * r].view(m, r))
        off += m * r
    # call 1 inputs are the same Ms (the reducer is stateless in M), so:
    outs, mems, newQ = powersgd_round(Ms_per_rank, Qs, R)
    rec1 = [d["rec"][1] for d in data]
    for i, ref in enumerate(outs):
        got = rec1[0]["outs"][i].double()
        assert torch.allclose(got, ref, atol=1e-5 * (ref.abs().max().item() + 1e-6), rtol=1e-4), i
    for r in range(world):
        for i in range(len(shapes)):
            if mems[r][i] is None:
                assert torch.count_nonzero(rec1[r]["mems"][i]) == 0
            else:
                M = Ms_per_rank[r][i]
                assert torch.equal(rec1[r]["mems"][i], M - rec1[r]["outs"][i])


@pytest.mark.parametrize("world", [2])
def test_training_replicas_identical_and_fused_equals_reference(tmp_path, world):
    for kind in ("powersgd", "powersgd-ref", "dense", "dense-ref"):
        spawn(H.train_rank_body, world, args=(str(tmp_path), kind, 4, False))
    res = {k: [torch.load(os.path.join(tmp_path, f"{k}_rank{r}.pt"), weights_only=True) for r in range(world)]
           for k in ("powersgd", "powersgd-ref", "dense", "dense-ref")}
    for k, rs in res.items():
        for r in range(1, world):
            for a, b in zip(rs[r]["params"], rs[0]["params"]):
                assert torch.equal(a, b), f"{k}: replicas diverged"
    # fused optimizer (torch path) == reference loop
    for a, b in zip(res["powersgd"][0]["params"], res["powersgd-ref"][0]["params"]):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5)
    # bucketed dense DP == reference per-parameter all-reduce + torch.optim.SGD
    for a, b in zip(res["dense"][0]["params"], res["dense-ref"][0]["params"]):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5)


def test_replica_checker_catches_corruption(tmp_path):
    spawn(H.checker_rank_body, 2, args=(str(tmp_path),))
    r0 = torch.load(os.path.join(tmp_path, "chk0.pt"), weights_only=True)
    r1 = torch.load(os.path.join(tmp_path, "chk1.pt"), weights_only=True)
    assert r1["fired"]
    assert r0["caught"] is not None and r0["caught"] == r1["caught"]


@pytest.mark.parametrize("kind", ["powersgd", "dense"])
def test_forced_collectives_rehearsal_is_identity(tmp_path, kind):
    """NDP_FORCE_COLLECTIVES=1 (the one-GPU rehearsal of the N>1 path) issues the
    collectives in a 1-rank group; results equal the skipped-collective run."""
    for force in (False, True):
        spawn(H.forced_rank_body, 1, args=(str(tmp_path), kind, force))
    meta = {f: torch.load(os.path.join(tmp_path, f"{kind}_f{f}_meta.pt"), weights_only=True) for f in (0, 1)}
    assert not meta[0]["active"] and meta[0]["calls"] == 0
    assert meta[1]["active"] and meta[1]["calls"] > 0
    a = torch.load(os.path.join(tmp_path, f"{kind}_f0_rank0.pt"), weights_only=True)
    b = torch.load(os.path.join(tmp_path, f"{kind}_f1_rank0.pt"), weights_only=True)
    for x, y in zip(a["params"], b["params"]):
        assert torch.equal(x, y)
