"""Split-K slab hand-off (ops/slablink.py): a direct conv leaves its partial slabs for the
fused BN kernel next to it (forward: conv -> BN; backward: conv2 grad-x -> BN1).  The BN
kernel sums them in the conv_slab_sum order, so the step must be BITWISE equal to the
path with the separate sum launches, at every strong-scaling per-GPU batch."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd import ops
from network_distributed_pytorch_amd.models import build_resnet
from network_distributed_pytorch_amd.models import resnet as resnet_mod
from network_distributed_pytorch_amd.ops._ext import ext
from network_distributed_pytorch_amd.ops.batchnorm import BatchNormAct2d
from network_distributed_pytorch_amd.ops.slablink import SlabLink

pytestmark = pytest.mark.gpu


def _step(model, x, y):
    model.zero_grad(set_to_none=True)
    loss = F.cross_entropy(model(x), y)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("batch", [64, 128, 256])
def test_resnet18_slab_links_bitwise(device, batch, monkeypatch):
    """Same model, same state: links off / on / off — on must equal off bitwise (and off
    must equal off: the step itself is deterministic)."""
    assert ops.native_available()
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    # the slab hand-off alone (the epilogue BN statistics change the summation order:
    # tests/test_conv_bnstats_gpu.py)
    from network_distributed_pytorch_amd.ops import conv as conv_mod
    monkeypatch.setattr(conv_mod, "CONV_BN_STATS", False)
    monkeypatch.setattr(conv_mod, "_STATS", {})
    from network_distributed_pytorch_amd.ops import batchnorm as bn_mod
    monkeypatch.setattr(bn_mod, "_BWD_STATS", False)
    torch.manual_seed(0)
    m = build_resnet(18, 1000).to(device)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.rand(batch, 3, 32, 32, device=device) * 2 - 1
    y = torch.randint(0, 10, (batch,), device=device)
    runs = []
    for on in (False, True, False):
        monkeypatch.setattr(resnet_mod, "SLAB_LINKS", on)
        m.load_state_dict(state)
        loss, grads = _step(m, x, y)
        runs.append((loss, grads, {k: v.clone() for k, v in m.state_dict().items()}))
    (l0, g0, s0), (l1, g1, s1), (l2, g2, s2) = runs
    assert torch.equal(l0, l2) and torch.equal(l0, l1)
    for n in g0:
        assert torch.equal(g0[n], g2[n]), f"step not deterministic: {n}"
    bad = [n for n in g0 if not torch.equal(g1[n], g0[n])]
    assert not bad, f"slab links change gradients of {bad}"
    for k in s0:
        assert torch.equal(s1[k], s0[k]), k


@pytest.mark.parametrize("fused_small", [True, False])
def test_bn_consumes_conv_slabs(device, fused_small):
    """A BN given slabs sums them (fused kernel) or finishes the sum first (fallback path)."""
    torch.manual_seed(3)
    N, C, H, W, ks = 64, 64, 8, 8, 4
    parts = torch.randn(ks, N, C, H, W, device=device)
    full = parts[0].clone()
    for z in range(1, ks):
        full += parts[z]
    a = BatchNormAct2d(C).to(device)
    b = BatchNormAct2d(C).to(device)
    a.fused_small = b.fused_small = fused_small
    xa = torch.empty(N, C, H, W, device=device).requires_grad_(True)
    link = SlabLink()
    link.put_fwd(parts.reshape(-1), ks)
    ya = a(xa, relu=True, slab_in=link)
    xb = full.clone().requires_grad_(True)
    yb = b(xb, relu=True)
    torch.testing.assert_close(ya, yb, rtol=1e-6, atol=1e-6)
    assert torch.equal(xa.detach(), full)  # the BN wrote the conv output it saved
    assert link.fwd is None


def test_slab_sum_matches_sequential(device):
    torch.manual_seed(4)
    parts = torch.randn(8, 4096, device=device)
    out = torch.empty(4096, device=device)
    ext().slab_sum(parts.reshape(-1), out, 8)
    ref = parts[0].clone()
    for z in range(1, 8):
        ref += parts[z]
    assert torch.equal(out, ref)


@pytest.mark.parametrize("batch", [64, 512])
def test_resnet18_branch_links_match(device, batch, monkeypatch):
    """Downsample blocks: conv1 / downsample grad-x accumulated in place (BranchLink) equals
    autograd's add of the two (GEMM beta = 1 may pick another library solution: tolerance)."""
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(1)
    m = build_resnet(18, 1000).to(device)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.rand(batch, 3, 32, 32, device=device) * 2 - 1
    y = torch.randint(0, 10, (batch,), device=device)
    runs = []
    for on in (True, False):
        monkeypatch.setattr(resnet_mod, "BRANCH_LINKS", on)
        m.load_state_dict(state)
        runs.append(_step(m, x, y))
    (l1, g1), (l0, g0) = runs
    assert torch.equal(l1, l0)
    for n in g0:
        scale = g0[n].abs().max().item() + 1e-12
        torch.testing.assert_close(g1[n], g0[n], rtol=1e-4, atol=1e-5 * scale, msg=n)


@pytest.mark.parametrize("batch", [64, 512])
def test_direct_branch_link_bitwise(device, batch, monkeypatch):
    """layer2's entry block on the direct kernels: conv1's (3x3/2) grad-x kernel adds the 1x1/2
    downsample's grad-x in its epilogue / split-K sum (BranchLink, deferred first member) —
    bitwise equal to autograd's add of the two (the same fp32 sum, addend added last)."""
    from network_distributed_pytorch_amd.models.resnet import BasicBlock, conv1x1

    torch.manual_seed(2)
    ds = torch.nn.Sequential(conv1x1(64, 128, 2), BatchNormAct2d(128))
    blk = BasicBlock(64, 128, 2, ds, norm=BatchNormAct2d).to(device).train()
    state = {k: v.clone() for k, v in blk.state_dict().items()}
    x0 = torch.randn(batch, 64, 8, 8, device=device)
    g = torch.randn(batch, 128, 4, 4, device=device)
    runs = []
    for on in (False, True, True):
        monkeypatch.setattr(resnet_mod, "BRANCH_LINKS", on)
        blk.load_state_dict(state)
        blk.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        blk(x).backward(g)
        torch.cuda.synchronize()
        runs.append((x.grad.clone(), {n: p.grad.clone() for n, p in blk.named_parameters()}))
    for xg, pg in runs[1:]:
        assert torch.equal(xg, runs[0][0])
        for n in pg:
            assert torch.equal(pg[n], runs[0][1][n]), n
