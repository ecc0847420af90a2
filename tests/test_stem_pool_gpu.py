"""ResNet stem tail BN -> ReLU -> MaxPool(3, 2, 1) in one pass (csrc/batchnorm.hip
bn_relu_maxpool, ops/batchnorm.BatchNormAct2d.relu_maxpool): the BN output is never stored and
the backward recomputes its ReLU mask from x.  Checked against fp64 PyTorch, against the
unfused BN + pool kernels, and for bitwise run-to-run repeatability."""
import pytest
import torch
import torch.nn.functional as F

from tests._oracle import assert_fused_no_worse, resnet18_fp64_step

from network_distributed_pytorch_amd import ops
from network_distributed_pytorch_amd.models import build_resnet
from network_distributed_pytorch_amd.ops import batchnorm as bn_mod
from network_distributed_pytorch_amd.ops.batchnorm import BatchNormAct2d
from network_distributed_pytorch_amd.ops.pool import MaxPool2d

pytestmark = pytest.mark.gpu


def _run(bn, pool, x, g, fused):
    bn.zero_grad(set_to_none=True)
    xi = x.clone().requires_grad_(True)
    y = bn.relu_maxpool(xi, pool) if fused else pool(bn(xi, relu=True))
    assert y is not None
    y.backward(g)
    torch.cuda.synchronize()
    return (y.detach().clone(), xi.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone(),
            bn.running_mean.clone(), bn.running_var.clone(), bn.num_batches_tracked.clone())


@pytest.mark.parametrize("N,C,H", [(32, 64, 16), (8, 64, 16), (4, 16, 12)])
def test_bn_relu_maxpool_matches_fp64_and_unfused(device, N, C, H):
    assert ops.native_available()
    torch.manual_seed(N + C + H)
    x = torch.randn(N, C, H, H, device=device) * 1.3 + 0.2
    bn = BatchNormAct2d(C).to(device).train()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    pool = MaxPool2d(3, 2, 1)
    state = {k: v.clone() for k, v in bn.state_dict().items()}
    OH = (H - 1) // 2 + 1
    g = torch.randn(N, C, OH, OH, device=device)
    runs = []
    for fused in (True, True, False):
        bn.load_state_dict(state)
        runs.append(_run(bn, pool, x, g, fused))
    a, b, u = runs
    for p, q in zip(a, b):  # fused: bitwise repeatable
        assert torch.equal(p, q)
    for p, q in zip(a[:4], u[:4]):  # fused vs BN + pool kernels (scale / shift rounding: 1 ulp)
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-5 * (q.abs().max().item() + 1e-6))
    for p, q in zip(a[4:], u[4:]):  # running statistics: the same computation
        assert torch.equal(p, q)
    # fp64 reference
    xd = x.double().requires_grad_(True)
    wd = state["weight"].double().requires_grad_(True)
    bd = state["bias"].double().requires_grad_(True)
    yd = F.max_pool2d(F.relu(F.batch_norm(xd, None, None, wd, bd, True, 0.1, 1e-5)), 3, 2, 1)
    yd.backward(g.double())
    for p, q in zip(a[:4], (yd, xd.grad, wd.grad, bd.grad)):
        scale = q.abs().max().item() + 1e-12
        assert (p.double() - q).abs().max().item() < 1e-4 * scale


def test_resnet18_stem_pool_matches_unfused(device, monkeypatch):
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(0)
    m = build_resnet(18, 1000).to(device)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.rand(64, 3, 32, 32, device=device) * 2 - 1
    y = torch.randint(0, 10, (64,), device=device)
    outs = []
    for on in (False, True, True):
        monkeypatch.setattr(bn_mod, "STEM_POOL", on)
        m.load_state_dict(state)
        m.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x), y)
        loss.backward()
        torch.cuda.synchronize()
        outs.append((loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters()},
                     {k: v.clone() for k, v in m.state_dict().items()}))
    (l0, g0, s0), (l1, g1, s1), (l2, g2, s2) = outs
    assert torch.equal(l1, l2) and all(torch.equal(g1[n], g2[n]) for n in g1)
    assert abs(l0.item() - l1.item()) < 1e-5 * max(1.0, abs(l0.item()))
    # the arms' statistics differ in summation order only: both judged against the exact step
    # (tests/_oracle.py: the arms' mutual distance is chaotic rounding amplification)
    assert_fused_no_worse(g1, g0, resnet18_fp64_step(state, x, y)[1])
    for k in s0:
        if s0[k].dtype.is_floating_point:
            assert torch.allclose(s0[k], s1[k], rtol=1e-5, atol=1e-6), k


@pytest.mark.parametrize("N", [64, 512, 6])
def test_stem_pool_bwd_one_pass_is_bitwise(device, monkeypatch, N):
    """The stem backward from the pooled gradient in one pass (statistics-only pool backward +
    csrc/batchnorm.hip stem_pool_bwd_apply_kernel) == pool backward + BN backward apply, bitwise."""
    torch.manual_seed(0)
    C, H = 64, 16
    x = torch.randn(N, C, H, H, device=device)
    pool = MaxPool2d(3, 2, 1)
    outs = []
    for on in (False, True):
        monkeypatch.setattr(bn_mod, "_STEM_BWD", on)
        torch.manual_seed(1)
        bn = BatchNormAct2d(C).to(device)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
        g = torch.randn(N, C, H // 2, H // 2, device=device, generator=torch.Generator(device=device).manual_seed(2))
        outs.append(_run(bn, pool, x, g, True))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
