"""Fused BN(+residual)(+ReLU) gfx950 kernels vs torch.nn.BatchNorm2d (fp32 reference)."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd import ops
from network_distributed_pytorch_amd.models import build_resnet
from network_distributed_pytorch_amd.ops.batchnorm import BatchNormAct2d

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(512, 64, 8, 8), (64, 128, 4, 4), (32, 512, 1, 1), (16, 24, 7, 7),
                                   (8, 64, 16, 16), (3, 5, 2, 3), (512, 256, 2, 2), (40, 96, 2, 1),
                                   (7, 40, 2, 4), (8192, 64, 1, 1), (33, 300, 1, 1), (17, 70, 2, 2),
                                   (64, 64, 8, 8), (128, 64, 8, 8), (100, 32, 8, 8)])
@pytest.mark.parametrize("res,relu", [(False, False), (False, True), (True, True)])
def test_bn_act_train_fwd_bwd(device, shape, res, relu):
    assert ops.native_available()
    torch.manual_seed(0)
    C = shape[1]
    ref = torch.nn.BatchNorm2d(C).to(device)
    ours = BatchNormAct2d(C).to(device)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.5, 0.5)
    ours.load_state_dict(ref.state_dict())
    x = (torch.randn(shape, device=device) * 2 + 0.3).requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    r = torch.randn(shape, device=device, requires_grad=True) if res else None
    r2 = r.detach().clone().requires_grad_(True) if res else None
    y_ref = ref(x)
    if res:
        y_ref = y_ref + r
    if relu:
        y_ref = F.relu(y_ref)
    y = ours(x2, residual=r2, relu=relu)
    assert torch.allclose(y, y_ref, atol=2e-5, rtol=1e-4), (y - y_ref).abs().max()
    g = torch.randn(shape, device=device)
    y_ref.backward(g)
    y.backward(g)
    assert torch.allclose(x2.grad, x.grad, atol=5e-5, rtol=1e-3), (x2.grad - x.grad).abs().max()
    assert torch.allclose(ours.weight.grad, ref.weight.grad, atol=1e-3, rtol=1e-4)
    assert torch.allclose(ours.bias.grad, ref.bias.grad, atol=1e-3, rtol=1e-4)
    if res:
        assert torch.allclose(r2.grad, r.grad, atol=1e-6)
    assert torch.allclose(ours.running_mean, ref.running_mean, atol=1e-6)
    assert torch.allclose(ours.running_var, ref.running_var, atol=1e-5, rtol=1e-5)
    assert int(ours.num_batches_tracked) == int(ref.num_batches_tracked) == 1
    # eval mode uses running statistics
    ref.eval()
    ours.eval()
    with torch.no_grad():
        ye = ours(x, relu=relu)
        yr = F.relu(ref(x)) if relu else ref(x)
    assert torch.allclose(ye, yr, atol=2e-5, rtol=1e-4)


@pytest.mark.parametrize("n", [512, 64, 100])  # 64 / 100: the row-split single-launch kernel (8x8 maps)
def test_bn_deterministic(device, n):
    torch.manual_seed(1)
    m = BatchNormAct2d(64).to(device)
    x = torch.randn(n, 64, 8, 8, device=device, requires_grad=True)
    g = torch.randn(n, 64, 8, 8, device=device)
    outs = []
    for _ in range(2):
        x.grad = None
        m.weight.grad = None
        y = m(x, relu=True)
        y.backward(g)
        outs.append((y.detach().clone(), x.grad.clone(), m.weight.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_resnet18_fused_matches_unfused(device):
    torch.manual_seed(0)
    fused = build_resnet(18, 10, fused_bn=True).to(device)
    plain = build_resnet(18, 10, fused_bn=False).to(device)
    plain.load_state_dict(fused.state_dict())
    assert list(fused.state_dict()) == list(plain.state_dict())
    x = torch.randn(64, 3, 32, 32, device=device)
    y = torch.randint(0, 10, (64,), device=device)
    lf = F.cross_entropy(fused(x), y)
    lp = F.cross_entropy(plain(x), y)
    assert torch.allclose(lf, lp, atol=1e-4, rtol=1e-4)
    lf.backward()
    lp.backward()
    for (n, a), b in zip(fused.named_parameters(), plain.parameters()):
        scale = b.grad.abs().max().item() + 1e-8
        assert torch.allclose(a.grad, b.grad, atol=2e-3 * scale, rtol=1e-2), n


@pytest.mark.parametrize("shape", [(512, 512, 1, 1), (512, 256, 2, 2), (40, 96, 2, 1), (3, 20, 1, 1),
                                   (512, 128, 4, 4), (100, 64, 4, 2), (64, 64, 8, 8), (128, 64, 8, 8),
                                   (7, 16, 8, 8)])
def test_bn_single_launch_small_path(device, shape):
    """Single-launch register-resident small-map BN: matches the 3-kernel path and is
    deterministic (run twice, bitwise equal)."""
    torch.manual_seed(2)
    C = shape[1]
    a = BatchNormAct2d(C).to(device)
    b = BatchNormAct2d(C).to(device)
    b.fused_small = False
    b.load_state_dict(a.state_dict())
    x = torch.randn(shape, device=device) * 1.5 + 0.2
    r = torch.randn(shape, device=device)
    g = torch.randn(shape, device=device)
    outs = []
    for m in (a, b, a):
        xx = x.clone().requires_grad_(True)
        rr = r.clone().requires_grad_(True)
        y = m(xx, residual=rr, relu=True)
        y.backward(g)
        outs.append((y.detach(), xx.grad, rr.grad, m.weight.grad.clone(), m.bias.grad.clone()))
        m.weight.grad = None
        m.bias.grad = None
    for t0, t1, t2 in zip(*outs):
        assert torch.equal(t0, t2)              # deterministic
        torch.testing.assert_close(t0, t1, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("shape", [(512, 512, 1, 1), (512, 256, 2, 2), (512, 128, 4, 4), (256, 64, 2, 2)])
def test_bn_single_launch_running_stats(device, shape):
    """Single-launch small-map BN over repeated steps: output and running statistics (written
    once per channel) equal to the statistics + apply path's, num_batches_tracked advanced once
    per call.  (The round-4 row-split variant this test also covered was removed in round 5.)"""
    torch.manual_seed(3)
    C = shape[1]
    a = BatchNormAct2d(C).to(device)
    b = BatchNormAct2d(C).to(device)
    b.fused_small = False
    b.load_state_dict(a.state_dict())
    for it in range(3):
        x = torch.randn(shape, device=device) * (1.0 + it) + 0.3
        ya, yb = a(x, relu=False), b(x, relu=False)
        torch.testing.assert_close(ya, yb, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(a.running_mean, b.running_mean, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(a.running_var, b.running_var, rtol=1e-6, atol=1e-6)
    assert a.num_batches_tracked.item() == b.num_batches_tracked.item() == 3


@pytest.mark.parametrize("shape", [(512, 512, 1, 1), (64, 512, 1, 1), (512, 256, 2, 2), (64, 256, 2, 2),
                                   (512, 128, 4, 4), (64, 128, 4, 4), (40, 96, 2, 1), (3, 20, 1, 1),
                                   (100, 64, 4, 2), (33, 300, 1, 1), (64, 64, 8, 8), (128, 64, 8, 8),
                                   (200, 256, 2, 2)])
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_bn_vec4_vs_fp64(device, shape, res, relu):
    """float4 single-launch small-map BN (csrc/batchnorm.hip bn_small_fused_v4): forward output,
    statistics and every gradient against an fp64 PyTorch reference; bitwise run-to-run."""
    from network_distributed_pytorch_amd.ops._ext import ext
    torch.manual_seed(4)
    C = shape[1]
    m = BatchNormAct2d(C).to(device)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    x = torch.randn(shape, device=device) * 1.7 + 0.4
    r = torch.randn(shape, device=device) if res else None
    g = torch.randn(shape, device=device)
    # fp64 reference
    xd = x.double().cpu().requires_grad_(True)
    rd = r.double().cpu().requires_grad_(True) if res else None
    wd = m.weight.detach().double().cpu().requires_grad_(True)
    bd = m.bias.detach().double().cpu().requires_grad_(True)
    yd = F.batch_norm(xd, None, None, wd, bd, True, 0.0, m.eps)
    if res:
        yd = yd + rd
    if relu:
        yd = F.relu(yd)
    yd.backward(g.double().cpu())
    runs = []
    ext().bn_set_vec4(True)
    try:
        for _ in range(2):
            xx = x.clone().requires_grad_(True)
            rr = r.clone().requires_grad_(True) if res else None
            m.weight.grad = m.bias.grad = None
            y = m(xx, residual=rr, relu=relu)
            y.backward(g)
            runs.append([y.detach(), xx.grad, m.weight.grad.clone(), m.bias.grad.clone()]
                        + ([rr.grad] if res else []))
    finally:
        ext().bn_set_vec4(True)
    for a, b in zip(*runs):
        assert torch.equal(a, b)  # deterministic
    y, dx, dw, db = runs[0][:4]
    torch.testing.assert_close(y.double().cpu(), yd.detach(), rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(dx.double().cpu(), xd.grad, rtol=1e-4, atol=5e-5)
    torch.testing.assert_close(dw.double().cpu(), wd.grad, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(db.double().cpu(), bd.grad, rtol=1e-5, atol=1e-4)
    if res:
        torch.testing.assert_close(runs[0][4].double().cpu(), rd.grad, rtol=0, atol=1e-6)
