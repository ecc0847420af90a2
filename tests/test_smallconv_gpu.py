"""Small-map conv kernels (csrc/smallconv.hip) against an fp64 PyTorch reference: forward,
grad-x and grad-W for every covered geometry, at batches that hit the whole-tile path, the
split-K slabs (small batch) and ragged row tiles; bitwise determinism; the fused-BN slab
hand-off and the residual addend."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (C, H, W, Co, K, stride, pad): the ResNet-18 / -50 layer3 / layer4 geometries
GEOMS = [
    (64, 2, 2, 96, 3, 1, 1),    # 3x3 on 2x2
    (64, 4, 4, 64, 3, 2, 1),    # 3x3 / 2, 4x4 -> 2x2
    (64, 4, 4, 128, 1, 2, 0),   # 1x1 / 2, 4x4 -> 2x2
    (96, 2, 2, 64, 3, 2, 1),    # 3x3 / 2, 2x2 -> 1x1
    (64, 1, 1, 64, 3, 1, 1),    # 3x3 on 1x1 (centre tap)
    (64, 2, 2, 128, 1, 2, 0),   # 1x1 / 2, 2x2 -> 1x1
    (128, 2, 2, 64, 1, 1, 0),   # 1x1 on 2x2
    (64, 1, 1, 96, 1, 1, 0),    # 1x1 on 1x1
]


def _run(geom, B, device, seed=0):
    from network_distributed_pytorch_amd.ops._ext import ext

    C, H, W, Co, K, s, p = geom
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(B, C, H, W, generator=g).to(device)
    w = (torch.randn(Co, C, K, K, generator=g) / (C * K * K) ** 0.5).to(device)
    OH = (H + 2 * p - K) // s + 1
    OW = (W + 2 * p - K) // s + 1
    dy = torch.randn(B, Co, OH, OW, generator=g).to(device)
    gl = [C, H, W, Co, K, K, s, p]
    cls, fs, ds, ws = ext().sm_plan(gl, B)
    assert cls >= 0, geom
    y = torch.empty(B, Co, OH, OW, device=device)
    part = torch.empty(max(fs, 1) * y.numel(), device=device)
    assert ext().sm_fwd(x, w, y, gl, part if fs > 1 else None, False) == 1
    dx = torch.empty_like(x)
    partx = torch.empty(max(ds, 1) * x.numel(), device=device)
    assert ext().sm_dgrad(dy, w, dx, gl, partx if ds > 1 else None, None, False) == 1
    wout = torch.empty(max(ws, 1) * w.numel(), device=device)
    z = ext().sm_wgrad(x, dy, wout, gl)
    dw = wout.view(z, *w.shape).double().sum(0)  # reference order is irrelevant at fp64
    xd, wd = x.double().requires_grad_(), w.double().requires_grad_()
    yr = F.conv2d(xd, wd, stride=s, padding=p)
    yr.backward(dy.double())
    return (y, dx, dw), (yr.detach(), xd.grad, wd.grad), (fs, ds, ws)


def _close(a, b, what):
    err = (a.double() - b).abs().max().item()
    scale = b.abs().max().item() + 1e-12
    assert err / scale < 2e-6, (what, err, scale)


@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("B", [8, 20, 64, 256])
def test_smallconv_matches_fp64(device, geom, B):
    (y, dx, dw), (yr, dxr, dwr), _ = _run(geom, B, device)
    _close(y, yr, "forward")
    _close(dx, dxr, "grad-x")
    _close(dw, dwr, "grad-W")


def test_smallconv_splits_exercised_and_deterministic(device):
    from network_distributed_pytorch_amd.ops._ext import ext

    # batch 64, 256 channels: the row kernels split the channels, grad-W splits the batch
    geom = (256, 2, 2, 256, 3, 1, 1)
    C, H, W, Co, K, s, p = geom
    cls, fs, ds, ws = ext().sm_plan([C, H, W, Co, K, K, s, p], 64)
    assert fs > 1 and ds > 1, (fs, ds)
    a, ref, _ = _run(geom, 64, device, seed=3)
    for t, r, n in zip(a, ref, ("forward", "grad-x", "grad-W")):
        _close(t, r, n)
    b, _, _ = _run(geom, 64, device, seed=3)
    for t, u in zip(a, b):
        assert torch.equal(t, u)
    cls, fs, ds, ws = ext().sm_plan([C, H, W, Co, K, K, s, p], 512)
    assert ws > 1  # 512 images, 256 x 256 channels: batch-split grad-W slabs


def test_smallconv_slab_defer_and_addend(device):
    from network_distributed_pytorch_amd.ops._ext import ext

    C, H, W, Co, K, s, p = geom = (256, 2, 2, 256, 3, 1, 1)
    gl = [C, H, W, Co, K, K, s, p]
    B = 64
    x = torch.randn(B, C, H, W, device=device)
    w = torch.randn(Co, C, K, K, device=device) * 0.05
    dy = torch.randn(B, Co, H, W, device=device)
    cls, fs, ds, ws = ext().sm_plan(gl, B)
    y = torch.empty(B, Co, H, W, device=device)
    part = torch.empty(fs * y.numel(), device=device)
    left = ext().sm_fwd(x, w, y, gl, part, True)
    assert left == fs > 1
    yref = torch.empty_like(y)
    ext().sm_fwd(x, w, yref, gl, torch.empty_like(part), False)
    ext().slab_sum(part, y.view(-1), left)
    assert torch.equal(y, yref)  # the deferred slabs summed later are bitwise the kernel's own sum
    add = torch.randn_like(x)
    want = torch.empty_like(x)
    ext().sm_dgrad(dy, w, want, gl, torch.empty(ds * x.numel(), device=device), None, False)
    want = want + add
    got = add.clone()
    ext().sm_dgrad(dy, w, got, gl, torch.empty(ds * x.numel(), device=device), got, False)
    assert torch.allclose(got, want, rtol=1e-6, atol=1e-6)


def test_resnet18_layer34_on_smallconv_matches_toeplitz(device, monkeypatch):
    """ResNet-18 step: the small-map kernels against the hipBLASLt Toeplitz path (NDP_SM off)."""
    from network_distributed_pytorch_amd.models import build_model
    from network_distributed_pytorch_amd.ops import smconv, smstage

    monkeypatch.setattr(smstage, "_ON", False)  # per-module path: conv kernels vs hipBLASLt only
    torch.manual_seed(0)
    m = build_model("resnet18", 10).to(device)
    x = torch.randn(64, 3, 32, 32, device=device)
    yl = torch.randint(0, 10, (64,), device=device)

    def grads(on):
        monkeypatch.setattr(smconv, "_ON", on)
        m.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x), yl)
        loss.backward()
        return loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters()}

    state = {k: v.clone() for k, v in m.state_dict().items()}
    l1, g1 = grads(True)
    m.load_state_dict(state)
    l0, g0 = grads(False)
    assert abs(l1.item() - l0.item()) < 1e-4
    for n in g0:
        a, b = g1[n].flatten().double(), g0[n].flatten().double()
        cos = (a @ b / (a.norm() * b.norm() + 1e-30)).item()
        assert cos > 0.9999, (n, cos)


@pytest.mark.parametrize("B", [64, 512, 24])
def test_fused_stage_matches_module_path(device, monkeypatch, B):
    """layer3 + layer4 as one fused-BN node (ops/smstage.py) against the per-module path (small-map
    convs + the BatchNorm kernels): output, loss, every gradient, running statistics."""
    from network_distributed_pytorch_amd.models import build_model
    from network_distributed_pytorch_amd.ops import smconv, smstage

    monkeypatch.setattr(smconv, "_ON", True)  # both paths on the small-map convs (off by default)
    torch.manual_seed(1)
    m = build_model("resnet18", 1000).to(device)
    with torch.no_grad():  # non-trivial BN affine parameters
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(B, 3, 32, 32, device=device)
    yl = torch.randint(0, 1000, (B,), device=device)

    def run(on):
        monkeypatch.setattr(smstage, "_ON", on)
        m.load_state_dict(state)
        m.zero_grad(set_to_none=True)
        out = m(x)
        loss = F.cross_entropy(out, yl)
        loss.backward()
        return out.detach(), {n: p.grad.clone() for n, p in m.named_parameters()}, \
            {k: v.clone() for k, v in m.state_dict().items()}

    o1, g1, s1 = run(True)
    o0, g0, s0 = run(False)
    assert torch.allclose(o1, o0, rtol=1e-4, atol=1e-4), (o1 - o0).abs().max()
    for n in g0:
        a, b = g1[n].double(), g0[n].double()
        err = ((a - b).norm() / (b.norm() + 1e-30)).item()
        assert err < 1e-4, (n, err)
    for k in s0:
        if s0[k].dtype.is_floating_point:
            assert torch.allclose(s1[k], s0[k], rtol=1e-4, atol=1e-5), k
        else:
            assert torch.equal(s1[k], s0[k]), k
