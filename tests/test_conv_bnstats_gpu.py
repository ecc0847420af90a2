"""BatchNorm statistics from the direct-conv forward epilogue (csrc/conv.hip ``stats``,
ops/slablink.py): the stem 7x7 and layer1 3x3 convs emit per-channel, per-batch-tile fp64
sums of their output and the consuming BN's apply kernel folds them instead of running its
statistics pass.  Checked against fp64 sums of the conv output, and end to end against the
BN statistics pass (same math, different summation order: close, not bitwise) plus bitwise
run-to-run repeatability."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd import ops
from network_distributed_pytorch_amd.models import build_resnet
from network_distributed_pytorch_amd.ops import conv as conv_mod
from network_distributed_pytorch_amd.ops._ext import ext
from network_distributed_pytorch_amd.ops.batchnorm import BatchNormAct2d
from network_distributed_pytorch_amd.ops.slablink import SlabLink
from tests._oracle import assert_fused_no_worse, resnet18_fp64_step

pytestmark = pytest.mark.gpu

# (B, C, H, W, Co, k, stride, pad): the stem at a small batch, layer1 at an unsplit batch
CASES = [(16, 3, 32, 32, 64, 7, 2, 3), (256, 64, 8, 8, 64, 3, 1, 1), (512, 64, 8, 8, 64, 3, 1, 1)]


@pytest.mark.parametrize("case", CASES)
def test_epilogue_stats_match_fp64(device, case):
    assert ops.native_available()
    B, C, H, W, Co, k, s, p = case
    torch.manual_seed(B)
    x = torch.randn(B, C, H, W, device=device)
    w = torch.randn(Co, C, k, k, device=device) * (2.0 / (C * k * k)) ** 0.5
    geom = [C, H, W, Co, k, k, s, p]
    S = int(ext().conv_stats_slices(geom, B))
    assert S > 0, "this geometry / batch should carry the statistics epilogue"
    OH = (H + 2 * p - k) // s + 1
    y = torch.empty(B, Co, OH, OH, device=device)
    stats = torch.full((Co * S * 2,), float("nan"), device=device, dtype=torch.float64)
    assert ext().conv_fwd(x, w, y, geom, None, False, stats) == 1
    ref = F.conv2d(x.double(), w.double(), stride=s, padding=p)
    assert (y.double() - ref).abs().max().item() < 1e-4 * ref.abs().max().item()
    st = stats.view(Co, S, 2)
    if S > B:  # the stem's output-row blocks (conv.hip PSPLIT): one partial per (image, block)
        rb = S // B
        yt = y.double().view(B, Co, rb, OH * OH // rb).permute(0, 2, 1, 3).reshape(S, 1, Co, OH * OH // rb)
        imgs, npix = 1, OH * OH // rb
    else:
        imgs, npix = B // S, OH * OH
        yt = y.double().view(S, imgs, Co, npix)
    tile_sum = yt.sum((1, 3)).t()  # [Co][S]
    tile_sq = (yt * yt).sum((1, 3)).t()
    assert torch.allclose(st[..., 0], tile_sum, rtol=1e-9, atol=1e-6 * imgs * npix)
    assert torch.allclose(st[..., 1], tile_sq, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("C,HW,N", [(64, 256, 32), (64, 64, 256)])
def test_bn_fold_of_conv_partials(device, C, HW, N):
    """bn_fwd with xstats (the apply folds S partials) == bn_fwd with its own statistics pass
    (to fp32 rounding of the statistics) — y, saved statistics, running statistics."""
    torch.manual_seed(C + HW)
    H = int(HW ** 0.5)
    x = torch.randn(N, C, H, H, device=device) * 1.7 + 0.3
    S = N  # one partial per image
    xd = x.double().view(N, C, HW)
    stats = torch.stack([xd.sum(2).t(), (xd * xd).sum(2).t()], dim=-1).contiguous().view(-1)
    outs = []
    for use in (False, True):
        bn = BatchNormAct2d(C).to(device)
        bn._ensure_part(x)
        y = torch.empty_like(x)
        sm, si = torch.empty(C, device=device), torch.empty(C, device=device)
        ext().bn_fwd(x, None, y, bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var,
                     bn.num_batches_tracked, sm, si, bn._part, 1e-5, 0.1, True, True, True, None, 0,
                     stats if use else None, S if use else 0)
        outs.append((y, sm, si, bn.running_mean.clone(), bn.running_var.clone(), bn.num_batches_tracked.clone()))
    for a, b in zip(*outs):
        if a.dtype == torch.int64:
            assert torch.equal(a, b)
        else:
            assert torch.allclose(a, b, rtol=2e-6, atol=2e-6), (a - b).abs().max().item()


def _step(model, x, y):
    model.zero_grad(set_to_none=True)
    loss = F.cross_entropy(model(x), y)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()}, \
        {k: v.clone() for k, v in model.state_dict().items()}


@pytest.mark.parametrize("batch", [64, 512])
def test_resnet18_epilogue_stats_close_and_repeatable(device, batch, monkeypatch):
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(0)
    m = build_resnet(18, 1000).to(device)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.rand(batch, 3, 32, 32, device=device) * 2 - 1
    y = torch.randint(0, 10, (batch,), device=device)
    runs = []
    for on in (False, True, True):
        monkeypatch.setattr(conv_mod, "CONV_BN_STATS", on)
        monkeypatch.setattr(conv_mod, "_STATS", {})
        m.load_state_dict(state)
        runs.append(_step(m, x, y))
    (l0, g0, s0), (l1, g1, s1), (l2, g2, s2) = runs
    # on is deterministic
    assert torch.equal(l1, l2)
    for n in g1:
        assert torch.equal(g1[n], g2[n]), n
    # on == off up to the summation order of the statistics: both judged against the exact step
    # (tests/_oracle.py: the arms' mutual distance is chaotic rounding amplification)
    lr, gr = resnet18_fp64_step(state, x, y)
    assert abs(l1.item() - lr) < 1e-5 * max(1.0, abs(lr)) and abs(l0.item() - lr) < 1e-5 * max(1.0, abs(lr))
    assert_fused_no_worse(g1, g0, gr)
    for k in s0:
        if s0[k].dtype.is_floating_point:
            assert torch.allclose(s0[k], s1[k], rtol=1e-5, atol=1e-6), k
        else:
            assert torch.equal(s0[k], s1[k]), k


def test_stats_link_unused_by_unfused_bn(device):
    """A link whose consumer is not the fused kernel leaves nothing pending."""
    link = SlabLink()
    link.put_stats(torch.zeros(4, device=device, dtype=torch.float64), 1)
    bn = BatchNormAct2d(2, momentum=None).to(device)
    x = torch.randn(4, 2, 4, 4, device=device)
    bn(x, slab_in=link)
    assert link.stats is None


@pytest.mark.parametrize("B", [256, 512])
@pytest.mark.parametrize("Co,st", [(64, 1), (128, 2)])
def test_dgrad_epilogue_bwd_stats_match_fp64(device, B, Co, st):
    """Backward mode: the layer1 grad-x epilogue (and layer2's strided entry conv's, run as the
    same kernel on the zero-inserted dY) emits, per channel and image, the sums of
    dz = dx * (y > 0) and dz * (x - mean) * invstd for the BN whose output gradient dx is."""
    C, H = 64, 8
    geom = [C, H, H, Co, 3, 3, st, 1]
    S = int(ext().conv_dgrad_stats_slices(geom, B))
    assert S > 0 and B % S == 0  # per image (direct kernel) or per 4-image tile (Winograd)
    torch.manual_seed(B + 1)
    OH = (H - 1) // st + 1
    dy = torch.randn(B, Co, OH, OH, device=device)
    w = torch.randn(Co, C, 3, 3, device=device) * 0.05
    bx = torch.randn(B, C, H, H, device=device) * 1.5 + 0.2
    by = torch.relu(torch.randn(B, C, H, H, device=device))
    mean = torch.randn(C, device=device) * 0.1
    invstd = torch.rand(C, device=device) + 0.5
    dx = torch.empty_like(bx)
    dx_ref = torch.empty_like(bx)
    stats = torch.full((C * S * 2,), float("nan"), device=device, dtype=torch.float64)
    ext().conv_dgrad(dy, w, dx_ref, geom, None, None, False)
    ext().conv_dgrad(dy, w, dx, geom, None, None, False, stats, bx, by, mean, invstd)
    assert torch.equal(dx, dx_ref)
    dz = dx.double() * (by > 0).double()
    xh = (bx.double() - mean.double().view(1, C, 1, 1)) * invstd.double().view(1, C, 1, 1)
    st = stats.view(C, S, 2)
    ref_a = dz.sum((2, 3)).view(S, B // S, C).sum(1).t()
    ref_b = (dz * xh).sum((2, 3)).view(S, B // S, C).sum(1).t()
    tol = 1e-5 * (dz.abs().max().item() * H * H)
    assert (st[..., 0] - ref_a).abs().max().item() < tol
    assert (st[..., 1] - ref_b).abs().max().item() < tol * 8


@pytest.mark.parametrize("batch", [256, 512])
def test_resnet18_bwd_epilogue_stats_close_and_repeatable(device, batch, monkeypatch):
    from network_distributed_pytorch_amd.ops import batchnorm as bn_mod

    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(0)
    m = build_resnet(18, 1000).to(device)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.rand(batch, 3, 32, 32, device=device) * 2 - 1
    y = torch.randint(0, 10, (batch,), device=device)
    runs = []
    for on in (False, True, True):
        monkeypatch.setattr(bn_mod, "_BWD_STATS", on)
        m.load_state_dict(state)
        runs.append(_step(m, x, y))
    (l0, g0, s0), (l1, g1, s1), (l2, g2, s2) = runs
    assert torch.equal(l1, l2) and torch.equal(l0, l1)
    for n in g1:
        assert torch.equal(g1[n], g2[n]), n
    # the arms differ in the BN backward statistics' summation order only: both judged against
    # the exact step (tests/_oracle.py)
    assert_fused_no_worse(g1, g0, resnet18_fp64_step(state, x, y)[1])
