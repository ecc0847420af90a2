"""The downsample block's bn2 + downsample BN + ReLU in one launch per direction
(csrc/batchnorm.hip BnPair, ops/batchnorm.bn_pair_act): checked against fp64 torch math of
relu(bn(x) + bn2(x2)) (output, saved / running statistics, all four parameter gradients and
both input gradients), bitwise against the two single launches where both use the same kernel
family, and end to end in the ResNet-18 step."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd.models import build_resnet
from network_distributed_pytorch_amd.ops import batchnorm as bn_mod
from network_distributed_pytorch_amd.ops._ext import ext
from network_distributed_pytorch_amd.ops.batchnorm import BatchNormAct2d, bn_pair_act
from network_distributed_pytorch_amd.ops.slablink import SlabLink
from tests._oracle import assert_fused_no_worse, resnet18_fp64_step

pytestmark = pytest.mark.gpu

# (N, C, H): ResNet-18's layer2/3/4 entry maps at per-GPU batch 64 / 512, plus ragged batches
SHAPES = [(64, 128, 4), (64, 256, 2), (64, 512, 1), (512, 128, 4), (512, 256, 2), (512, 512, 1), (100, 256, 2),
          (37, 64, 4), (200, 128, 1)]


def _bns(C, device, seed):
    torch.manual_seed(seed)
    out = []
    for _ in range(2):
        b = BatchNormAct2d(C).to(device)
        with torch.no_grad():
            b.weight.uniform_(0.5, 1.5)
            b.bias.uniform_(-0.3, 0.3)
            b.running_mean.uniform_(-0.1, 0.1)
            b.running_var.uniform_(0.8, 1.2)
        out.append(b)
    return out


def _ref(x, x2, bns, go):
    """fp64 torch: relu(bn(x) + bn2(x2)) in training mode, its gradients, the running stats."""
    xd, x2d = x.double().requires_grad_(), x2.double().requires_grad_()
    ps = [(b.weight.detach().double().requires_grad_(), b.bias.detach().double().requires_grad_()) for b in bns]
    rs = [(b.running_mean.double().clone(), b.running_var.double().clone()) for b in bns]
    z = sum(F.batch_norm(t, rm, rv, w, bb, True, 0.1, 1e-5) for t, (w, bb), (rm, rv) in zip((xd, x2d), ps, rs))
    y = torch.relu(z)
    grads = torch.autograd.grad(y, (xd, x2d, ps[0][0], ps[0][1], ps[1][0], ps[1][1]), go.double())
    return y, grads, rs


def _close(a, b, tol, what):
    err = (a.double() - b).abs().max().item()
    scale = b.abs().max().item() + 1e-12
    assert err <= tol * scale + 1e-7, (what, err, scale)


@pytest.mark.parametrize("N,C,H", SHAPES)
def test_bn_pair_vs_fp64(device, N, C, H):
    assert ext().bn_pair_ok(N, C, H * H)
    torch.manual_seed(N + C + H)
    x = (torch.randn(N, C, H, H, device=device) * 1.3 + 0.2).requires_grad_()
    x2 = (torch.randn(N, C, H, H, device=device) * 0.7 - 0.1).requires_grad_()
    go = torch.randn(N, C, H, H, device=device)
    bns = _bns(C, device, 7)
    r, rg, rs = _ref(x.detach(), x2.detach(), bns, go)
    y = bn_pair_act(bns[0], bns[1], x, x2)
    assert y is not None
    _close(y, r, 2e-6, "y")
    g = torch.autograd.grad(y, (x, x2, bns[0].weight, bns[0].bias, bns[1].weight, bns[1].bias), go)
    for a, b, n in zip(g, rg, ("dx", "dx2", "dgamma", "dbeta", "dgamma2", "dbeta2")):
        _close(a, b, 2e-5, n)
    for b, (rm, rv) in zip(bns, rs):
        _close(b.running_mean, rm, 1e-6, "running_mean")
        _close(b.running_var, rv, 1e-6, "running_var")
        assert int(b.num_batches_tracked) == 1


@pytest.mark.parametrize("N,C,H", [(64, 128, 4), (64, 256, 2), (64, 512, 1), (512, 128, 4), (512, 256, 2)])
def test_bn_pair_bitwise_vs_two_launches(device, N, C, H):
    """Same kernel family on both sides (HW >= 4, or per-GPU batch <= 128): the pair's output,
    gradients and statistics are bitwise those of the downsample BN launch + the bn2 launch."""
    torch.manual_seed(3)
    x = torch.randn(N, C, H, H, device=device) * 1.3 + 0.2
    x2 = torch.randn(N, C, H, H, device=device) * 0.7 - 0.1
    go = torch.randn(N, C, H, H, device=device)
    outs = []
    for pair in (True, False):
        bns = _bns(C, device, 11)
        a, b = x.clone().requires_grad_(), x2.clone().requires_grad_()
        if pair:
            y = bn_pair_act(bns[0], bns[1], a, b)
        else:
            y = bns[0](a, residual=bns[1](b), relu=True)
        g = torch.autograd.grad(y, (a, b, bns[0].weight, bns[0].bias, bns[1].weight, bns[1].bias), go)
        outs.append((y,) + g + tuple(t.clone() for m in bns for t in (m.running_mean, m.running_var)))
    for u, v in zip(*outs):
        assert torch.equal(u, v)


def test_bn_pair_consumes_split_k_slabs(device):
    """x and x2 arriving as unsummed split-K slabs (ops/slablink.py) == the summed tensors."""
    N, C, H, ks = 64, 128, 4, 3
    torch.manual_seed(5)
    parts = [torch.randn(ks, N, C, H, H, device=device) for _ in range(2)]
    sums = [p[0] + p[1] + p[2] for p in parts]  # slab order, as the kernel adds them
    res = []
    for slabs in (False, True):
        bns = _bns(C, device, 13)
        x = torch.empty(N, C, H, H, device=device) if slabs else sums[0].clone()
        x2 = torch.empty(N, C, H, H, device=device) if slabs else sums[1].clone()
        l1 = l2 = None
        if slabs:
            l1, l2 = SlabLink(), SlabLink()
            l1.put_fwd(parts[0], ks)
            l2.put_fwd(parts[1], ks)
        y = bn_pair_act(bns[0], bns[1], x.requires_grad_(), x2.requires_grad_(), slab_in=l1, slab_in2=l2)
        res.append((y.detach(), x.detach().clone(), x2.detach().clone()))
    for u, v in zip(*res):
        assert torch.equal(u, v)


def _step(model, x, y):
    model.zero_grad(set_to_none=True)
    loss = F.cross_entropy(model(x), y)
    loss.backward()
    torch.cuda.synchronize()
    return loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()}, \
        {k: v.clone() for k, v in model.state_dict().items()}


@pytest.mark.parametrize("batch", [64, 512])
def test_resnet18_bn_pair_step(device, batch, monkeypatch):
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(0)
    m = build_resnet(18, 1000).to(device)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.rand(batch, 3, 32, 32, device=device) * 2 - 1
    y = torch.randint(0, 10, (batch,), device=device)
    calls = []
    orig = bn_mod._BNPairFn.apply

    def counting(*a):
        calls.append(1)
        return orig(*a)

    runs = []
    for on in (False, True):
        monkeypatch.setattr(bn_mod, "BN_PAIR", on)
        monkeypatch.setattr(bn_mod._BNPairFn, "apply", counting)
        m.load_state_dict(state)
        runs.append(_step(m, x, y))
    assert len(calls) == 3  # layer2 / layer3 / layer4 entry blocks, on-arm only
    (l0, g0, s0), (l1, g1, s1) = runs
    if batch == 64:  # the same kernel family on both arms (see the bitwise test): bitwise
        assert torch.equal(l0, l1)
        for n in g0:
            assert torch.equal(g0[n], g1[n]), n
        for k in s0:
            assert torch.equal(s0[k], s1[k]), k
    else:  # layer4 (1x1 maps): scalar pair kernel vs float4 single launches — summation order
        assert abs(l0.item() - l1.item()) < 1e-5 * max(1.0, abs(l0.item()))
        assert_fused_no_worse(g1, g0, resnet18_fp64_step(state, x, y)[1])  # tests/_oracle.py
        for k in s0:
            if s0[k].dtype.is_floating_point:
                assert torch.allclose(s0[k], s1[k], rtol=1e-5, atol=1e-6), k
            else:
                assert torch.equal(s0[k], s1[k]), k
