"""CPU checks for this round's fusion plumbing: the gradient / slab hand-off objects and the
CPU fallbacks of the fused ops (the device paths are covered by the GPU tests)."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd.ops.gradlink import BranchLink, GradLink
from network_distributed_pytorch_amd.ops.layernorm import AddLayerNorm
from network_distributed_pytorch_amd.ops.linear import linear, linear_gelu
from network_distributed_pytorch_amd.ops.loss import CrossEntropyLoss, cross_entropy
from network_distributed_pytorch_amd.ops.slablink import SlabLink


def test_slablink_put_take():
    link = SlabLink()
    assert link.take_fwd() == (None, 0) and link.take_bwd() == (None, 0)
    p = torch.zeros(8)
    link.put_fwd(p, 2)
    with pytest.raises(AssertionError):
        link.put_fwd(p, 2)
    t, n = link.take_fwd()
    assert t is p and n == 2 and link.fwd is None
    link.put_bwd(p, 4)
    assert link.take_bwd()[1] == 4 and link.bwd is None


def test_branchlink_needs_two_members():
    br = BranchLink()
    assert not br.active()
    br.join()
    assert not br.active()
    br.join()
    assert br.active()
    g = torch.ones(3)
    br.put(g)
    with pytest.raises(AssertionError):
        br.put(g)
    assert br.take() is g and br.take() is None


def test_gradlink_linear_cpu_adds_residual_grad():
    torch.manual_seed(0)
    x = torch.randn(5, 8, requires_grad=True)
    w = torch.randn(4, 8, requires_grad=True)
    b = torch.randn(4, requires_grad=True)
    link = GradLink()
    extra = torch.randn(5, 8)
    y = linear(x, w, b, link)
    link.put(extra)
    y.sum().backward()
    ref = torch.ones(5, 4) @ w.detach() + extra
    torch.testing.assert_close(x.grad, ref)


def test_cross_entropy_cpu_fallback_matches_torch():
    torch.manual_seed(1)
    x = torch.randn(9, 7, requires_grad=True)
    t = torch.randint(0, 7, (9,))
    t[3] = -100
    torch.testing.assert_close(CrossEntropyLoss()(x, t), F.cross_entropy(x, t))
    torch.testing.assert_close(cross_entropy(x, t, ignore_index=-100), F.cross_entropy(x, t))


@pytest.mark.parametrize("res", [False, True])
def test_add_layernorm_cpu_fallback(res):
    torch.manual_seed(2)
    m = AddLayerNorm(16)
    x = torch.randn(3, 5, 16)
    r = torch.randn(3, 5, 16) if res else None
    ref = F.layer_norm(x + r if res else x, (16,), m.weight, m.bias, m.eps)
    torch.testing.assert_close(m(x, residual=r), ref)
    assert list(m.state_dict()) == ["weight", "bias"]  # nn.LayerNorm keys (HF checkpoints load)


def test_linear_gelu_cpu_fallback():
    torch.manual_seed(3)
    x = torch.randn(6, 8)
    w = torch.randn(12, 8)
    b = torch.randn(12)
    torch.testing.assert_close(linear_gelu(x, w, b), F.gelu(F.linear(x, w, b)))


def test_ln_keep_mask_host_twin():
    """Host twin of the LayerNorm hash-dropout mask: deterministic per seed, ~p dropped,
    different seeds / rows / columns decorrelated."""
    from network_distributed_pytorch_amd.ops.layernorm import ln_keep_mask

    a = ln_keep_mask(3, 512, 768, 0.1)
    assert torch.equal(a, ln_keep_mask(3, 512, 768, 0.1))
    assert abs((1 - a.float().mean().item()) - 0.1) < 0.005
    b = ln_keep_mask(4, 512, 768, 0.1)
    assert (a != b).float().mean().item() > 0.15  # ~2 p (1 - p) for independent masks
    assert (a[1:] != a[:-1]).float().mean().item() > 0.15
    assert ln_keep_mask(3, 4, 256, 0.0).all()


def test_add_layernorm_dropout_cpu_path():
    """CPU (unfused) path of the fused-dropout LayerNorm keeps nn.Dropout semantics."""
    torch.manual_seed(0)
    m = AddLayerNorm(256)
    x = torch.randn(64, 256)
    r = torch.randn(64, 256)
    y = m(x, residual=r, p_out=0.5)
    zero = (y == 0).float().mean().item()
    assert 0.4 < zero < 0.6
    y_in = m(x, residual=r, p_in=0.0)
    torch.testing.assert_close(y_in, F.layer_norm(x + r, (256,), m.weight, m.bias, m.eps))
