"""Fused residual add + LayerNorm (csrc/layernorm.hip) vs an fp64 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd import ops
from network_distributed_pytorch_amd.ops.layernorm import AddLayerNorm

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(16, 512, 768), (3, 5, 768), (7, 256), (1000, 1024), (9, 512)])
@pytest.mark.parametrize("res", [False, True])
def test_add_layernorm_vs_fp64(device, shape, res):
    assert ops.native_available()
    torch.manual_seed(len(shape) + shape[-1])
    D = shape[-1]
    m = AddLayerNorm(D, eps=1e-12).to(device)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    x = (torch.randn(shape, device=device) * 2 + 0.5).requires_grad_(True)
    r = torch.randn(shape, device=device, requires_grad=True) if res else None
    y = m(x, residual=r)
    x64 = x.detach().double().requires_grad_(True)
    r64 = r.detach().double().requires_grad_(True) if res else None
    w64 = m.weight.detach().double().requires_grad_(True)
    b64 = m.bias.detach().double().requires_grad_(True)
    y64 = F.layer_norm(x64 + r64 if res else x64, (D,), w64, b64, 1e-12)
    torch.testing.assert_close(y.double(), y64, rtol=1e-5, atol=2e-5)
    g = torch.randn(shape, device=device)
    y.backward(g)
    y64.backward(g.double())
    torch.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-4, atol=2e-5)
    if res:
        torch.testing.assert_close(r.grad.double(), r64.grad, rtol=1e-4, atol=2e-5)
    rows = x.numel() // D
    tol = 2e-5 * rows ** 0.5
    torch.testing.assert_close(m.weight.grad.double(), w64.grad, rtol=1e-4, atol=tol)
    torch.testing.assert_close(m.bias.grad.double(), b64.grad, rtol=1e-4, atol=tol)


def test_add_layernorm_deterministic(device):
    torch.manual_seed(5)
    m = AddLayerNorm(768).to(device)
    x = torch.randn(8192, 768, device=device)
    r = torch.randn(8192, 768, device=device)
    g = torch.randn(8192, 768, device=device)
    outs = []
    for _ in range(2):
        xx = x.clone().requires_grad_(True)
        y = m(xx, residual=r)
        y.backward(g)
        outs.append((y.detach(), xx.grad, m.weight.grad.clone(), m.bias.grad.clone()))
        m.weight.grad = m.bias.grad = None
    for a, b in zip(*outs):
        assert torch.equal(a, b)
