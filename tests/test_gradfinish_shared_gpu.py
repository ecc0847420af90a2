"""Deferred gradient finishing (ops/gradfinish.py) with a module applied twice in one forward.

A Linear bias / LayerNorm gamma-beta gradient whose final sum is deferred to the end of the
backward returns an unfilled buffer; when the same parameter gets a second gradient in the
same graph task autograd adds the two buffers at once.  gradfinish must finish the first
before that add: the gradients here are compared with plain torch in fp64.
"""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd.ops import gradfinish
from network_distributed_pytorch_amd.ops.layernorm import AddLayerNorm
from network_distributed_pytorch_amd.ops.linear import Linear

pytestmark = pytest.mark.gpu


def test_shared_linear_and_layernorm_grads_vs_fp64(device):
    assert gradfinish.enabled()
    torch.manual_seed(3)
    D = 768
    lin = Linear(D, D).to(device)
    ln = AddLayerNorm(D, eps=1e-12).to(device)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.5, 0.5)
    x = torch.randn(8, 64, D, device=device)
    g = torch.randn(8, 64, D, device=device)
    # shared modules: lin and ln each run twice in one forward
    y = ln(lin(ln(lin(x))))
    y.backward(g)

    p64 = {n: p.detach().double().requires_grad_(True) for n, p in
           (("w", lin.weight), ("b", lin.bias), ("lw", ln.weight), ("lb", ln.bias))}

    def ref(t):
        t = F.linear(t, p64["w"], p64["b"])
        return F.layer_norm(t, (D,), p64["lw"], p64["lb"], 1e-12)

    ref(ref(x.double())).backward(g.double())
    rows = x.numel() // D
    for name, p in (("w", lin.weight), ("b", lin.bias), ("lw", ln.weight), ("lb", ln.bias)):
        exp = p64[name].grad
        tol = 3e-5 * rows ** 0.5 * max(1.0, exp.abs().max().item())
        err = (p.grad.double() - exp).abs().max().item()
        assert err <= tol, (name, err, tol)
    assert gradfinish.pending() == 0
