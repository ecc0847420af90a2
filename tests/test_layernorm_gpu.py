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


@pytest.mark.parametrize("mode", ["in", "out"])
@pytest.mark.parametrize("shape", [(4, 128, 768), (33, 512)])
def test_add_layernorm_hash_dropout_vs_fp64(device, mode, shape):
    """Hash dropout fused into the LayerNorm (DistilBERT FFN: LN(drop(a) + x); embeddings:
    drop(LN(a + x))) against fp64 math with the host twin of the kernel's keep mask."""
    from network_distributed_pytorch_amd.ops.layernorm import add_layer_norm, ln_keep_mask

    torch.manual_seed(11)
    D, p = shape[-1], 0.1
    R = torch.Size(shape[:-1]).numel()
    w = torch.empty(D, device=device).uniform_(0.5, 1.5).requires_grad_(True)
    b = torch.empty(D, device=device).uniform_(-0.5, 0.5).requires_grad_(True)
    a = torch.randn(shape, device=device, requires_grad=True)
    x = torch.randn(shape, device=device, requires_grad=True)
    seed = torch.tensor([987654], device=device, dtype=torch.int32)
    kw = dict(p_in=p) if mode == "in" else dict(p_out=p)
    y = add_layer_norm(a, x, w, b, 1e-12, seed=seed, **kw)
    keep = ln_keep_mask(987654, R, D, p, device=device).view(shape).double()
    assert 0.08 < 1 - keep.mean().item() < 0.12  # drops about p
    a64, x64, w64, b64 = (t.detach().double().requires_grad_(True) for t in (a, x, w, b))
    if mode == "in":
        y64 = F.layer_norm(a64 * keep / (1 - p) + x64, (D,), w64, b64, 1e-12)
    else:
        y64 = F.layer_norm(a64 + x64, (D,), w64, b64, 1e-12) * keep / (1 - p)
    torch.testing.assert_close(y.double(), y64, rtol=1e-5, atol=3e-5)
    g = torch.randn(shape, device=device)
    y.backward(g)
    y64.backward(g.double())
    for t, t64 in ((a, a64), (x, x64)):
        torch.testing.assert_close(t.grad.double(), t64.grad, rtol=1e-4, atol=3e-5)
    tol = 3e-5 * R ** 0.5
    torch.testing.assert_close(w.grad.double(), w64.grad, rtol=1e-4, atol=tol)
    torch.testing.assert_close(b.grad.double(), b64.grad, rtol=1e-4, atol=tol)


def test_distilbert_dropout_fused_into_layernorm(device):
    """DistilBERT in training mode draws its hidden dropouts inside the LayerNorm kernels: no
    ATen dropout kernels, and the masks differ per call (fresh device seeds)."""
    from network_distributed_pytorch_amd.models.distilbert import distilbert_base

    torch.manual_seed(0)
    m = distilbert_base(2, n_layers=2, seq_classif_dropout=0.0).to(device).train()
    ids = torch.randint(1, 1000, (2, 64), device=device)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        out = m(ids)[0]
        out.sum().backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events()]
    assert not any("dropout" in n.lower() or "bernoulli" in n.lower() for n in names), \
        sorted({n for n in names if "drop" in n.lower() or "bernoulli" in n.lower()})
    with torch.no_grad():
        o1, o2 = m(ids)[0], m(ids)[0]
    assert not torch.equal(o1, o2)  # training-mode dropout: fresh masks per call
    m.eval()
    with torch.no_grad():
        assert torch.equal(m(ids)[0], m(ids)[0])
