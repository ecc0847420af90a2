"""Fused softmax cross-entropy (csrc/loss.hip) vs an fp64 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd import ops
from network_distributed_pytorch_amd.ops.loss import CrossEntropyLoss, cross_entropy

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,K", [(512, 1000), (64, 1000), (16, 2), (1, 7), (333, 10), (1029, 129)])
def test_cross_entropy_matches_fp64(device, B, K):
    assert ops.native_available()
    torch.manual_seed(B + K)
    x = (torch.randn(B, K, device=device) * 3).requires_grad_(True)
    t = torch.randint(0, K, (B,), device=device)
    if B > 8:
        t[::7] = -100  # ignored rows
    x64 = x.detach().double().requires_grad_(True)
    ref = F.cross_entropy(x64, t)
    loss = cross_entropy(x, t)
    assert loss.dtype == torch.float32 and loss.dim() == 0
    torch.testing.assert_close(loss.double(), ref, rtol=2e-6, atol=2e-6)
    g = torch.tensor(1.7, device=device)
    (loss * g).backward()
    (ref * g.double()).backward()
    torch.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-5, atol=1e-7)


def test_cross_entropy_deterministic_and_graph_safe(device):
    torch.manual_seed(0)
    x = torch.randn(256, 1000, device=device)
    t = torch.randint(0, 1000, (256,), device=device)
    crit = CrossEntropyLoss()
    a = [crit(x, t) for _ in range(3)]
    assert all(torch.equal(a[0], v) for v in a)
    xs = x.clone().requires_grad_(True)
    out = torch.zeros((), device=device)
    crit(xs, t).backward()  # warm-up (eager) allocates the counter
    xs.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss = crit(xs, t)
        loss.backward()
        out.copy_(loss)
    for _ in range(3):
        xs.grad.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, a[0])
    torch.testing.assert_close(xs.grad, torch.autograd.grad(F.cross_entropy(x.requires_grad_(True), t), x)[0],
                               rtol=1e-5, atol=1e-7)


def test_cross_entropy_cpu_fallback():
    x = torch.randn(8, 5, requires_grad=True)
    t = torch.randint(0, 5, (8,))
    torch.testing.assert_close(CrossEntropyLoss()(x, t), F.cross_entropy(x, t))


def test_cross_entropy_accumulates_running_sum(device):
    """``accumulate``: the kernel adds each loss into the running sum (no add launch); the
    same sum as adding the returned losses, and the loss / gradient are unchanged."""
    torch.manual_seed(5)
    acc = torch.zeros((), device=device)
    crit = CrossEntropyLoss()
    crit.accumulate = acc
    ref = torch.zeros((), device=device)
    for i in range(3):
        x = (torch.randn(64, 1000, device=device) * 2).requires_grad_(True)
        t = torch.randint(0, 10, (64,), device=device)
        loss = crit(x, t)
        plain = cross_entropy(x.detach(), t)
        assert torch.equal(loss.detach(), plain)
        ref += plain
        loss.backward()
        assert torch.isfinite(x.grad).all()
    torch.cuda.synchronize()
    assert torch.equal(acc, ref)
