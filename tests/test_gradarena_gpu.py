"""Dense arm: native conv / BN backwards write gradients straight into the bucket arena
(ops/gradarena.py) — no flatten copy for them — with the same update as
the reference arm (per-parameter all-reduce + torch SGD, ddp_guide_cifar10/ddp_init.py:57-62,111)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def test_dense_arena_gradients_in_place(device, monkeypatch):
    from network_distributed_pytorch_amd.models import build_model
    from network_distributed_pytorch_amd.parallel.ddp import BucketedDataParallel

    # MIOpen's strided 3x3 grad-x (the one non-native kernel) may accumulate atomically
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(0)
    ours = build_model("resnet18", 10).to(device)
    ref = build_model("resnet18", 10).to(device)
    ref.load_state_dict(ours.state_dict())
    ddp = BucketedDataParallel(ours, lr=0.1, momentum=0.9)
    opt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    lo, hi = ddp.g.data_ptr(), ddp.g.data_ptr() + ddp.g.numel() * 4
    x = torch.randn(32, 3, 32, 32, device=device)
    y = torch.randint(0, 10, (32,), device=device)
    ddp.zero_grad()
    F.cross_entropy(ours(x), y).backward()
    inside = {n: lo <= p.grad.data_ptr() < hi for n, p in ours.named_parameters()}
    assert all(v for n, v in inside.items() if ".bn" in n or "conv" in n or "downsample" in n), inside
    assert not inside["fc.weight"]  # ATen Linear (10 classes): copied by the bucket flatten
    opt.zero_grad()
    F.cross_entropy(ref(x), y).backward()
    for (n, a), (_, b) in zip(ours.named_parameters(), ref.named_parameters()):
        assert torch.equal(a.grad, b.grad), n  # same kernels: in-place grads are bitwise the same
    ddp.step()
    opt.step()
    for (n, a), (_, b) in zip(ours.named_parameters(), ref.named_parameters()):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), n  # fused SGD vs torch.optim.SGD


def test_tied_weight_not_aliased(device):
    """a parameter used twice in one forward (a shared BN here) gets two gradient
    contributions in the same backward; the second must not alias the arena slice handed
    to the first (that would give 2 x g2 instead of g1 + g2)."""
    from network_distributed_pytorch_amd.ops.batchnorm import BatchNormAct2d
    from network_distributed_pytorch_amd.parallel.ddp import BucketedDataParallel

    class Tied(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.bn = BatchNormAct2d(8)
            self.head = torch.nn.Linear(8 * 16, 3)

        def forward(self, x):
            h = self.bn(x, relu=True)
            h = self.bn(h * 1.5 - 0.25, relu=True)  # the same weight / bias again
            return self.head(h.flatten(1))

    torch.manual_seed(0)
    ours = Tied().to(device)
    ref = Tied().to(device)
    ref.load_state_dict(ours.state_dict())
    with torch.no_grad():
        ours.bn.weight.uniform_(0.5, 1.5)
        ref.bn.weight.copy_(ours.bn.weight)
    ddp = BucketedDataParallel(ours, lr=0.1, momentum=0.9)
    x = torch.randn(16, 8, 4, 4, device=device)
    y = torch.randint(0, 3, (16,), device=device)
    for _ in range(2):  # the second step re-hands the slices after zero_grad
        ddp.zero_grad()
        for p in ref.parameters():
            p.grad = None
        F.cross_entropy(ours(x), y).backward()
        F.cross_entropy(ref(x), y).backward()  # not registered: plain autograd accumulation
        for (n, a), (_, b) in zip(ours.named_parameters(), ref.named_parameters()):
            assert torch.allclose(a.grad, b.grad, rtol=1e-5, atol=1e-6), n
