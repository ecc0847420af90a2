"""Native max-pool (csrc/pool.hip) vs torch's max_pool2d (fp32 reference)."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd import ops
from network_distributed_pytorch_amd.ops.pool import MaxPool2d


def test_maxpool_module_cpu_matches_torch():
    torch.manual_seed(0)
    x = torch.randn(2, 3, 9, 10, requires_grad=True)
    y = MaxPool2d(3, 2, 1)(x)
    ref = F.max_pool2d(x, 3, 2, 1)
    assert torch.equal(y, ref)
    assert MaxPool2d(3, 2, 1).state_dict() == {}


@pytest.mark.gpu
@pytest.mark.parametrize("shape,k,s,p", [((512, 64, 16, 16), 3, 2, 1), ((4, 8, 15, 13), 3, 2, 1),
                                         ((3, 5, 7, 7), 2, 2, 0), ((2, 3, 11, 9), 5, 3, 2),
                                         ((1, 1, 1, 1), 1, 1, 0), ((6, 4, 8, 8), 3, 1, 1),
                                         # vectorised stem paths (even maps, W % 4 == 0)
                                         ((3, 4, 8, 8), 3, 2, 1), ((2, 3, 32, 32), 3, 2, 1), ((64, 64, 16, 16), 3, 2, 1)])
def test_maxpool_fwd_bwd(device, shape, k, s, p):
    assert ops.native_available()
    torch.manual_seed(0)
    x = torch.randn(shape, device=device).requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    y = MaxPool2d(k, s, p)(x)
    ref = F.max_pool2d(x2, k, s, p)
    assert torch.equal(y, ref)
    dy = torch.randn_like(ref)
    y.backward(dy)
    ref.backward(dy)
    # fp32 sums of <= ceil(k/s)^2 terms in a different order: equal to ~1 ulp
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("hw", [6, 16])  # generic kernel / vectorised stem path
def test_maxpool_ties_pick_first_and_deterministic(device, hw):
    x = torch.zeros(2, 3, hw, hw, device=device, requires_grad=True)  # every window is a tie
    x2 = x.detach().clone().requires_grad_(True)
    y = MaxPool2d(3, 2, 1)(x)
    ref = F.max_pool2d(x2, 3, 2, 1)
    dy = torch.randn_like(ref)
    y.backward(dy)
    ref.backward(dy)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-6, atol=1e-6)
    g1 = x.grad.clone()
    x.grad = None
    MaxPool2d(3, 2, 1)(x).backward(dy)
    assert torch.equal(g1, x.grad)
