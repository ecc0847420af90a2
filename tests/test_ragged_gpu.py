"""Ragged batches (the reference's DataLoader keeps the short last batch) on the native conv
kernels: a batch the direct kernels cannot tile runs zero-padded on them (models/conv_gemm.py,
ops/conv.direct_plan_padded) — exact against fp64 and bitwise repeatable, where the former
fallback (MIOpen with a run-dependent algorithm) made resumed training drift from the
uninterrupted run."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(128, 4, 4, 128, 3, 1, 1), (64, 8, 8, 128, 3, 2, 1), (64, 8, 8, 128, 1, 2, 0), (64, 8, 8, 64, 3, 1, 1)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("B", [2, 3, 5])
def test_ragged_batch_direct_conv_exact_and_repeatable(device, shape, B):
    from network_distributed_pytorch_amd.models.conv_gemm import GemmConv2d
    from network_distributed_pytorch_amd.ops.conv import direct_plan, direct_plan_padded

    C, H, W, Co, k, s, p = shape
    torch.manual_seed(B)
    conv = GemmConv2d(C, Co, kernel_size=k, stride=s, padding=p, bias=False).to(device)
    x0 = torch.randn(B, C, H, W, device=device)
    if direct_plan(x0, conv.weight, s, p) is None:
        assert direct_plan_padded(x0, conv.weight, s, p) is not None
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    g = torch.randn(B, Co, OH, OW, device=device)
    outs = []
    for _ in range(2):
        junk = torch.full((64 << 20,), float("nan"), device=device)  # poison the allocator's free blocks
        del junk
        x = x0.clone().requires_grad_(True)
        conv.weight.grad = None
        y = conv(x)
        y.backward(g)
        outs.append((y.detach().clone(), x.grad.clone(), conv.weight.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    xd, wd = x0.double().requires_grad_(True), conv.weight.detach().double().requires_grad_(True)
    yr = F.conv2d(xd, wd, stride=s, padding=p)
    yr.backward(g.double())
    for got, ref in zip(outs[0], (yr.detach(), xd.grad, wd.grad)):
        err = (got.double() - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)
        assert err < 2e-6, err
