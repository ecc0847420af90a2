"""The whole-step fp64 oracle (tests/_oracle.py) must catch a small SYSTEMATIC drift, not only
wiring bugs: a 1 % error in every BatchNorm scale — what a fused BN kernel
applying gamma * 1.01 would produce — fails ``assert_fused_no_worse``, while the unperturbed
native step passes it."""
import pytest
import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd.models import build_resnet
from tests._oracle import assert_fused_no_worse, resnet18_fp64_step

pytestmark = pytest.mark.gpu


def _grads(model, state, x, y):
    model.load_state_dict(state)
    model.zero_grad(set_to_none=True)
    F.cross_entropy(model(x), y).backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().clone() for n, p in model.named_parameters()}


def test_oracle_flags_one_percent_bn_scale_drift(device):
    torch.manual_seed(0)
    m = build_resnet(18, 1000).to(device)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.rand(64, 3, 32, 32, device=device) * 2 - 1
    y = torch.randint(0, 10, (64,), device=device)
    ref = resnet18_fp64_step(state, x, y)[1]
    g0 = _grads(m, state, x, y)
    assert_fused_no_worse(g0, g0, ref)  # the native step itself is within the bounds
    drift = {k: (v * 1.01 if ("bn" in k or "downsample.1" in k) and k.endswith("weight") else v)
             for k, v in state.items()}
    g1 = _grads(m, drift, x, y)
    with pytest.raises(AssertionError):
        assert_fused_no_worse(g1, g0, ref)
