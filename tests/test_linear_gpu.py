"""Native Linear bias gradient (csrc/linear.hip column sums) vs fp64; graph replay."""
import pytest
import torch

from network_distributed_pytorch_amd.ops.linear import Linear

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(16, 512, 768), (8192, 3072), (5, 4), (37, 132)])
def test_linear_grads_vs_fp64(device, shape):
    torch.manual_seed(0)
    k = 96
    lin = Linear(k, shape[-1]).to(device)
    x = torch.randn(*shape[:-1], k, device=device, requires_grad=True)
    g = torch.randn(*shape, device=device)
    lin(x).backward(g)
    ref_db = g.double().reshape(-1, shape[-1]).sum(0)
    err = (lin.bias.grad.double() - ref_db).abs().max().item()
    assert err <= 1e-5 * max(1.0, ref_db.abs().max().item()) * (g.numel() / shape[-1]) ** 0.5, err
    ref = torch.nn.Linear(k, shape[-1]).to(device)
    ref.load_state_dict(lin.state_dict())
    x2 = x.detach().clone().requires_grad_(True)
    ref(x2).backward(g)
    torch.testing.assert_close(x.grad, x2.grad)
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad)


def test_linear_bias_grad_graph_replay(device):
    torch.manual_seed(1)
    lin = Linear(64, 3072).to(device)
    xs = [torch.randn(8192, 64, device=device) for _ in range(3)]
    gs = [torch.randn(8192, 3072, device=device) for _ in range(3)]
    sx, sg = xs[0].clone(), gs[0].clone()

    def fb():
        lin.bias.grad = None
        lin.weight.grad = None
        lin(sx).backward(sg)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fb()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        fb()
    for i in range(9):
        sx.copy_(xs[i % 3])
        sg.copy_(gs[i % 3])
        graph.replay()
        torch.cuda.synchronize()
        ref = gs[i % 3].double().sum(0)
        assert (lin.bias.grad.double() - ref).abs().max().item() < 1e-3, i


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(8192, 768, 3072), (100, 64, 256), (3, 8, 12)])
def test_linear_gelu_fused_backward_vs_fp64(device, shape):
    """gelu(linear(x)): one native pass for dh = da * gelu'(h) and the bias column sums."""
    from network_distributed_pytorch_amd.ops.linear import linear_gelu

    M, K, N = shape
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=device, requires_grad=True)
    w = (torch.randn(N, K, device=device) / K ** 0.5).requires_grad_(True)
    b = torch.randn(N, device=device, requires_grad=True)
    y = linear_gelu(x, w, b)
    x64, w64, b64 = (t.detach().double().requires_grad_(True) for t in (x, w, b))
    y64 = torch.nn.functional.gelu(torch.nn.functional.linear(x64, w64, b64))
    torch.testing.assert_close(y.double(), y64, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    y64.backward(g.double())
    for got, ref, name in ((x.grad, x64.grad, "dx"), (w.grad, w64.grad, "dw"), (b.grad, b64.grad, "db")):
        scale = ref.abs().max().item()
        torch.testing.assert_close(got.double(), ref, rtol=1e-3, atol=2e-5 * scale * M ** 0.5, msg=name)
