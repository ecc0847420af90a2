"""test_deferred_gradw_finishing_is_bitwise[64] diagnosis: which grads differ between runs?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from network_distributed_pytorch_amd.models import build_resnet  # noqa: E402
from network_distributed_pytorch_amd.ops import gradfinish  # noqa: E402

torch.backends.cudnn.deterministic = True
runs = {}
for tag, defer in (("nodefer1", False), ("defer1", True), ("nodefer2", False), ("defer2", True)):
    gradfinish._ENABLED = defer
    torch.manual_seed(3)
    m = build_resnet(18, 10).cuda()
    x = torch.randn(64, 3, 32, 32, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    m(x).square().mean().backward()
    torch.cuda.synchronize()
    runs[tag] = (list(n for n, _ in m.named_parameters()), [p.grad.clone() for p in m.parameters()])
names = runs["nodefer1"][0][::-1]
for a, b in (("nodefer1", "nodefer2"), ("defer1", "defer2"), ("nodefer1", "defer1")):
    ga, gb = runs[a][1][::-1], runs[b][1][::-1]
    diff = [(n, float((x - y).abs().max())) for n, x, y in zip(names, ga, gb) if not torch.equal(x, y)]
    print(a, "vs", b, len(diff), "differ; first (backward order):", diff[:4], flush=True)
