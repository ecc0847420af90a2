#!/usr/bin/env python3
"""Per-layer time of ResNet-18's Toeplitz-GEMM convs (layer3 / layer4) at batch argv[1]:
forward + backward of GemmConv2d (autograd, 20 calls in one hipGraph, tuned GEMM table on),
and for the 1x1 stride-2 downsamples the subsample-first variant (strided copy, then the
1x1 stride-1 Toeplitz on the compact map) to size the zero-row waste of the in-W_big stride."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd.models.conv_gemm import GemmConv2d  # noqa: E402
from network_distributed_pytorch_amd.ops import gemm_tuning  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
print("tuned GEMM table:", gemm_tuning.enable())
SHAPES = [("l3_3x3s2", 128, 256, 3, 2, 1, 4, 1), ("l3_ds1x1s2", 128, 256, 1, 2, 0, 4, 1),
          ("l3_3x3", 256, 256, 3, 1, 1, 2, 3), ("l4_3x3s2", 256, 512, 3, 2, 1, 2, 1),
          ("l4_ds1x1s2", 256, 512, 1, 2, 0, 2, 1), ("l4_3x3", 512, 512, 3, 1, 1, 1, 3)]


def timeit(fn, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


tot = 0.0
print("| conv | x | fwd+bwd us | subsample-first us |")
print("|---|---:|---:|---:|")
for name, cin, cout, k, s, p, hw, cnt in SHAPES:
    m = GemmConv2d(cin, cout, k, stride=s, padding=p, bias=False).to(dev)
    x = torch.randn(B, cin, hw, hw, device=dev, requires_grad=True)
    g = torch.randn_like(m(x))

    def fb():
        x.grad = None
        m.weight.grad = None
        m(x).backward(g)
    t = timeit(fb)
    alt = float("nan")
    if k == 1 and s > 1:
        m1 = GemmConv2d(cin, cout, 1, stride=1, padding=0, bias=False).to(dev)

        def fb2():
            x.grad = None
            m1.weight.grad = None
            m1(x[:, :, ::s, ::s].contiguous()).backward(g)
        alt = timeit(fb2)
    tot += cnt * t
    print(f"| {name} | {cnt} | {t:.1f} | {alt:.1f} |")
print(f"\nweighted fwd+bwd total: {tot:.0f} us")
