#!/usr/bin/env python3
"""Direct fp32-MFMA conv kernels vs MIOpen on ResNet-18's CIFAR shapes (batch argv[1], default 512).

Per shape: forward, grad-input and grad-weight time of the csrc/conv.hip kernels and of
MIOpen (F.conv2d / aten.convolution_backward), each timed as 20 calls in one hipGraph.
"""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd import ops  # noqa: E402
from network_distributed_pytorch_amd.ops.conv import direct_plan  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
X = ops.ext()

SHAPES = [("stem7x7s2", 3, 64, 7, 2, 3, 32, 1), ("l1_3x3", 64, 64, 3, 1, 1, 8, 4),
          ("l2_3x3s2", 64, 128, 3, 2, 1, 8, 1), ("l2_3x3", 128, 128, 3, 1, 1, 4, 3)]


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


print("| conv | x | GF | MIOpen fwd | direct fwd | MIOpen dgrad | direct dgrad | MIOpen wgrad | direct wgrad | "
      "direct fwd TF | direct wgrad TF |")
print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
tot = {"mi": 0.0, "di": 0.0}
for name, cin, cout, k, s, p, hw, cnt in SHAPES:
    x = torch.randn(B, cin, hw, hw, device=dev)
    w = torch.randn(cout, cin, k, k, device=dev) * 0.05
    plan = direct_plan(x, w, s, p)
    geom, _, wi, dd, ksf, ksd = plan
    y = F.conv2d(x, w, stride=s, padding=p)
    g = torch.randn_like(y)
    yd = torch.empty_like(y)
    dx = torch.empty_like(x)
    dw = torch.empty_like(w)
    part = torch.empty((B // wi) * w.numel(), device=dev)
    pf = torch.empty(ksf * y.numel(), device=dev) if ksf > 1 else None
    pd = torch.empty(ksd * x.numel(), device=dev) if ksd > 1 else None
    oh = y.shape[2]
    fl = 2.0 * B * oh * oh * cout * cin * k * k
    t_mf = timeit(lambda: F.conv2d(x, w, stride=s, padding=p))
    t_md = timeit(lambda: torch.ops.aten.convolution_backward(g, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                              [True, False, False]))
    t_mw = timeit(lambda: torch.ops.aten.convolution_backward(g, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                              [False, True, False]))
    t_df = timeit(lambda: X.conv_fwd(x, w, yd, list(geom), pf))
    t_dd = timeit(lambda: X.conv_dgrad(g, w, dx, list(geom), pd)) if dd else float("nan")
    t_dw = timeit(lambda: X.conv_wgrad(x, g, part, dw, list(geom)))
    X.conv_fwd(x, w, yd, list(geom), pf)
    err = (yd - y).abs().max().item() / y.abs().max().item()
    need_dx = name != "stem7x7s2"
    tot["mi"] += cnt * (t_mf + (t_md if need_dx else 0) + t_mw)
    tot["di"] += cnt * (t_df + ((t_dd if dd else t_md) if need_dx else 0) + t_dw)
    print(f"| {name} | {cnt} | {fl / 1e9:.2f} | {t_mf:.1f} | {t_df:.1f} | {t_md:.1f} | {t_dd:.1f} | {t_mw:.1f} | "
          f"{t_dw:.1f} | {fl / t_df / 1e6:.1f} | {fl / t_dw / 1e6:.1f} |  (rel err fwd {err:.1e}, ksplit {ksf}/{ksd}, wgrad imgs {wi})")
print(f"\nper ResNet-18 step (these shapes, x count, grad-x only where needed): MIOpen {tot['mi']:.0f} us, "
      f"direct {tot['di']:.0f} us")
