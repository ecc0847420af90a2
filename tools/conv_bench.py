#!/usr/bin/env python3
"""Per-shape timing of ResNet-18's convolutions on MI355X (batch 512, 32x32 input, fp32).

For every distinct conv of the model: MIOpen forward / backward-data / backward-weight time
(autograd, cudnn.benchmark) and, as a reference point, the time of the same FLOPs as a
plain hipBLASLt GEMM (M = N*OH*OW, N = Cout, K = Cin*kh*kw).  Used to decide which convs
deserve hand-written kernels.
"""
import json
import sys

import torch
import torch.nn.functional as F

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512

# (name, cin, cout, k, stride, pad, in_hw, count_in_resnet18)
SHAPES = [
    ("stem7x7s2", 3, 64, 7, 2, 3, 32, 1),
    ("l1_3x3", 64, 64, 3, 1, 1, 8, 4),
    ("l2_3x3s2", 64, 128, 3, 2, 1, 8, 1),
    ("l2_ds1x1s2", 64, 128, 1, 2, 0, 8, 1),
    ("l2_3x3", 128, 128, 3, 1, 1, 4, 3),
    ("l3_3x3s2", 128, 256, 3, 2, 1, 4, 1),
    ("l3_ds1x1s2", 128, 256, 1, 2, 0, 4, 1),
    ("l3_3x3", 256, 256, 3, 1, 1, 2, 3),
    ("l4_3x3s2", 256, 512, 3, 2, 1, 2, 1),
    ("l4_ds1x1s2", 256, 512, 1, 2, 0, 2, 1),
    ("l4_3x3", 512, 512, 3, 1, 1, 1, 3),
]


def timeit(fn, iters=20):
    """GPU time per call: `iters` calls captured in one hipGraph (no host launch overhead)."""
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
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


rows = []
tot = {"fwd": 0.0, "bwd": 0.0, "gemm": 0.0}
for name, cin, cout, k, s, p, hw, cnt in SHAPES:
    x = torch.randn(B, cin, hw, hw, device=dev)
    w = torch.randn(cout, cin, k, k, device=dev)
    y = F.conv2d(x, w, stride=s, padding=p)
    oh = y.shape[2]
    g = torch.randn_like(y)
    t_f = timeit(lambda: F.conv2d(x, w, stride=s, padding=p))

    def bwd_only():
        torch.ops.aten.convolution_backward(g, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                            [True, True, False])
    t_fb = t_f + timeit(bwd_only)
    M, N, K = B * oh * oh, cout, cin * k * k
    A = torch.randn(M, K, device=dev)
    Bm = torch.randn(K, N, device=dev)
    t_g = timeit(lambda: A @ Bm)
    fl = 2.0 * M * N * K

    t_uf = t_ufb = 0.0
    rows.append(dict(name=name, count=cnt, out_hw=oh, M=M, N=N, K=K, gflop=fl / 1e9, fwd_us=t_f,
                     bwd_us=t_fb - t_f, gemm_us=t_g, fwd_tflops=fl / t_f / 1e6, gemm_tflops=fl / t_g / 1e6,
                     unf_fwd_us=t_uf, unf_bwd_us=t_ufb - t_uf))
    tot.setdefault("unf_fwd", 0.0)
    tot.setdefault("unf_bwd", 0.0)
    tot["unf_fwd"] += cnt * t_uf
    tot["unf_bwd"] += cnt * (t_ufb - t_uf)
    tot["fwd"] += cnt * t_f
    tot["bwd"] += cnt * (t_fb - t_f)
    tot["gemm"] += cnt * 3 * t_g

print("| conv | x | out | M x N x K | GF | fwd us | bwd us | unfold+GEMM fwd us | unfold+GEMM bwd us | "
      "same-FLOP GEMM us | fwd TF | GEMM TF |")
print("|---|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|---:|")
for r in rows:
    print(f"| {r['name']} | {r['count']} | {r['out_hw']} | {r['M']}x{r['N']}x{r['K']} | {r['gflop']:.2f} | "
          f"{r['fwd_us']:.1f} | {r['bwd_us']:.1f} | {r['unf_fwd_us']:.1f} | {r['unf_bwd_us']:.1f} | "
          f"{r['gemm_us']:.1f} | {r['fwd_tflops']:.1f} | {r['gemm_tflops']:.1f} |")
print(f"\nweighted totals per step: fwd {tot['fwd']:.0f} us, bwd {tot['bwd']:.0f} us, "
      f"3x same-FLOP GEMMs {tot['gemm']:.0f} us")
print(json.dumps(tot))
