#!/usr/bin/env python3
"""A/B of the tgemm pointwise conv path (csrc/tgemm.hip) against the previous path (MIOpen
1x1 convs) on the ResNet-50/152 bottleneck shapes, per batch size.  (The small-map family this
tool also measured in round 3, profiles/r3/tg_bench.md, was deleted in round 6.)

    python tools/tg_bench.py [--batches 64 512] [--iters 50]

Times forward + backward (grad-x and grad-W) of one GemmConv2d, hipGraph-captured so that
the numbers are launch-overhead-free like the training step; prints one JSON line per
(shape, batch, path)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from network_distributed_pytorch_amd.models.conv_gemm import GemmConv2d, ToeplitzBank  # noqa: E402
from network_distributed_pytorch_amd.ops import gemm_tuning, gradfinish, tgconv  # noqa: E402

SHAPES = {  # name: (C, H, W, Co, k, stride, pad)
    "r50.l1.pw_in": (256, 8, 8, 64, 1, 1, 0),
    "r50.l1.pw_out": (64, 8, 8, 256, 1, 1, 0),
    "r50.l2.pw_in": (512, 4, 4, 128, 1, 1, 0),
    "r50.l3.pw_in": (1024, 2, 2, 256, 1, 1, 0),
    "r50.l3.pw_out": (256, 2, 2, 1024, 1, 1, 0),
}


def time_conv(shape, B, use_tg, iters):
    C, H, W, Co, k, s, p = shape
    tgconv._ON = use_tg
    tgconv._PLANS.clear()
    conv = GemmConv2d(C, Co, kernel_size=k, stride=s, padding=p, bias=False).cuda()
    conv.bank = ToeplitzBank()
    x = torch.randn(B, C, H, W, device="cuda", requires_grad=True)
    g = torch.randn(B, Co, (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1, device="cuda")

    def step():
        x.grad = None
        conv.weight.grad = None
        conv(x).backward(g)

    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    torch.cuda.synchronize()
    for _ in range(5):
        graph.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[64, 512])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", nargs="*", default=None)
    a = ap.parse_args()
    gemm_tuning.enable()
    assert gradfinish.enabled()
    for name, shape in SHAPES.items():
        if a.shapes and name not in a.shapes:
            continue
        for B in a.batches:
            row = {"shape": name, "batch": B}
            for tag, on in (("tgemm", True), ("previous", False)):
                row[f"{tag}_us"] = round(time_conv(shape, B, on, a.iters), 2)
            row["speedup"] = round(row["previous_us"] / row["tgemm_us"], 3)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
