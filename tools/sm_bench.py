#!/usr/bin/env python3
"""Per-direction timing of the small-map conv kernels (csrc/smallconv.hip) on the ResNet-18
layer3 / layer4 shapes: forward, grad-x and grad-W launched on their own (plain operands, the
split-K slab sum included where the plan splits), hipGraph-captured so the numbers carry no
host overhead.  Prints one JSON line per (shape, batch, direction) with µs / launch and the
useful TFLOP/s (2 x batch x Co x C x (input, output) pixel pairs).

    python tools/sm_bench.py [--batches 64 512] [--iters 40]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from network_distributed_pytorch_amd.ops._ext import ext  # noqa: E402

SHAPES = {  # name: (C, H, W, Co, k, stride, pad)
    "r18.l3.conv": (256, 2, 2, 256, 3, 1, 1),
    "r18.l3.entry": (128, 4, 4, 256, 3, 2, 1),
    "r18.l3.ds": (128, 4, 4, 256, 1, 2, 0),
    "r18.l4.conv": (512, 1, 1, 512, 3, 1, 1),
    "r18.l4.entry": (256, 2, 2, 512, 3, 2, 1),
    "r18.l4.ds": (256, 2, 2, 512, 1, 2, 0),
}


def pairs(C, H, W, Co, k, s, p):
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    n = 0
    for oh in range(OH):
        for ow in range(OW):
            for kh in range(k):
                for kw in range(k):
                    ih, iw = oh * s - p + kh, ow * s - p + kw
                    n += 0 <= ih < H and 0 <= iw < W
    return n, OH, OW


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn()
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / (5 * iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[64, 512])
    ap.add_argument("--iters", type=int, default=40)
    args = ap.parse_args()
    X = ext()
    for name, (C, H, W, Co, k, s, p) in SHAPES.items():
        npairs, OH, OW = pairs(C, H, W, Co, k, s, p)
        gl = [C, H, W, Co, k, k, s, p]
        for B in args.batches:
            cls, fs, ds, ws = X.sm_plan(gl, B)
            if cls < 0:
                continue
            x = torch.randn(B, C, H, W, device="cuda")
            w = torch.randn(Co, C, k, k, device="cuda") * 0.05
            dy = torch.randn(B, Co, OH, OW, device="cuda")
            y = torch.empty_like(dy)
            dx = torch.empty_like(x)
            fpart = torch.empty(max(fs, 1) * y.numel(), device="cuda")
            dpart = torch.empty(max(ds, 1) * x.numel(), device="cuda")
            wout = torch.empty(max(ws, 1) * w.numel(), device="cuda")
            flop = 2.0 * B * Co * C * npairs
            runs = {
                "fwd": lambda: X.sm_fwd(x, w, y, gl, fpart if fs > 1 else None, False),
                "dgrad": lambda: X.sm_dgrad(dy, w, dx, gl, dpart if ds > 1 else None, None, False),
                "wgrad": lambda: X.sm_wgrad(x, dy, wout, gl),
            }
            for d, fn in runs.items():
                us = timed(fn, args.iters)
                print(json.dumps({"shape": name, "batch": B, "dir": d, "us": round(us, 2),
                                  "tflops": round(flop / us / 1e6, 1),
                                  "splits": {"fwd": fs, "dgrad": ds, "wgrad": ws}[d]}), flush=True)


if __name__ == "__main__":
    main()
