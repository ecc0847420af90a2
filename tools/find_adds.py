#!/usr/bin/env python3
"""Which Python frames launch the non-native elementwise kernels of one ResNet-18 r=4 step (eager)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import argparse  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    args = bench.parse(["--graph-mode", "none", "--no-supervise"])
    wl = bench.Workload(args, torch.device("cuda", 0), 1, 0)
    step = wl.make_step(a.batch)
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA],
                                with_stack=True) as prof:
        step(3)
        torch.cuda.synchronize()
    for ev in prof.events():
        if ev.name in ("aten::add", "aten::add_", "aten::copy_", "aten::fill_", "aten::zero_", "aten::sum", "aten::mul_"):
            st = [f for f in (ev.stack or []) if "network_distributed" in f or "bench.py" in f][:4]
            print(ev.name, [tuple(i) for i in ev.input_shapes][:2] if ev.input_shapes else "", st)


if __name__ == "__main__":
    main()
