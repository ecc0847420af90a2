#!/usr/bin/env python3
"""Time fused (csrc/attention.hip) vs explicit attention fwd+bwd at the DistilBERT shape.

    python tools/attn_bench.py [--batch 16 --seq 512 --heads 12 --p 0.1]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.ops.attention import attention, attention_reference  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--p", type=float, default=0.1)
    a = ap.parse_args()
    dev = torch.device("cuda")
    q, k, v = (torch.randn(a.batch, a.seq, a.heads, 64, device=dev, requires_grad=True) for _ in range(3))
    mask = torch.ones(a.batch, a.seq, dtype=torch.int32, device=dev)
    mask[:, a.seq * 3 // 4:] = 0
    go = torch.randn_like(q)
    flops = 4 * a.batch * a.heads * a.seq * a.seq * 64   # fwd: 2 GEMMs
    for name, f in (("fused", lambda: attention(q, k, v, mask, a.p)),
                    ("explicit", lambda: attention_reference(q, k, v, mask, a.p))):
        tf = timeit(lambda: f())
        tb = timeit(lambda: torch.autograd.grad(f(), (q, k, v), go)) - tf
        print(f"{name:9s} fwd {tf:7.3f} ms ({flops / tf / 1e9:6.1f} TF/s)   bwd {tb:7.3f} ms "
              f"({2.5 * flops / tb / 1e9:6.1f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
