"""Diagnostic: one native conv (ops/conv.py direct path) forward / grad-x / grad-W, repeated with
the allocator's free blocks poisoned between runs; prints which outputs are not bitwise stable.
    python tools/diag/conv_repeat.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from network_distributed_pytorch_amd.models.conv_gemm import GemmConv2d  # noqa: E402

SHAPES = [(64, 8, 8, 64, 3, 1, 1), (64, 8, 8, 128, 3, 2, 1), (128, 4, 4, 128, 3, 1, 1), (64, 8, 8, 128, 1, 2, 0),
          (3, 32, 32, 64, 7, 2, 3)]


def poison(kind):
    t = torch.empty(256 << 20, device="cuda")
    t.fill_(float("nan")) if kind == 0 else t.uniform_(-1e3, 1e3)
    del t


for (C, H, W, Co, k, s, p) in SHAPES:
    for B in (2, 3, 4, 8, 32):
        torch.manual_seed(0)
        conv = GemmConv2d(C, Co, kernel_size=k, stride=s, padding=p, bias=False).cuda()
        x0 = torch.randn(B, C, H, W, device="cuda")
        OH = (H + 2 * p - k) // s + 1
        g = torch.randn(B, Co, OH, (W + 2 * p - k) // s + 1, device="cuda")
        res = []
        for kind in (0, 1, 0):
            poison(kind)
            x = x0.clone().requires_grad_(True)
            conv.weight.grad = None
            y = conv(x)
            poison(kind)
            y.backward(g)
            torch.cuda.synchronize()
            res.append((y.detach().clone(), x.grad.clone(), conv.weight.grad.clone()))
        bad = [n for i, n in enumerate(("fwd", "dgrad", "wgrad"))
               if not (torch.equal(res[0][i], res[1][i]) and torch.equal(res[0][i], res[2][i]))]
        print((C, H, W, Co, k, s, p), "B", B, "UNSTABLE " + ",".join(bad) if bad else "stable", flush=True)
