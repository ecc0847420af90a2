#!/usr/bin/env python3
"""One tgemm conv direction in a loop (eager), for kernel traces / PMC passes of the GEMM itself.

    python tools/tg_micro.py --shape r50.l1.pw_in --batch 512 --dir fwd --iters 20
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from network_distributed_pytorch_amd.ops._ext import ext  # noqa: E402
from tools.tg_bench import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="r50.l1.pw_in")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--dir", default="all", choices=["fwd", "dgrad", "wgrad", "all"])
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C, H, W, Co, k, s, p = SHAPES[a.shape]
    geom = [C, H, W, Co, k, k, s, p]
    B = a.batch
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    cls, fs, ds, ws = ext().tg_plan(geom, B)
    assert cls >= 0, "no tgemm path"
    x = torch.randn(B, C, H, W, device="cuda")
    w = torch.randn(Co, C, k, k, device="cuda")
    y = torch.empty(B, Co, OH, OW, device="cuda")
    dy = torch.randn_like(y)
    dx = torch.empty_like(x)
    dw = torch.empty(Co * OH * OW, C * H * W, device="cuda") if cls == 1 else torch.empty_like(w)
    sc = lambda n, numel: torch.empty(n * numel, device="cuda") if n > 1 else None  # noqa: E731
    pf, pd, pw = sc(fs, y.numel()), sc(ds, x.numel()), sc(ws, dw.numel())
    for _ in range(a.iters):
        if a.dir in ("fwd", "all"):
            ext().tg_fwd(x, w, y, geom, pf, False)
        if a.dir in ("dgrad", "all"):
            ext().tg_dgrad(dy, w, dx, geom, pd, None, False)
        if a.dir in ("wgrad", "all"):
            ext().tg_wgrad(x, dy, dw, geom, pw, False)
    torch.cuda.synchronize()
    print("ok", a.shape, B, "splits", fs, ds, ws)


if __name__ == "__main__":
    main()
