"""Direct-conv split-K paths (forward UPS = 1, 1x1/2 grad-x UPS = 2) against ATen, printing the
first mismatches: python tools/diag/splitk_fin_check.py [batch]."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd.ops._ext import ext  # noqa: E402

X = ext()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
torch.manual_seed(0)
for (C, H, Co, k, s, p) in [(128, 4, 256, 1, 2, 0), (64, 8, 128, 1, 2, 0), (64, 8, 64, 3, 1, 1), (128, 4, 128, 3, 1, 1)]:
    geom = [C, H, H, Co, k, k, s, p]
    x = torch.randn(B, C, H, H, device=dev)
    w = torch.randn(Co, C, k, k, device=dev)
    y = F.conv2d(x, w, stride=s, padding=p)
    dy = torch.randn_like(y)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=s, padding=p)
    part = torch.empty(16 * max(x.numel(), y.numel()), device=dev)
    dx = torch.full_like(x, float("nan"))
    left = X.conv_dgrad(dy, w, dx, geom, part)
    err = (dx - dx_ref).abs().max().item() if left == 1 else float("nan")
    yy = torch.full_like(y, float("nan"))
    lf = X.conv_fwd(x, w, yy, geom, part)
    erry = (yy - y).abs().max().item() if lf == 1 else float("nan")
    print(f"geom {geom} B {B}: dgrad left {left} err {err:.3e} | fwd left {lf} err {erry:.3e}", flush=True)
    if left == 1 and err > 1e-2:
        bad = ((dx - dx_ref).abs() > 1e-2).nonzero()[:6].tolist()
        print("  first bad dx idx", bad, "got", [dx[tuple(i)].item() for i in bad], "ref",
              [dx_ref[tuple(i)].item() for i in bad])
