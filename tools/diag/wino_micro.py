"""Winograd layer1 conv (forward + grad-x) at batch argv[1], a few eager iterations: a small
program to run under rocprofv3 --pmc for per-kernel stall counters."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd.ops.conv import conv2d_direct  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
x = torch.randn(B, 64, 8, 8, device=dev, requires_grad=True)
w = torch.randn(64, 64, 3, 3, device=dev, requires_grad=True)
for _ in range(5):
    y = conv2d_direct(x, w, 1, 1)
    y.backward(torch.ones_like(y))
torch.cuda.synchronize()
print("ok")
