"""GPU micro-probe: flag_signal / flag_wait kernels eagerly and inside a replayed graph."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.ops import ext  # noqa: E402

X = ext()
dev = torch.device("cuda", 0)
f = torch.zeros(16, dtype=torch.int32, device=dev)
for _ in range(10):
    X.flag_signal(f, 0)
torch.cuda.synchronize()
print("eager x10 signal ->", f[0].item(), flush=True)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.graph(g, stream=s):
    X.flag_signal(f, 1)
    X.flag_signal(f, 1)
    X.flag_signal(f, 2)
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
print("graph x5 replay (2 signals on [1], 1 on [2]) ->", f[1].item(), f[2].item(), flush=True)
# eager wait after signal
X.flag_signal(f, 3)
X.flag_wait(f, 3, 4, 5, 1 << 20)
torch.cuda.synchronize()
print("signal+wait: ctr", f[3].item(), "seen", f[4].item(), "err", f[5].item(), flush=True)
# plain add_ in a graph for comparison
t = torch.zeros(1, device=dev)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2, stream=s):
    t.add_(1)
for _ in range(5):
    g2.replay()
torch.cuda.synchronize()
print("graph add_ x5 ->", t.item(), flush=True)
