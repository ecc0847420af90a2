#!/usr/bin/env python3
"""Step-by-step parameter divergence between two eager runs and a hipGraph run (ResNet-18)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd.models import build_resnet  # noqa: E402
from network_distributed_pytorch_amd.parallel.trainer import build_grad_sync  # noqa: E402
from network_distributed_pytorch_amd.utils.graph import StepRunner  # noqa: E402

dev = torch.device("cuda", 0)
kind = sys.argv[1] if len(sys.argv) > 1 else "powersgd"
g = torch.Generator(device="cpu").manual_seed(0)
batches = [(torch.randn(32, 3, 32, 32, generator=g).to(dev), torch.randint(0, 10, (32,), generator=g).to(dev))
           for _ in range(4)]


def run(mode):
    torch.manual_seed(3)
    model = build_resnet(18, 10).to(dev)
    sync = build_grad_sync(kind, model, lr=float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3, momentum=0.9, rank=4)
    static = [batches[0][0].clone(), batches[0][1].clone()]

    def pre():
        sync.zero_grad()
        torch.nn.functional.cross_entropy(model(static[0]), static[1]).backward()

    runner = StepRunner(pre, sync, mode=mode, warmup=2)
    snaps = []
    if mode == "none":
        for _ in range(2):
            runner()
            snaps.append(torch.cat([p.detach().flatten() for p in model.parameters()]).clone())
    for x, y in batches:
        static[0].copy_(x)
        static[1].copy_(y)
        runner()
        torch.cuda.synchronize()
        snaps.append(torch.cat([p.detach().flatten() for p in model.parameters()]).clone())
    return snaps


a = run("none")
b = run("none")
c = run("full")
print("eager-vs-eager per step:", [f"{(x - y).abs().max().item():.2e}" for x, y in zip(a, b)])
print("eager-vs-graph (last 4 steps):", [f"{(x - y).abs().max().item():.2e}" for x, y in zip(a[2:], c)])
