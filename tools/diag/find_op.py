"""Which autograd node launches a given ATen op inside a ResNet step (torch.profiler CPU
events: the op's enclosing ``autograd::engine::evaluate_function`` / Python function).
  python tools/diag/find_op.py --op aten::add --global-batch 64"""
import argparse

import torch
import torch.nn.functional as F

from network_distributed_pytorch_amd.models import build_resnet


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="aten::add")
    ap.add_argument("--global-batch", type=int, default=64)
    ap.add_argument("--model", default="resnet18")
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = build_resnet(int(a.model.replace("resnet", "")), 1000).to(dev)
    x = torch.rand(a.global_batch, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (a.global_batch,), device=dev)
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        F.cross_entropy(m(x), y).backward()
    torch.cuda.synchronize()
    m.zero_grad(set_to_none=True)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        F.cross_entropy(m(x), y).backward()
        torch.cuda.synchronize()
    for e in prof.events():
        if e.name != a.op:
            continue
        chain, p = [], e.cpu_parent
        while p is not None:
            chain.append(p.name)
            p = p.cpu_parent
        print(a.op, [tuple(s) for s in e.input_shapes] if e.input_shapes else "", "<-", " <- ".join(chain[:4]))


if __name__ == "__main__":
    main()
