"""PowerSGD reducer micro-benchmark: one fused optimizer step (P, orth, Q, update + rank-1)
of a model's parameter set, captured in a hipGraph and replayed; µs per step for each arm.

  python tools/psgd_bench.py [resnet18|resnet50|resnet152|distilbert] [rank] [reps]

Arms: ``fused`` (in-kernel split-K finish, csrc/powersgd.hip PFin/QFin/R1Step) and ``seg``
(separate seg_reduce / rank1_step launches).  Gradients are random (the reducer's cost does
not depend on their values).  One JSON line per arm."""
import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd.models import build_model  # noqa: E402
from network_distributed_pytorch_amd.parallel.powersgd import PowerSGDOptimizer  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
    rank = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    arms = os.environ.get("PSGD_ARMS", "fused,seg,fused").split(",")
    for arm in arms:
        model = build_model(name, num_classes=1000 if name.startswith("resnet") else 2).to(dev)
        opt = PowerSGDOptimizer(model.parameters(), lr=1e-3, momentum=0.9, rank=rank)
        opt.buf.fused = arm == "fused" and opt.buf.fused
        grads = [torch.randn_like(p) for p in model.parameters()]

        def step():
            for p, g in zip(model.parameters(), grads):
                p.grad = g
            opt.step()

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        for _ in range(10):
            g.replay()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0.record()
        for _ in range(reps):
            g.replay()
        t1.record()
        torch.cuda.synchronize()
        us = t0.elapsed_time(t1) * 1000 / reps
        print(json.dumps({"model": name, "rank": rank, "arm": arm, "fused": opt.buf.fused, "us_per_step": round(us, 2),
                          "numel": sum(p.numel() for p in model.parameters())}), flush=True)


if __name__ == "__main__":
    main()
