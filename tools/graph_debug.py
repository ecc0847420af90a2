"""Bisect which part of the training step breaks hipGraph capture."""
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.models import resnet18  # noqa: E402
from network_distributed_pytorch_amd.parallel.trainer import build_grad_sync  # noqa: E402

dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = os.environ.get("BENCH", "1") == "1"


def attempt(stage, kind="powersgd"):
    torch.manual_seed(0)
    model = resnet18().to(dev)
    sync = build_grad_sync(kind, model)
    x = torch.randn(512, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (512,), device=dev)
    crit = torch.nn.CrossEntropyLoss()

    def body():
        if stage >= 1:
            sync.zero_grad()
        out = model(x)
        if stage >= 1:
            loss = crit(out, y)
            loss.backward()
        if stage >= 2:
            sync.step()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            body()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        print(f"stage {stage} ({kind}): capture OK", flush=True)
        return True
    except Exception:
        print(f"stage {stage} ({kind}): capture FAILED", flush=True)
        traceback.print_exc(limit=12)
        return False


for st in (0, 1, 2):
    if not attempt(st):
        break
