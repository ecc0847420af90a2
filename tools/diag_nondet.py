"""Which ResNet-18 gradients differ between two identical backward passes? (nondeterminism hunt)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from network_distributed_pytorch_amd.models import build_resnet  # noqa: E402
from network_distributed_pytorch_amd.ops import gemm_tuning  # noqa: E402

torch.backends.cudnn.deterministic = True
for tuned in (False, True):
    if tuned:
        gemm_tuning.enable()
    for fc_kind in ("native", "nn"):
        torch.manual_seed(0)
        m = build_resnet(18).cuda()
        if fc_kind == "nn":
            fc = torch.nn.Linear(512, 1000).cuda()
            fc.load_state_dict(m.fc.state_dict())
            m.fc = fc
        x = torch.randn(64, 3, 32, 32, device="cuda")
        y = torch.randint(0, 10, (64,), device="cuda")
        grads = []
        for _ in range(3):
            m.zero_grad(set_to_none=True)
            torch.nn.functional.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
            grads.append({n: p.grad.clone() for n, p in m.named_parameters()})
        names = [n for n, _ in m.named_parameters()][::-1]  # backward production order
        diff = [n for n in names if not all(torch.equal(grads[0][n], g[n]) for g in grads[1:])]
        print(f"tuned={tuned} fc={fc_kind}: {len(diff)} differ; first in backward order: {diff[:4]}", flush=True)
