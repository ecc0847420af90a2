"""ResNet-18 one training step, epilogue BN statistics on / off, each vs an fp64 CPU oracle:
mean / max L2-relative gradient error per arm, with the GEMM solution table off and on
(diagnoses an arm that is systematically less accurate vs rounding-state noise)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from network_distributed_pytorch_amd.models import build_resnet  # noqa: E402
from network_distributed_pytorch_amd.ops import conv as conv_mod, gemm_tuning  # noqa: E402
from tests._oracle import rel_err, resnet18_fp64_step  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
SEED = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dev = torch.device("cuda", 0)
torch.backends.cudnn.deterministic = True
torch.manual_seed(SEED)
m = build_resnet(18, 1000).to(dev)
state = {k: v.clone() for k, v in m.state_dict().items()}
x = torch.rand(B, 3, 32, 32, device=dev) * 2 - 1
y = torch.randint(0, 10, (B,), device=dev)
lr, gr = resnet18_fp64_step(state, x, y)
for table in (False, True):
    if table:
        gemm_tuning.enable()
    else:
        gemm_tuning.disable()
    for stats in (False, True):
        conv_mod.CONV_BN_STATS = stats
        conv_mod._STATS.clear()
        m.load_state_dict(state)
        m.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x), y)
        loss.backward()
        errs = {n: rel_err(p.grad, gr[n]) for n, p in m.named_parameters()}
        worst = sorted(errs.items(), key=lambda kv: -kv[1])[:3]
        print(f"seed={SEED} table={table} stats={stats}: loss err {abs(loss.item() - lr):.2e} mean {sum(errs.values()) / len(errs):.2e} "
              f"conv1 {errs['conv1.weight']:.2e} bn1.w {errs['bn1.weight']:.2e} worst {[(n, f'{e:.1e}') for n, e in worst]}",
              flush=True)
