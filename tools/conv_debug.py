#!/usr/bin/env python3
"""Per-parameter gradient error of ResNet-18 conv paths vs an fp64 CPU oracle."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd.models import build_resnet  # noqa: E402
from network_distributed_pytorch_amd.models.conv_gemm import GemmConv2d  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
torch.manual_seed(0)
models = {}
base = build_resnet(18, 10, gemm_convs=True).to(dev)
sd = base.state_dict()
for name, (gemm, direct) in {"direct+toeplitz": (True, True), "toeplitz": (True, False), "miopen": (False, False)}.items():
    m = build_resnet(18, 10, gemm_convs=False).to(dev)
    m.load_state_dict(sd)
    for mod in m.modules():
        if isinstance(mod, GemmConv2d):
            mod.gemm, mod.direct = gemm, direct
    models[name] = m
ref = build_resnet(18, 10, gemm_convs=False).double()
ref.load_state_dict(sd)
EVAL = len(sys.argv) > 2 and sys.argv[2] == "eval"
if EVAL:  # BN as a fixed affine map: no batch-statistics amplification of rounding noise
    for m in list(models.values()) + [ref]:
        m.eval()
x = torch.randn(B, 3, 32, 32)
y = torch.randint(0, 10, (B,))
F.cross_entropy(ref(x.double()), y).backward()
for name, m in models.items():
    F.cross_entropy(m(x.to(dev)), y.to(dev)).backward()
rows = []
for (pn, pr) in ref.named_parameters():
    g = pr.grad
    errs = {}
    for name, m in models.items():
        pa = dict(m.named_parameters())[pn]
        errs[name] = (pa.grad.cpu().double() - g).abs().max().item() / (g.abs().max().item() + 1e-30)
    rows.append((pn, errs))
print("param | " + " | ".join(models))
for pn, errs in rows:
    if pn.endswith("weight") and ("conv" in pn or "downsample.0" in pn or pn == "fc.weight"):
        print(pn, " | ".join(f"{errs[k]:.2e}" for k in models))
