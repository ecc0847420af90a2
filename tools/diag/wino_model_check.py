"""ResNet-18 one training step (batch argv[1]) under the four (Winograd, epilogue BN statistics)
arms vs an fp64 CPU oracle of the same model: L2-relative gradient error per arm, for the stem
and a few deeper layers (diagnoses whether an arm is inaccurate or only differently rounded)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd.models import build_resnet  # noqa: E402
from network_distributed_pytorch_amd.ops import conv as conv_mod  # noqa: E402
from network_distributed_pytorch_amd.ops._ext import ext  # noqa: E402
from network_distributed_pytorch_amd.ops.conv import set_winograd  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = build_resnet(18, 1000).to(dev)
state = {k: v.clone() for k, v in m.state_dict().items()}
x = torch.rand(B, 3, 32, 32, device=dev) * 2 - 1
y = torch.randint(0, 10, (B,), device=dev)
ref = build_resnet(18, 1000, fused_bn=False, gemm_convs=False).double()
ref.load_state_dict({k: v.cpu() for k, v in state.items()})
F.cross_entropy(ref(x.double().cpu()), y.cpu()).backward()
rg = {n: p.grad for n, p in ref.named_parameters()}
names = ["conv1.weight", "layer1.0.conv1.weight", "layer1.1.conv2.weight", "layer2.0.conv1.weight", "fc.weight"]
arms = {}
for wino in (True, False):
    for stats in (True, False):
        set_winograd(wino)
        conv_mod.CONV_BN_STATS = stats
        conv_mod._STATS.clear()
        m.load_state_dict(state)
        m.zero_grad(set_to_none=True)
        F.cross_entropy(m(x), y).backward()
        g = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}
        arms[(wino, stats)] = g
        errs = [f"{n.split('.weight')[0]}={((g[n] - rg[n]).norm() / rg[n].norm()).item():.2e}" for n in names]
        print(f"wino={wino} stats={stats}: vs fp64 " + " ".join(errs))
for a in arms:
    for b in arms:
        if a < b:
            d = ((arms[a]['conv1.weight'] - arms[b]['conv1.weight']).norm() / rg['conv1.weight'].norm()).item()
            print(f"{a} vs {b}: conv1 L2-rel {d:.2e}")
