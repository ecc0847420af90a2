"""Serial full-graph step vs eager for ResNet-18 (dense / PowerSGD): NaN / mismatch hunt.
Run under different env toggles (NDP_GRAD_ARENA, NDP_DEFER_GRADW) by the caller."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from network_distributed_pytorch_amd.models import build_resnet  # noqa: E402
from network_distributed_pytorch_amd.parallel.trainer import build_grad_sync  # noqa: E402
from network_distributed_pytorch_amd.utils.graph import StepRunner  # noqa: E402

torch.backends.cudnn.deterministic = True
g = torch.Generator(device="cpu").manual_seed(0)
batches = [(torch.randn(32, 3, 32, 32, generator=g).cuda(), torch.randint(0, 10, (32,), generator=g).cuda())
           for _ in range(3)]
for kind in ("dense", "powersgd"):
    res = {}
    for mode in ("none", "full"):
        torch.manual_seed(3)
        model = build_resnet(18, 10).cuda()
        sync = build_grad_sync(kind, model, lr=1e-3, momentum=0.9, rank=4, overlap=False)
        static = [batches[0][0].clone(), batches[0][1].clone()]

        def pre():
            sync.zero_grad()
            torch.nn.functional.cross_entropy(model(static[0]), static[1]).backward()
        runner = StepRunner(pre, sync, mode=mode, warmup=2, state_tensors=list(model.buffers()))
        norms = []
        for x, y in batches:
            static[0].copy_(x)
            static[1].copy_(y)
            runner()
            torch.cuda.synchronize()
            norms.append(sum(float(p.detach().double().norm()) for p in model.parameters()))
        res[mode] = ([p.detach().clone() for p in model.parameters()], norms)
    names = [n for n, _ in model.named_parameters()]
    bad = [n for n, a, b in zip(names, res["none"][0], res["full"][0]) if not torch.equal(a, b)]
    nan = [n for n, b in zip(names, res["full"][0]) if not torch.isfinite(b).all()]
    print(kind, "eager norms", [round(v, 6) for v in res["none"][1]], "graph norms",
          [round(v, 6) for v in res["full"][1]], "differ", len(bad), bad[:3], "nonfinite", nan[:3], flush=True)
