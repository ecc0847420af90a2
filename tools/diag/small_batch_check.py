"""Diagnostic: ResNet-18 forward + backward at a tiny batch, run repeatedly with the caching
allocator's free blocks poisoned (NaN / random) in between; reports every module output and
parameter gradient that is not bitwise repeatable (a kernel reading memory it does not own).
    python tools/diag/small_batch_check.py [B ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from network_distributed_pytorch_amd.models import build_model  # noqa: E402


def poison(kind):
    t = torch.empty(256 << 20, device="cuda") if kind else None
    if kind == "nan":
        t.fill_(float("nan"))
    elif kind == "rand":
        t.uniform_(-1e3, 1e3)
    del t


def run(model, x, y, kind):
    outs = {}
    hooks = [m.register_forward_hook(lambda m, i, o, n=n: outs.__setitem__(n, o.detach().clone()))
             for n, m in model.named_modules() if n and not any(True for _ in m.children())]
    poison(kind)
    model.zero_grad(set_to_none=True)
    loss = F.cross_entropy(model(x), y)
    poison(kind)
    loss.backward()
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    return outs, {n: p.grad.clone() for n, p in model.named_parameters()}


for B in [int(a) for a in sys.argv[1:]] or [2, 4]:
    torch.manual_seed(0)
    model = build_model("resnet18", 10).cuda()
    x = torch.randn(B, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (B,), device="cuda")
    state = {k: v.clone() for k, v in model.state_dict().items()}
    res = []
    for kind in ("nan", "rand", "nan"):
        model.load_state_dict(state)
        res.append(run(model, x, y, kind))
    bad = False
    for n in res[0][0]:
        a, b = res[0][0][n], res[1][0][n]
        if not torch.equal(a, b) or torch.isnan(a).any():
            print(f"B={B} forward output differs: {n} nan={torch.isnan(a).any().item()} "
                  f"maxdiff={(a - b).abs().max().item()}", flush=True)
            bad = True
            break
    for n in reversed(list(res[0][1])):
        a, b = res[0][1][n], res[1][1][n]
        if not torch.equal(a, b) or torch.isnan(a).any():
            print(f"B={B} grad differs: {n} nan={torch.isnan(a).any().item()} maxdiff={(a - b).abs().max().item()}",
                  flush=True)
            bad = True
            break
    print(f"B={B}", "NOT REPEATABLE" if bad else "repeatable", flush=True)
