"""Diagnostic: the BN kernels in isolation against plain streaming ops over the same bytes,
run eagerly 20x each — read the per-kernel durations from
    rocprofv3 --kernel-trace --stats -d OUT -- python tools/diag/bn_micro.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from network_distributed_pytorch_amd.ops.batchnorm import BatchNormAct2d  # noqa: E402


def timed(fn, iters=20):
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return 0.0


for shape in [(512, 128, 4, 4), (512, 256, 2, 2), (512, 512, 1, 1), (64, 128, 4, 4), (512, 64, 8, 8)]:
    C = shape[1]
    bn = BatchNormAct2d(C).cuda()
    x = torch.randn(shape, device="cuda")
    r = torch.randn(shape, device="cuda")
    g = torch.randn(shape, device="cuda")
    out = torch.empty_like(x)
    y = bn(x, residual=r, relu=True)
    xx = x.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True)

    def fwd():
        bn(x, residual=r, relu=True)

    yy = bn(xx, residual=rr, relu=True)

    def bwd():
        torch.autograd.grad(yy, (xx, rr), g, retain_graph=True)

    def stream3():
        torch.add(x, r, out=out)

    timed(fwd), timed(bwd), timed(stream3)
    print(shape, "done", flush=True)
