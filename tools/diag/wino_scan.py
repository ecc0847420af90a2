"""Winograd layer1-shape forward timing vs input channels (per-chunk slope / fixed intercept),
batch argv[1]; each row: Cin, Cout, µs per launch (graph-captured, 50 launches)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd.ops._ext import ext  # noqa: E402
from network_distributed_pytorch_amd.ops.conv import set_winograd  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)


def timeit(fn, iters=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


for cin, cout in [(64, 64), (128, 64), (256, 64), (512, 64), (64, 128), (128, 128)]:
    x = torch.randn(B, cin, 8, 8, device=dev)
    w = torch.randn(cout, cin, 3, 3, device=dev)
    y = torch.empty(B, cout, 8, 8, device=dev)
    u = torch.empty(32 * cout * cin, device=dev)
    ext().wino_weights(w, u)
    geom = [cin, 8, 8, cout, 3, 3, 1, 1]
    set_winograd(True)
    tw = timeit(lambda: ext().conv_fwd(x, w, y, geom, None, False, None, u))
    set_winograd(False)
    try:
        td = timeit(lambda: ext().conv_fwd(x, w, y, geom, None, False, None, None))
    except Exception as e:  # noqa: BLE001
        td = float("nan")
    set_winograd(True)
    print(f"Cin {cin:4d} Cout {cout:4d}: winograd {tw:7.2f} us   direct {td:7.2f} us", flush=True)
