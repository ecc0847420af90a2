"""Winograd forward cost split (graph-timed, 100 launches): layer1 / layer2 shapes at batch argv[1],
with and without the BN-statistics epilogue, and an input-channel sweep (per-chunk slope vs the
fixed per-launch intercept).  One row per arm: µs per launch."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from network_distributed_pytorch_amd.ops._ext import ext  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
dev = torch.device("cuda", 0)
X = ext()


def timeit(fn, iters=100):
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


for hw, cin, cout in [(8, 64, 64), (8, 128, 64), (8, 256, 64), (8, 512, 64), (4, 128, 128), (4, 256, 128),
                      (4, 512, 128)]:
    if not X.conv_wino([cin, hw, hw, cout, 3, 3, 1, 1], B, False):
        print(f"H {hw} Cin {cin} Cout {cout}: not on the Winograd path at batch {B}", flush=True)
        continue
    x = torch.randn(B, cin, hw, hw, device=dev)
    w = torch.randn(cout, cin, 3, 3, device=dev)
    y = torch.empty(B, cout, hw, hw, device=dev)
    u = torch.empty(32 * cout * cin, device=dev)
    X.wino_weights(w, u)
    geom = [cin, hw, hw, cout, 3, 3, 1, 1]
    part = torch.empty(32 * y.numel(), device=dev)  # split-K slabs (small batches)
    t0 = timeit(lambda: X.conv_fwd(x, w, y, geom, part, False, None, u))
    S = X.conv_stats_slices(geom, B)
    ts = float("nan")
    if S > 0:
        st = torch.empty(cout * S * 2, device=dev, dtype=torch.float64)
        ts = timeit(lambda: X.conv_fwd(x, w, y, geom, part, False, st, u))
    gf = 2 * B * cout * cin * hw * hw * 9 / 1e3
    print(f"H {hw} Cin {cin:4d} Cout {cout:4d} B {B}: {t0:7.2f} us plain, {ts:7.2f} us +stats "
          f"({gf / t0 / 1e3:6.1f} direct-equiv TF/s)", flush=True)
