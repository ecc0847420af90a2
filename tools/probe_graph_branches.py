"""GPU probe: do independent branches of ONE captured hipGraph run concurrently on MI355X?

graph A (serial): K pairs of delay kernels on one stream.
graph B (forked): the same kernels, the second of each pair on a forked side stream (event
fork / join inside the capture) so every pair is two independent graph nodes.
Prints the replay time of each; B ~= A/2 means the runtime dispatches branches to
separate queues.  Run under different DEBUG_HIP_FORCE_GRAPH_QUEUES /
DEBUG_CLR_GRAPH_PACKET_CAPTURE settings to see which knob governs it.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.ops import delay_ns  # noqa: E402


def timed(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    d_us = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    a = torch.randn(4096, 4096, device=dev)
    b = torch.randn(4096, 4096, device=dev)
    c1 = torch.empty_like(a)
    c2 = torch.empty_like(a)
    side = torch.cuda.Stream()
    torch.mm(a, b, out=c1)  # hipBLASLt handle / workspace set up outside any capture
    with torch.cuda.stream(side):
        torch.mm(b, a, out=c2)
    torch.cuda.synchronize()

    gA = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gA):
        for _ in range(k):
            delay_ns(d_us * 1000)
            delay_ns(d_us * 1000)
    gB = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gB):
        main_s = torch.cuda.current_stream()
        for _ in range(k):
            side.wait_stream(main_s)
            delay_ns(d_us * 1000)
            with torch.cuda.stream(side):
                delay_ns(d_us * 1000)
            main_s.wait_stream(side)
    # real work: two independent 4096^3 fp32 GEMMs (each fills the chip; concurrency can only
    # show up as overlap of ramp-up / tail, not 2x)
    gC = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gC):
        for _ in range(4):
            torch.mm(a, b, out=c1)
            torch.mm(b, a, out=c2)
    gD = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gD):
        main_s = torch.cuda.current_stream()
        for _ in range(4):
            side.wait_stream(main_s)
            torch.mm(a, b, out=c1)
            with torch.cuda.stream(side):
                torch.mm(b, a, out=c2)
            main_s.wait_stream(side)
    env = {key: os.environ.get(key) for key in ("DEBUG_HIP_FORCE_GRAPH_QUEUES", "DEBUG_CLR_GRAPH_PACKET_CAPTURE")}
    print(env, f"k={k} d={d_us}us serial {timed(gA):.1f} us  forked {timed(gB):.1f} us  "
          f"gemm serial {timed(gC, 5):.1f} us forked {timed(gD, 5):.1f} us", flush=True)


if __name__ == "__main__":
    main()
