"""GPU probe: when do comm-graph event-wait nodes resolve against compute-graph record nodes?
Compute graph: 12 x 100 us delay kernels, record events after kernels 3, 6, 9.
Comm graph: wait e_i -> tiny delay kernel (10+i us).  Run under rocprofv3 --kernel-trace."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.ops import delay_ns  # noqa: E402
from network_distributed_pytorch_amd.parallel.comm import Communicator  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Communicator(device=dev)
    gM, gS = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gM):
        for k in range(12):
            delay_ns(100_000 + 1000 * k)
            if k in (3, 6, 9):
                comm.record_event(k // 3 - 1)
    with torch.cuda.graph(gS, stream=torch.cuda.Stream()):
        for i in range(3):
            comm.wait_event(i)
            delay_ns(10_000 + 1000 * i)
    for _ in range(5):
        gM.replay()
        with comm.on_side():
            gS.replay()
        comm.join()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        gM.replay()
        with comm.on_side():
            gS.replay()
        comm.join()
    torch.cuda.synchronize()
    print("ms/step", (time.perf_counter() - t0) / 10 * 1e3, flush=True)


if __name__ == "__main__":
    main()
