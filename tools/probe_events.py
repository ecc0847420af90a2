"""GPU probe: when do comm-graph event-wait nodes resolve against compute-graph record nodes?
Compute graph: N delay kernels of D us, records after kernels in RECS.
Comm graph: wait e_i -> tiny delay kernel.  Run under rocprofv3 --kernel-trace."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.ops import delay_ns  # noqa: E402
from network_distributed_pytorch_amd.parallel.comm import Communicator  # noqa: E402


def main():
    n, d = int(sys.argv[1]), int(sys.argv[2])
    recs = [int(x) for x in sys.argv[3].split(",")]
    mode = sys.argv[4] if len(sys.argv) > 4 else "graph"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Communicator(device=dev)
    x = torch.zeros(1 << 20, device=dev)

    def body_m():
        for k in range(n):
            delay_ns(d * 1000)
            if k % 7 == 3:
                x.add_(1.0)  # a torch elementwise kernel
            if k in recs:
                comm.record_event(recs.index(k))

    def body_s():
        for i in range(len(recs)):
            comm.wait_event(i)
            delay_ns(3000 + 1000 * i)

    if mode == "graph":
        gM, gS = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(gM):
            body_m()
        with torch.cuda.graph(gS, stream=torch.cuda.Stream()):
            body_s()

        def step():
            gM.replay()
            with comm.on_side():
                gS.replay()
            comm.join()
    else:
        def step():
            body_m()
            with comm.on_side():
                body_s()
            comm.join()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    print("ms/step", (time.perf_counter() - t0) / 10 * 1e3, flush=True)


if __name__ == "__main__":
    main()
