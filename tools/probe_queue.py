"""GPU probe (run under rocprofv3 --kernel-trace): when does the side queue dispatch the
comm graph relative to the compute graph's train of short kernels?

compute graph: wait(DONE) + N delay kernels of D us, a flag signal after kernel S
comm graph:    marker delay (1 us) + wait(signal 0) + delay 2 us + signal(DONE)
order: "cc" = compute then comm replay on the host (StepRunner), "sc" = comm first.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.ops import delay_ns, ext  # noqa: E402
from network_distributed_pytorch_amd.parallel.comm import Communicator  # noqa: E402


def main():
    n, d, sig = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    order = sys.argv[4] if len(sys.argv) > 4 else "cc"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Communicator(device=dev)
    comm._flag_buf()
    X = ext()

    gM, gS = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(gM):
        comm.graph_prologue()
        for k in range(n):
            delay_ns(d * 1000)
            if k == sig:
                X.flag_signal(comm._flag_buf(), 0)
    with torch.cuda.graph(gS, stream=torch.cuda.Stream()):
        delay_ns(1000)
        comm.graph_wait(0)
        delay_ns(2000)
        comm.graph_epilogue()
    comm.reset_flags()

    def step():
        if order == "cc":
            gM.replay()
            with comm.on_side():
                gS.replay()
        else:
            with comm.on_side():
                gS.replay()
            gM.replay()

    for _ in range(30):
        step()
    torch.cuda.synchronize()
    print("flag error", comm.flag_error(), flush=True)


if __name__ == "__main__":
    main()
