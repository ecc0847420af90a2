"""Per-segment timing of the piecewise hipGraph step (diagnostic).

    NDP_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 tools/piecewise_diag.py
"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.models import build_model  # noqa: E402
from network_distributed_pytorch_amd.parallel.comm import Communicator  # noqa: E402
from network_distributed_pytorch_amd.parallel.trainer import build_grad_sync  # noqa: E402
from network_distributed_pytorch_amd.utils.graph import StepRunner  # noqa: E402


def main():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group(os.environ.get("NDP_BACKEND", "nccl"))
    torch.manual_seed(714)
    model = build_model("resnet18", None).to(dev)
    comm = Communicator()
    sync = build_grad_sync("powersgd", model, comm, lr=1e-3, momentum=0.9, rank=4)
    x = torch.rand(512, 3, 32, 32, device=dev) * 2 - 1
    y = torch.randint(0, 10, (512,), device=dev)

    def pre():
        sync.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()

    mode = os.environ.get("MODE", "piecewise")
    runner = StepRunner(pre, sync, mode=mode, warmup=3)
    runner()
    torch.cuda.synchronize()
    for it in range(4):
        times = []
        if runner.graphs is None:
            t0 = time.perf_counter()
            runner()
            torch.cuda.synchronize()
            times.append(("eager-step", time.perf_counter() - t0))
        else:
            for k, ((fn, _), g) in enumerate(zip(runner.segments, runner.graphs)):
                t0 = time.perf_counter()
                if g is None:
                    fn()
                else:
                    g.replay()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                times.append((f"seg{k}{'G' if g is not None else 'C'}", t1 - t0, t2 - t0))
        print(f"rank{rank} it{it} " + " ".join(f"{n}:{'/'.join(f'{v*1e3:.2f}' for v in vs)}ms"
                                              for n, *vs in times), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
