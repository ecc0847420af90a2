"""Probe: can RCCL run two ranks on ONE GPU?  (torchrun --nproc-per-node 2, both on cuda:0)

If it can, the captured multi-rank RCCL path (compute + comm graphs, device-flag ordering)
is testable on a one-GPU box; if ncclCommInitRank refuses ("duplicate GPU"), the opt-in
IPC data plane is the only multi-process device path there.
"""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((1024,), float(rank + 1), device="cuda")
try:
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: c10d all_reduce ok -> {t[0].item()} (expect {world * (world + 1) / 2})", flush=True)
except Exception as e:  # noqa: BLE001
    print(f"rank {rank}: c10d all_reduce FAILED: {e!r}"[:400], flush=True)
    sys.exit(3)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.parallel.comm import create_native_comm  # noqa: E402

try:
    c = create_native_comm(None, torch.device("cuda", 0))
    u = torch.full((1024,), float(rank + 1), device="cuda")
    c.all_reduce(u, "sum")
    torch.cuda.synchronize()
    print(f"rank {rank}: native all_reduce ok -> {u[0].item()} nranks={c.nranks}", flush=True)
except Exception as e:  # noqa: BLE001
    print(f"rank {rank}: native FAILED: {e!r}"[:400], flush=True)
dist.destroy_process_group()
