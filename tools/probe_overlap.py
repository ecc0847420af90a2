"""GPU probe: do hipGraph parallel branches run concurrently, and does the native RCCL
communicator work eagerly and under stream capture (1-rank group)?

    torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/probe_overlap.py
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.ops import ext  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    X = ext()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    # 1. graph branch concurrency: 2 x 2 ms delay kernels on forked streams
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    with torch.cuda.stream(cap):
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cap):
            side.wait_stream(torch.cuda.current_stream())
            X.delay_ns(2_000_000)
            with torch.cuda.stream(side):
                X.delay_ns(2_000_000)
            torch.cuda.current_stream().wait_stream(side)
    out["graph_two_branches_2ms_each_ms"] = timed(g.replay)

    # eager two streams
    def eager2():
        side.wait_stream(torch.cuda.current_stream())
        X.delay_ns(2_000_000)
        with torch.cuda.stream(side):
            X.delay_ns(2_000_000)
        torch.cuda.current_stream().wait_stream(side)
    out["eager_two_streams_2ms_each_ms"] = timed(eager2)

    # compute overlap: matmul chain on main, matmul chain on side
    a = torch.randn(2048, 2048, device=dev)
    b = torch.randn(2048, 2048, device=dev)

    def chain():
        for _ in range(4):
            torch.mm(a, b)
    one = timed(chain)

    def two():
        side.wait_stream(torch.cuda.current_stream())
        chain()
        with torch.cuda.stream(side):
            chain()
        torch.cuda.current_stream().wait_stream(side)
    out["mm_chain_ms"] = one
    out["mm_chain_x2_two_streams_ms"] = timed(two)

    # 2. native RCCL communicator, 1 rank
    dist.init_process_group("nccl", device_id=dev)
    store = dist.distributed_c10d._get_default_store()
    if dist.get_rank() == 0:
        store.set("ndp_probe_uid", X.rccl_unique_id())
    uid = store.get("ndp_probe_uid")
    comm = X.RcclComm(uid, dist.get_world_size(), dist.get_rank(), 0)
    t = torch.randn(1 << 20, device=dev)
    ref = t.clone()
    dist.all_reduce(ref)
    mine = t.clone()
    comm.all_reduce(mine)
    torch.cuda.synchronize()
    out["native_vs_c10d_bitwise"] = bool(torch.equal(ref, mine))
    comm.check()
    # side stream fork/join in a graph
    ext_side = torch.cuda.ExternalStream(comm.side_stream, device=dev)
    buf = torch.randn(1 << 16, device=dev)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g2, stream=cap):
            buf.mul_(2.0)
            comm.fork()
            with torch.cuda.stream(ext_side):
                comm.all_reduce(buf)
                X.delay_ns(1_000_000)
            X.delay_ns(1_000_000)
            comm.join()
            buf.add_(1.0)
    x0 = buf.clone()
    g2.replay()
    torch.cuda.synchronize()
    out["captured_native_allreduce_ok"] = bool(torch.equal(buf, x0 * 2 + 1))
    out["captured_native_fork_join_1ms_each_ms"] = timed(g2.replay)
    comm.check()
    comm.destroy()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
