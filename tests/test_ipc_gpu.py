"""The opt-in HIP-IPC data plane (csrc/ipc.hip, NDP_COMM=ipc) with 2 and 4 processes sharing
ONE MI355X: raw all-reduce exactness and cross-rank bitwise equality,
graph-captured replays, and the full captured, backward-overlapped PowerSGD step (compute
graph + comm graph ordered by device flags) — bitwise equal to the serial step, replicas
equal, no flag-wait timeouts.  RCCL refuses two ranks on one GPU; this is the only
pre-multi-GPU execution of the multi-rank stream-ordered protocol."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

WORKER = r'''
import os, sys, json
sys.path.insert(0, ROOT)
import torch, torch.distributed as dist
os.environ["NDP_COMM"] = "ipc"
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
from network_distributed_pytorch_amd.parallel.comm import Communicator
comm = Communicator(device=torch.device("cuda", 0))
assert comm.backend == "ipc-native", comm.backend
out = {}
# 1. exactness + bitwise equality over sizes (tiny, one chunk, several, > 8 MB capacity)
sums = []
for n in (1, 4096, 70001, 3_000_000):
    g = torch.Generator(device="cuda").manual_seed(1000 * rank + n)
    t = torch.randn(n, device="cuda", generator=g)
    ref = torch.zeros(n, dtype=torch.float64, device="cuda")
    for r in range(world):
        gr = torch.Generator(device="cuda").manual_seed(1000 * r + n)
        ref += torch.randn(n, device="cuda", generator=gr).double()
    comm.all_reduce(t)
    torch.cuda.synchronize()
    out[f"err_{n}"] = float((t.double() - ref).abs().max() / ref.abs().max())
    sums.append(float(t.double().sum()))
out["sums"] = sums
# 2. captured all-reduce, replayed with fresh inputs
x = torch.zeros(50000, device="cuda")
gph = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    comm.all_reduce(x)  # warm-up outside capture
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
with torch.cuda.graph(gph):
    comm.all_reduce(x)
ok = True
for k in range(5):
    x.fill_(float(rank + k))
    gph.replay()
    torch.cuda.synchronize()
    want = sum(r + k for r in range(world))
    ok &= bool((x == want).all())
out["graph_ok"] = ok
# 3. all_reduce_many: a list of tensors is ONE launch (segment table), exact in each tensor
dp = comm._native
sizes = (3, 4095, 4097, 123457, 7)
ts = [torch.full((n,), float(rank + 1 + i), device="cuda") for i, n in enumerate(sizes)]
before = dp.launches
dp.all_reduce_many(ts)
torch.cuda.synchronize()
out["many_launches"] = dp.launches - before
out["many_ok"] = all(bool((t == sum(r + 1 + i for r in range(world))).all()) for i, t in enumerate(ts))
out["uncached"] = dp.uncached
comm.check()
out["rank"] = rank
print("RESULT " + json.dumps(out), flush=True)
dist.barrier()
dist.destroy_process_group()
'''


def _spawn(world, code, extra_env=None, timeout=240):
    from network_distributed_pytorch_amd.utils.launcher import find_free_port

    port = find_free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + code], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-4000:]
    return [json.loads([ln for ln in o.splitlines() if ln.startswith("RESULT ")][0][7:]) for o in outs]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_ipc_allreduce_multi_process_one_gpu(device, world):
    res = _spawn(world, WORKER)
    for r in res:
        for k, v in r.items():
            if k.startswith("err_"):
                assert v < 1e-5, (k, v)
        assert r["graph_ok"], r
        assert r["many_launches"] == 1 and r["many_ok"], r
    assert all(r["sums"] == res[0]["sums"] for r in res), "ranks disagree bitwise"


def _bench(args, env_extra):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=400, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, (p.stdout + p.stderr)[-4000:]
    return json.loads(lines[-1])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_captured_overlapped_powersgd_multi_process(device, world):
    """The N > 1 default step shape — compute graph + comm graph (PowerSGD group pipelines and
    their collectives on the side stream, overlapping backward), ordered by device flags —
    with `world` real processes: no fallback, no flag error, replicas equal, and bitwise the
    same parameters as the serial (non-overlapped) step."""
    env = {"NDP_BACKEND": "gloo", "NDP_COMM": "ipc"}
    common = ["--gpus", str(world), "--steps", "4", "--warmup", "3", "--global-batch", str(32 * world)]
    ov = _bench(common + ["--overlap", "on"], env)
    assert ov["comm_backend"] == "ipc-native" and ov["n_gpus"] == world
    assert ov["config"]["hip_graph"] == "full" and ov["config"]["overlap"] is True
    assert ov["fallback"] is None and ov["supervisor"]["failed"] == [], ov["supervisor"]
    assert ov["replicas_equal"] and ov["flag_errors"] == 0
    assert ov["collectives_per_step"] >= 5 and ov["collectives_per_step"] % 2 == 1  # 2 per group + rank-1
    serial = _bench(common + ["--overlap", "off"], env)
    assert serial["config"]["overlap"] is False and serial["fallback"] is None
    assert ov["param_checksum"] == serial["param_checksum"], (ov["param_checksum"], serial["param_checksum"])


STALL = r'''
import os, sys, json, time
sys.path.insert(0, ROOT)
import torch, torch.distributed as dist
os.environ["NDP_COMM"] = "ipc"
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
from network_distributed_pytorch_amd.parallel.comm import Communicator
comm = Communicator(device=torch.device("cuda", 0))
t = torch.ones(10000, device="cuda")
comm.all_reduce(t)  # one healthy collective first
torch.cuda.synchronize()
comm.check()
dist.barrier()
if rank == world - 1:
    time.sleep(2.0)  # stall past the 0.3 s flag-wait bound of the others
comm.all_reduce(t)
torch.cuda.synchronize()
err = None
try:
    comm.check()
except RuntimeError as e:
    err = str(e)
print("RESULT " + json.dumps({"rank": rank, "err": err}), flush=True)
dist.barrier()
dist.destroy_process_group()
'''


@pytest.mark.timeout(300)
def test_ipc_timeout_fails_every_rank(device):
    """a stalled rank makes the others' waits time out; they return without
    touching data or flags and poison every peer, so the check raises on EVERY rank (the
    stalled one included, whose later collective would otherwise read half-published
    chunks) instead of producing a silently wrong sum."""
    res = _spawn(2, STALL, extra_env={"NDP_FLAG_WAIT_US": "300000"})
    for r in res:
        assert r["err"] is not None and "timed out" in r["err"], r
