"""Stand-in GPU worker for the supervisor tests (tests/test_supervisor_cpu.py).

SUP_TEST_MODE = comma-separated ``level:rank:action`` (rank ``*`` = every rank):
  fail   exit 3 after reporting an error
  hang   declare a 1 s allowance, then sleep (a stalled rank)
  crash  exit -9-like without any report
  late   complete, then exit 5 in "teardown" (done marker already written)
SUP_TEST_DIST=1: gloo process group + one all_reduce (proves the per-attempt rendezvous).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd.utils.supervisor import Heartbeat, worker_env_info  # noqa: E402

role, level, _ = worker_env_info()
assert role == "worker"
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
hb = Heartbeat(rank)
hb.beat("start", 60)
action = None
for spec in filter(None, os.environ.get("SUP_TEST_MODE", "").split(",")):
    lvl, r, act = spec.split(":")
    if int(lvl) == level and r in ("*", str(rank)):
        action = act
if action == "fail":
    hb.error(f"boom at level {level}")
    sys.exit(3)
if action == "crash":
    os._exit(9)
if action == "hang":
    hb.beat("hang", 1)
    time.sleep(120)
if os.environ.get("SUP_TEST_DIST") == "1" and world > 1:
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    t = torch.ones(1)
    dist.all_reduce(t)
    assert t.item() == world
    dist.destroy_process_group()
if rank == 0:
    hb.result(json.dumps({"value": 1.0, "level": level, "world": world, "port": os.environ["MASTER_PORT"]}))
hb.done()
if action == "late":
    sys.exit(5)
