"""Every other N > 1 path rehearsed with 2 / 4 real processes sharing ONE MI355X on the IPC data
plane (csrc/ipc.hip, NDP_COMM=ipc; RCCL refuses two ranks on one GPU) — VERDICT r3 item 5:

* the dense arm's backward-overlapped buckets in captured compute + comm graphs
  (reference dense arm: ddp_guide_cifar10/ddp_init.py:57-62,124), bitwise the serial step;
* DistilBERT PowerSGD r=8 — the largest P / Q payloads
  (ddp_powersgd_distillBERT_IMDb/ddp_init.py:140-231), overlapped vs serial;
* the engine's graph-mode ``run_task`` with a ragged last batch, a health check after every
  step and per-rank checkpoints, then a resume (ddp_powersgd_guide_cifar10/ddp_init.py:118,
  142,183): every rank ends with the same parameters, which equal an uninterrupted run's.
Each passes only with replicas equal and no flag-wait timeout."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

IPC = {"NDP_BACKEND": "gloo", "NDP_COMM": "ipc"}


def _bench(args, env_extra, timeout=500):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, (p.stdout + p.stderr)[-4000:]
    return json.loads(lines[-1])


def _healthy(rec, world):
    assert rec["comm_backend"] == "ipc-native" and rec["n_gpus"] == world, rec["comm_backend"]
    assert rec["fallback"] is None and rec["supervisor"]["failed"] == [], rec.get("supervisor")
    assert rec["replicas_equal"] and rec["flag_errors"] == 0


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 4])
def test_dense_overlapped_buckets_multi_process(device, world):
    common = ["--gpus", str(world), "--steps", "4", "--warmup", "3", "--global-batch", str(32 * world),
              "--reducer", "dense", "--bucket-mb", "4"]
    ov = _bench(common + ["--overlap", "on"], IPC)
    _healthy(ov, world)
    assert ov["config"]["hip_graph"] == "full" and ov["config"]["overlap"] is True
    assert ov["collectives_per_step"] > 1  # one per bucket
    serial = _bench(common + ["--overlap", "off"], IPC)
    _healthy(serial, world)
    assert serial["config"]["overlap"] is False
    assert ov["param_checksum"] == serial["param_checksum"], (ov["param_checksum"], serial["param_checksum"])


@pytest.mark.timeout(900)
def test_distilbert_powersgd_r8_multi_process(device):
    world = 2
    common = ["--gpus", str(world), "--steps", "3", "--warmup", "2", "--model", "distilbert", "--rank", "8",
              "--batch", "2", "--seq-len", "128"]
    ov = _bench(common + ["--overlap", "on"], IPC)
    _healthy(ov, world)
    assert ov["bytes_per_step"] == 4000600  # the reference's r=8 accounting
    serial = _bench(common + ["--overlap", "off"], IPC)
    _healthy(serial, world)
    assert ov["param_checksum"] == serial["param_checksum"], (ov["param_checksum"], serial["param_checksum"])


ENGINE = r'''
import os, sys, json
sys.path.insert(0, ROOT)
import torch
from network_distributed_pytorch_amd import engine
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
ck = os.environ["CKDIR"]
base = dict(task="cifar", model="resnet18", num_classes=10, grad_sync=os.environ["SYNC"], dataset_size=200,
            global_batch=64, graph_mode="full", verbose=False, rank=rank, n_workers=world, cuda_rank=0,
            distributed_backend="gloo", init_method="tcp://127.0.0.1:" + os.environ["MASTER_PORT"],
            check_health_every=1, log_file=None)
cfg = engine.default_config(**dict(base, training_epochs=1, checkpoint_dir=ck))
engine.setup(cfg)
a = engine.run_task(cfg)
res = {"rank": rank, "ck1": a["param_checksum"], "steps1": a["steps"], "graph": a["graph_mode"],
       "backend": a["comm_backend"], "files": sorted(os.listdir(ck))}
b = engine.run_task(engine.default_config(**dict(base, training_epochs=2, resume=os.path.join(ck, "last.pt"))))
res.update(ck2=b["param_checksum"], steps2=b["steps"])
torch.manual_seed(714 + rank)
c = engine.run_task(engine.default_config(**dict(base, training_epochs=2)))
res.update(ck_straight=c["param_checksum"], steps_straight=c["steps"])
print("RESULT " + json.dumps(res), flush=True)
engine.cleanup(dict(cfg, verbose=False))
'''


def _spawn(world, code, env_extra, timeout=700):
    from network_distributed_pytorch_amd.utils.launcher import find_free_port

    port = find_free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0", "NDP_COMM": "ipc"})
        env.update(env_extra)
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


@pytest.mark.timeout(900)
@pytest.mark.parametrize("sync", ["powersgd", "dense"])
def test_engine_graph_mode_ragged_health_checkpoint_resume_multi_process(device, tmp_path, sync):
    res = _spawn(2, ENGINE, {"CKDIR": str(tmp_path / "ck"), "SYNC": sync})
    for r in res:
        assert r["backend"] == "ipc-native" and r["graph"] == "full", r
        assert r["steps1"] == 4 and r["steps2"] == 8  # 100 samples / rank at 32 per step: 32 32 32 4 (ragged)
        assert f"last.pt.rank{r['rank']}" in r["files"], r["files"]
    # replicas agree after the first epoch, after the resume, and the resumed run is the
    # uninterrupted two-epoch run
    assert res[0]["ck1"] == res[1]["ck1"]
    assert res[0]["ck2"] == res[1]["ck2"]
    assert res[0]["ck2"] == res[0]["ck_straight"], (res[0]["ck2"], res[0]["ck_straight"])
