"""Diagnostic: does engine resume reproduce the uninterrupted run?  Spawns 2 ranks on one GPU
(IPC data plane) and prints per-rank checksums after epoch 1 straight / epoch 1 of a fresh run,
and after 2 epochs straight / resumed, for the given grad_sync and graph mode.
    python tools/diag/resume_check.py powersgd full"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CODE = r'''
import os, sys, json
sys.path.insert(0, ROOT)
import torch
from network_distributed_pytorch_amd import engine
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
ck = os.environ["CKDIR"]
base = dict(task="cifar", model="resnet18", num_classes=10, grad_sync=os.environ["SYNC"], dataset_size=200,
            global_batch=64, graph_mode=os.environ["GMODE"], verbose=False, rank=rank, n_workers=world, cuda_rank=0,
            distributed_backend="gloo", init_method="tcp://127.0.0.1:" + os.environ["MASTER_PORT"],
            check_health_every=1, log_file=None,
            overlap=None if os.environ.get("OVERLAP", "") == "" else os.environ["OVERLAP"] == "1")
engine.setup(engine.default_config(**base))
res = {"rank": rank}
def run(tag, **kw):
    torch.manual_seed(714 + rank)
    r = engine.run_task(engine.default_config(**dict(base, **kw)))
    res[tag] = r["param_checksum"]
run("e1_straight", training_epochs=1)
run("e1_ck", training_epochs=1, checkpoint_dir=ck)
if os.environ.get("QUICK") != "1":
    run("e2_resumed", training_epochs=2, resume=os.path.join(ck, "last.pt"))
    run("e2_straight", training_epochs=2)
print("RESULT " + json.dumps(res), flush=True)
'''


def main():
    sync, gmode = sys.argv[1], sys.argv[2]
    sys.path.insert(0, ROOT)
    from network_distributed_pytorch_amd.utils.launcher import find_free_port

    port = find_free_port()
    ck = tempfile.mkdtemp()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), NDP_COMM="ipc", CKDIR=ck, SYNC=sync, GMODE=gmode)
        procs.append(subprocess.Popen([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CODE], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    for p in procs:
        out = p.communicate(timeout=600)[0]
        lines = [ln for ln in out.splitlines() if ln.startswith("RESULT ")]
        print(lines[0] if lines else out[-3000:], flush=True)


if __name__ == "__main__":
    main()
