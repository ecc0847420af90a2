"""Diagnostic: two identical engine runs in ONE process (world 1) — equal parameters?
    python tools/diag/repeat_check.py [grad_sync] [graph_mode]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from network_distributed_pytorch_amd import engine  # noqa: E402

sync = sys.argv[1] if len(sys.argv) > 1 else "powersgd"
gm = sys.argv[2] if len(sys.argv) > 2 else "none"
base = dict(task="cifar", model="resnet18", num_classes=10, grad_sync=sync, dataset_size=int(os.environ.get("NDS", "96")), global_batch=int(os.environ.get("GB", "32")),
            graph_mode=gm, verbose=False, rank=0, n_workers=1, cuda_rank=0, log_file=None, training_epochs=1)
engine.setup(engine.default_config(**base))
out = []
for i in range(3):
    torch.manual_seed(714)
    r = engine.run_task(engine.default_config(**base))
    out.append(r["param_checksum"])
print(sync, gm, os.environ.get("NDS", "96"), os.environ.get("GB", "32"), out, "EQUAL" if len(set(out)) == 1 else "DIFFER", flush=True)
