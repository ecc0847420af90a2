"""Per-step losses of the engine in graph vs eager mode (ragged last batch diagnosis)."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from network_distributed_pytorch_amd import engine  # noqa: E402

for n in (96, 100):
    for mode in ("full", "none"):
        d = tempfile.mkdtemp()
        cfg = engine.default_config(task="cifar", model="resnet18", num_classes=10, grad_sync="powersgd",
                                    training_epochs=2, dataset_size=n, global_batch=32, graph_mode=mode,
                                    verbose=False, log_file=os.path.join(d, "l.jsonl"))
        out = engine.run_task(cfg)
        recs = [json.loads(ln) for ln in open(os.path.join(d, "l.jsonl"))]
        print(n, mode, out["graph_mode"], [round(r["loss"], 5) for r in recs if r["kind"] == "step"],
              [round(r["mean_loss"], 5) for r in recs if r["kind"] == "epoch"], out["param_checksum"], flush=True)
