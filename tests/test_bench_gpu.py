"""bench.py end to end on one MI355X: supervisor + health checks + fallback,
and the engine's ragged last batch under graph capture."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _bench(args, env_extra=None, timeout=280):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, (json.loads(lines[-1]) if lines else None)


@pytest.mark.timeout(300)
def test_bench_two_gloo_ranks_on_one_gpu(device):
    """`bench.py --gpus 2` self-launches two ranks (gloo lets them share the GPU); the line
    says n_gpus 2 and the cross-rank parameter checksum agrees."""
    p, rec = _bench(["--gpus", "2", "--steps", "3", "--warmup", "2", "--global-batch", "64"],
                    {"NDP_BACKEND": "gloo"})
    assert p.returncode == 0 and rec is not None, (p.stdout + p.stderr)[-4000:]
    assert rec["n_gpus"] == 2 and rec["replicas_equal"] is True and rec["flag_errors"] == 0
    assert rec["config"]["per_gpu_batch"] == 32 and rec["comm_backend"] == "c10d-gloo"
    assert rec["supervisor"]["failed"] == []


@pytest.mark.timeout(300)
def test_bench_injected_flag_timeout_falls_back(device):
    """A flag wait that times out (NDP_FLAG_WAIT_US=0) must never yield a number for that
    configuration: the health check fails the attempt and the supervisor falls back."""
    p, rec = _bench(["--steps", "3", "--warmup", "2", "--global-batch", "64", "--overlap", "on"],
                    {"NDP_FLAG_WAIT_US": "0"})
    assert p.returncode == 0 and rec is not None, (p.stdout + p.stderr)[-4000:]
    failed = rec["supervisor"]["failed"]
    assert failed and failed[0]["level"] == 0 and "flag" in json.dumps(failed[0]["errors"]).lower(), failed
    assert rec["fallback"]["level"] >= 1 and rec["flag_errors"] == 0 and rec["replicas_equal"]


@pytest.mark.timeout(200)
def test_engine_graph_mode_trains_ragged_last_batch(device, tmp_path):
    from network_distributed_pytorch_amd import engine

    def run(mode):
        torch.manual_seed(0)  # the engine builds the model from the current RNG (setup() seeds it)
        cfg = engine.default_config(task="cifar", model="resnet18", num_classes=10, grad_sync="powersgd",
                                    training_epochs=1, dataset_size=100, global_batch=32, graph_mode=mode,
                                    verbose=False, log_file=str(tmp_path / f"{mode}.jsonl"))
        out = engine.run_task(cfg)
        recs = [json.loads(ln) for ln in (tmp_path / f"{mode}.jsonl").read_text().splitlines()]
        return out, [r for r in recs if r["kind"] == "epoch"][0]

    out_g, ep_g = run("full")
    out_e, ep_e = run("none")
    assert out_g["graph_mode"] == "full"
    assert ep_g["steps"] == ep_e["steps"] == ep_g["num_batches"] == 4
    assert abs(ep_g["mean_loss"] - ep_e["mean_loss"]) <= 1e-4 * abs(ep_e["mean_loss"])
    assert abs(out_g["param_checksum"] - out_e["param_checksum"]) <= 1e-6 * abs(out_e["param_checksum"]) + 1e-3
