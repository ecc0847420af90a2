"""``ddp_guide``: process-group bootstrap (reference: ddp_guide/ddp_init.py:9-47).

``main()`` seeds ``seed + rank``, initialises the process group through a shared-file
rendezvous (``file://<output_dir>/dist_init``, 120 s timeout) and prints the banners.
Addition (BASELINE.json config 1): ``config["toy_mlp_steps"] > 0`` then trains a toy MLP
with dense data parallelism for that many steps (CPU/gloo or GPU/RCCL) as a plumbing check.
Fix: the device is ``cuda:cuda_rank`` (the reference uses ``rank`` as the GPU index, Q12).
"""
from network_distributed_pytorch_amd import engine

config = dict(
    seed=714,
    rank=0,  # should be updated by caller
    cuda_rank=0,
    n_workers=4,
    distributed_init_file=None,  # (kind of socket)
    output_dir="./output.tmp",
    distributed_backend="nccl",  # gloo is more compatible (CPU tests use it)
    init_method=None,
    timeout_s=120,
    # additions
    toy_mlp_steps=0,
    task="mlp",
    grad_sync="dense",
    global_batch=64,
    learning_rate=0.05,
    momentum=0.9,
    training_epochs=1,
    verbose=True,
)


def _cfg():
    return engine.default_config(**{k: v for k, v in config.items()})


def main():
    cfg = _cfg()
    engine.setup(cfg)
    config.update({k: cfg[k] for k in ("distributed_init_file",)})
    if config.get("toy_mlp_steps", 0) > 0:
        cfg["max_steps_per_epoch"] = config["toy_mlp_steps"]
        cfg["dataset_size"] = max(cfg.get("dataset_size") or 0, config["toy_mlp_steps"] * cfg["global_batch"])
        return engine.run_task(cfg)
    return None


def setup():
    engine.setup(_cfg())


def run_task():
    """Toy-MLP dense-DP steps when ``toy_mlp_steps > 0``; the reference guide trains nothing."""
    if not config.get("toy_mlp_steps"):
        return None
    cfg = _cfg()
    cfg["max_steps_per_epoch"] = config["toy_mlp_steps"]
    cfg["dataset_size"] = max(cfg.get("dataset_size") or 0, config["toy_mlp_steps"] * cfg["global_batch"])
    return engine.run_task(cfg)


def cleanup():
    engine.cleanup(_cfg())


if __name__ == "__main__":
    main()
