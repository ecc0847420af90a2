"""PowerSGD data-parallel CIFAR-10 (reference: ddp_powersgd_guide_cifar10/ddp_init.py:22-194).

Reference semantics: ResNet (reference: ``resnet152(pretrained=True)``, 1000-class head),
per-rank batch ``512 / world``, PowerSGD rank 4 with error feedback and the
"Algorithm 2" momentum update (lr 1e-3, lambda 0.9).  ``grad_sync="powersgd"`` (default)
runs the fused gfx950 engine; ``"powersgd-ref"`` the reference's eager per-tensor loops;
``"powersgd-api"`` the reference loop around the API-compatible native
``PowerSGDReducer.reduce``.  Data synthetic CIFAR-10-shape; weights random-init.
"""
from network_distributed_pytorch_amd import engine
from network_distributed_pytorch_amd.parallel.ddp import average_gradients  # noqa: F401
from network_distributed_pytorch_amd.parallel.powersgd import PowerSGDReducer  # noqa: F401
from network_distributed_pytorch_amd.utils.data import DeviceLoader, SyntheticCIFAR10
from network_distributed_pytorch_amd.utils.partition_helper import DataPartitioner

config = dict(
    seed=714,
    rank=0,  # should be updated by caller
    cuda_rank=0,
    n_workers=4,
    distributed_init_file=None,
    output_dir="./output.tmp",
    distributed_backend="nccl",
    init_method=None,
    timeout_s=600,
    learning_rate=0.001,
    momentum=0.9,
    nesterov=False,
    training_epochs=100,
    batch_size=32,  # unused, as in the reference (batch = 512 / world)
    reducer_rank=4,
    # additions
    task="cifar",
    model="resnet152",
    num_classes=1000,
    global_batch=512,
    grad_sync="powersgd",
    graph_mode="auto",  # hipGraph on GPU (full / piecewise by data plane), eager on CPU
)


def _cfg():
    return engine.default_config(**config)


def partition_dataset():
    import torch.distributed as dist

    size = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    dev = engine.device_for(config)
    ds = SyntheticCIFAR10(n=config.get("dataset_size") or 50000, device=dev)
    bsz = int(config["global_batch"] / float(size))
    part = DataPartitioner(ds, [1.0 / size for _ in range(size)]).use(rank)
    return DeviceLoader(part, bsz, shuffle=True, seed=config["seed"] + rank), bsz


def setup():
    engine.setup(_cfg())


def run_task():
    return engine.run_task(_cfg())


def cleanup():
    engine.cleanup(_cfg())


if __name__ == "__main__":
    setup()
    run_task()
    cleanup()
