"""PowerSGD data-parallel DistilBERT on IMDb (reference: ddp_powersgd_distillBERT_IMDb/ddp_init.py).

Reference semantics: DistilBERT-base sequence classification (2 labels), per-rank batch
16 (global 16·N), PowerSGD rank 16, lr 5e-5, lambda 0.9, 5 epochs, the configurable
``init_method``.  IMDb-shape synthetic data (25k reviews x 512 tokens, 80/20 split on a
fixed seed — quirk Q2 fixed), random-init weights with rank-0 broadcast (Q3 fixed).
"""
from network_distributed_pytorch_amd import engine
from network_distributed_pytorch_amd.models.distilbert import DistilBertForSequenceClassification  # noqa: F401
from network_distributed_pytorch_amd.parallel.ddp import average_gradients  # noqa: F401
from network_distributed_pytorch_amd.parallel.powersgd import PowerSGDReducer  # noqa: F401
from network_distributed_pytorch_amd.utils.data import SyntheticIMDb, TensorDictDataset, train_val_split
from network_distributed_pytorch_amd.utils.partition_helper import DataPartitioner

config = dict(
    seed=714,
    rank=0,  # should be updated by caller
    cuda_rank=0,
    n_workers=4,
    distributed_init_file=None,
    output_dir="./output.tmp",
    distributed_backend="nccl",
    init_method=None,  # reference default: tcp://165.132.142.56:7392 (a lab host)
    timeout_s=600,
    learning_rate=5e-5,
    momentum=0.9,
    nesterov=False,
    training_epochs=5,
    batch_size=16,
    reducer_rank=16,
    # additions
    task="imdb",
    model="distilbert",
    global_batch=None,  # None -> 16 * world (reference)
    seq_len=512,
    grad_sync="powersgd",
    graph_mode="auto",  # hipGraph on GPU (full / piecewise by data plane), eager on CPU
)


class IMDbDataset(TensorDictDataset):
    """Reference name (ddp_init.py:43-54): dict items of input_ids / attention_mask / labels."""

    def __init__(self, encodings, labels):
        import torch

        cols = {k: torch.as_tensor(v) for k, v in encodings.items()}
        cols["labels"] = torch.as_tensor(labels)
        super().__init__(cols)


def prepare_IMDb():
    """((Partition, bsz), val, test) like the reference (ddp_init.py:68-83), synthetic."""
    import torch.distributed as dist

    size = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    dev = engine.device_for(config)
    full = SyntheticIMDb(n=config.get("dataset_size") or 25000, seq_len=config["seq_len"], device=dev)
    test = SyntheticIMDb(n=config.get("dataset_size") or 25000, seq_len=config["seq_len"], seed=1, device=dev)
    train, val = train_val_split(full, test_size=0.2, seed=42)
    return partition_dataset(train, size, rank), val, test


def partition_dataset(dataset, size=None, rank=None):
    import torch.distributed as dist

    size = size or (dist.get_world_size() if dist.is_initialized() else 1)
    rank = rank if rank is not None else (dist.get_rank() if dist.is_initialized() else 0)
    total_batch = 16 * size
    bsz = int(total_batch / float(size))
    part = DataPartitioner(dataset, [1.0 / size for _ in range(size)]).use(rank)
    return part, bsz


def _cfg():
    return engine.default_config(**config)


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
