"""Single-GPU DistilBERT/IMDb baseline with AdamW
(reference: ddp_powersgd_distillBERT_IMDb/IMDb_dataset_distributer.py:32-68 — lr 5e-5,
3 epochs, batch 16; the reference's name notwithstanding it distributes nothing).
``transformers.AdamW`` no longer exists (transformers >= 5); ``torch.optim.AdamW`` is used.

    python IMDb_dataset_distributer.py [-epochs E] [-steps S] [-dataset_size N]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

from network_distributed_pytorch_amd import engine  # noqa: E402

config = engine.default_config(task="imdb", model="distilbert", grad_sync="local-adamw", learning_rate=5e-5,
                               training_epochs=3, global_batch=16, n_workers=1)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-epochs", type=int, default=config["training_epochs"])
    ap.add_argument("-steps", type=int, default=None)
    ap.add_argument("-dataset_size", type=int, default=None)
    ap.add_argument("-seq_len", type=int, default=512)
    a = ap.parse_args(argv)
    cfg = dict(config, training_epochs=a.epochs, max_steps_per_epoch=a.steps, dataset_size=a.dataset_size,
               seq_len=a.seq_len)
    return engine.run_task(cfg)


if __name__ == "__main__":
    main()
