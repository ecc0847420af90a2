"""Single-GPU DistilBERT/IMDb baseline with SGD + Nesterov momentum
(reference: ddp_powersgd_distillBERT_IMDb/IMDb_distillBERT_example.py:34-75 — lr 5e-5,
momentum 0.9, nesterov, 5 epochs, batch 16, per-epoch loss print).  Synthetic IMDb-shape
data, random-init DistilBERT, no communication.

    python IMDb_distillBERT_example.py [-epochs E] [-steps S] [-dataset_size N]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

from network_distributed_pytorch_amd import engine  # noqa: E402

config = engine.default_config(task="imdb", model="distilbert", grad_sync="local-sgd-nesterov", learning_rate=5e-5,
                               momentum=0.9, training_epochs=5, global_batch=16, n_workers=1)


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
