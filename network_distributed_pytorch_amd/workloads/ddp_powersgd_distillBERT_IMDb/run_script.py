"""``python run_script.py -rank R -cuda C -world_size N [-init_method URL] [-spawn] ...``

Reference: ddp_powersgd_distillBERT_IMDb/run_script.py:25-45 (``-world_size`` and
``-init_method`` flags; the reference's lab-host default tcp://165.132.142.56:7392 is
replaced by env:// under torchrun or a file:// rendezvous).
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

from network_distributed_pytorch_amd.workloads import _cli  # noqa: E402
from network_distributed_pytorch_amd.workloads.ddp_powersgd_distillBERT_IMDb import ddp_init  # noqa: E402

if __name__ == "__main__":
    _cli.main(ddp_init, default_world=4)
