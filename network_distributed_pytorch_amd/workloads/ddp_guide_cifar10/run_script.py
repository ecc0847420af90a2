"""``python run_script.py -rank R -cuda C [-world_size N] [-init_method URL] [-spawn] ...``

Reference: ddp_guide_cifar10/run_script.py:25-41 (which hard-codes ``n_workers = 4``; kept as the default).
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

from network_distributed_pytorch_amd.workloads import _cli  # noqa: E402
from network_distributed_pytorch_amd.workloads.ddp_guide_cifar10 import ddp_init  # noqa: E402

if __name__ == "__main__":
    _cli.main(ddp_init, default_world=4)
