"""``python run_script.py -rank R -cuda C [-world_size N] [-spawn] [-toy_steps K]``.

Reference: ddp_guide/run_script.py:25-39 (init-only; its ``cuda_rnak`` typo and
rank-as-GPU-index are fixed).  ``-toy_steps K`` additionally trains a toy MLP with dense
data parallelism for K steps (BASELINE.json config 1: CPU/gloo, world size 2).
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

from network_distributed_pytorch_amd.workloads import _cli  # noqa: E402
from network_distributed_pytorch_amd.workloads.ddp_guide import ddp_init  # noqa: E402

if __name__ == "__main__":
    _cli.main(ddp_init, default_world=4)
