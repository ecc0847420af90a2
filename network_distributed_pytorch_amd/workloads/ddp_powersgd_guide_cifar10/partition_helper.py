"""Reference module name kept: ``import partition_helper as part_help``."""
from network_distributed_pytorch_amd.utils.partition_helper import DataPartitioner, Partition  # noqa: F401
