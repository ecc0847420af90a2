"""Reference module name kept: ``import tensor_buffer as tb``."""
from network_distributed_pytorch_amd.parallel.comm import all_gather, all_reduce  # noqa: F401
from network_distributed_pytorch_amd.parallel.tensor_buffer import TensorBuffer  # noqa: F401
