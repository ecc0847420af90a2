"""Reference module name kept: ``from reducer import PowerSGDReducer``."""
from network_distributed_pytorch_amd.parallel.comm import all_reduce, n_bits  # noqa: F401
from network_distributed_pytorch_amd.parallel.powersgd import PowerSGDReducer, Reducer, orthogonalize  # noqa: F401
