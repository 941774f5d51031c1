"""Data parallelism with global-batch negatives over RCCL/xGMI."""
from .distributed import DistNTXentFunction, cpu_dist_ntxent_loss, dist_ntxent_loss  # noqa: F401
