"""Data parallelism with global-batch negatives over RCCL/xGMI: all-gather (default) or a
point-to-point ring of negatives with O(local) memory."""
from .distributed import DistNTXentFunction, cpu_dist_ntxent_loss, dist_ntxent_loss  # noqa: F401
from .ring import RingNTXentFunction, ring_ntxent_loss  # noqa: F401
