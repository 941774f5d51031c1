"""Data parallelism with global-batch negatives over RCCL/xGMI: all-gather (default), symmetric
(each rank pair's similarity block computed once, point-to-point exchanges), or a
point-to-point ring of negatives with O(local) memory."""
from .commstats import use_compute_stream  # noqa: F401
from .distributed import DistNTXentFunction, cpu_dist_ntxent_loss, dist_ntxent_loss  # noqa: F401
from .ring import RingNTXentFunction, ring_ntxent_loss  # noqa: F401
from .symmetric import SymNTXentFunction, cpu_sym_ntxent_loss, sym_jobs, sym_ntxent_loss  # noqa: F401
