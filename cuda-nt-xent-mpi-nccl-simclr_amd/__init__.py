"""ntxent-mi355x: an MI355X-native (gfx950 / CDNA4) NT-Xent (SimCLR) contrastive-loss framework.

Layers: ``csrc/`` (HIP kernels + C++ runtime), ``ops`` (autograd op + oracle),
``parallel`` (RCCL/xGMI global-batch negatives), ``models`` (SimCLR head + synthetic
trainer), ``utils`` (device checks, memory tracking, timing).
"""
__version__ = "0.1.0"

from .ops import (  # noqa: F401,E402
    NTXentFunction,
    NTXentLoss,
    backward,
    check_matrix_core_support,
    check_tensor_core_support,
    forward,
    forward_with_stats,
    ntxent_loss,
)
