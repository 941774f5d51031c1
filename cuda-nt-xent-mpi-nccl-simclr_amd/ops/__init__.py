"""NT-Xent ops: HIP autograd op, raw reference-compatible API, pure-PyTorch oracle."""
from . import reference  # noqa: F401
from .ntxent import (  # noqa: F401
    NTXentFunction,
    NTXentLoss,
    backward,
    check_matrix_core_support,
    check_tensor_core_support,
    forward,
    forward_with_stats,
    ntxent_loss,
    resolve_compute,
)
