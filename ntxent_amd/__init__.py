"""Import alias for the framework package that lives in ``cuda-nt-xent-mpi-nccl-simclr_amd/``.

The on-disk package directory carries the project name (which is not a valid Python
identifier); this shim points the ``ntxent_amd`` package's search path at it, so
``import ntxent_amd.ops`` etc. resolve to the real modules there.
"""
import os as _os

_REAL = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                      "cuda-nt-xent-mpi-nccl-simclr_amd")
__path__ = [_REAL]
__file__ = _os.path.join(_REAL, "__init__.py")
with open(__file__) as _f:
    exec(compile(_f.read(), __file__, "exec"))
