"""Import name of the framework package that lives in ``cuda-nt-xent-mpi-nccl-simclr_amd/``.

The package directory carries the project name, which is not a valid Python identifier. This
module loads that directory as the package ``ntxent_amd`` through importlib (spec with the real
directory as its submodule search location) and puts the real package in ``sys.modules``, so
``import ntxent_amd.ops`` etc. resolve to the modules there.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_REAL = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                      "cuda-nt-xent-mpi-nccl-simclr_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_REAL, "__init__.py"),
                                     submodule_search_locations=[_REAL])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
