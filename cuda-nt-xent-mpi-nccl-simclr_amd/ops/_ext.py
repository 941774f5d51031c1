"""Loader for the in-tree HIP extension (``_C``).

The extension is built in-tree by ``tools/build_ext.py`` (hipcc, gfx950). On a GPU box a
missing or stale extension is an error, never a silent fallback: set
``NTXENT_ALLOW_REFERENCE=1`` to opt into the pure-PyTorch oracle explicitly.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _pkg_name() -> str:
    return __name__.rsplit(".", 2)[0]


def load(build_if_missing: bool = True):
    """Import (building first if needed) and return the ``_C`` extension module."""
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            _mod = importlib.import_module(_pkg_name() + "._C")
            return _mod
        except ImportError as e:  # not built yet
            _err = e
        if build_if_missing and os.environ.get("NTXENT_NO_BUILD", "0") != "1":
            import sys
            from pathlib import Path

            root = Path(__file__).resolve().parents[2]
            sys.path.insert(0, str(root / "tools"))
            try:
                import build_ext  # type: ignore

                build_ext.build(cpp_targets=False)
            finally:
                sys.path.pop(0)
            importlib.invalidate_caches()
            _mod = importlib.import_module(_pkg_name() + "._C")
            return _mod
        raise ImportError(f"ntxent HIP extension not available: {_err}")


def available() -> bool:
    try:
        load(build_if_missing=False)
        return True
    except Exception:
        return False


def ext_path() -> str:
    return load().__file__
