"""Tracing hooks for Python code (roctx ranges on ROCm).

The reference has only an unused ``ENABLE_PROFILING`` flag (CMakeLists.txt:10,82-84). Here:
``trace_range("name")`` emits a roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm) when
``NTXENT_ROCTX=1``, so Python-level phases (data, model, loss, optimizer, collectives) line
up with the native runtime's own ranges in a ``rocprofv3 --marker-trace`` timeline; with the
switch off it is a no-op context manager.
"""
from __future__ import annotations

import os
from contextlib import contextmanager

import torch

_ON = os.environ.get("NTXENT_ROCTX", "0") not in ("", "0", "false", "False")


def enabled() -> bool:
    return _ON and torch.cuda.is_available()


@contextmanager
def trace_range(name: str):
    if not enabled():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def mark(name: str) -> None:
    if enabled():
        torch.cuda.nvtx.mark(name)
