"""Per-rank communication-wait accounting for the data-parallel paths.

Every place where a data-parallel forward/backward makes the compute stream depend on a
collective (``work.wait()`` on an RCCL work handle, or a synchronous collective) is wrapped
in :func:`span`. When enabled, a span records a HIP event on the current stream before and
after the dependency: the elapsed time between the two is how long the compute stream stood
still waiting for communication (zero when the transfer was already hidden under earlier
kernels). Nothing is recorded (and nothing synchronises) when accounting is disabled, which is
the default; ``bench.py`` enables it around its timed steps and reports the per-step sum.

On the gloo rehearsal backend the collectives are host-staged and synchronous, so a span
brackets the whole host-side transfer.
"""
from __future__ import annotations

import contextlib
from collections import defaultdict
from typing import Dict, List, Tuple

import torch

_enabled = False
_spans: List[Tuple[str, object, object]] = []


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = bool(on)
    _spans.clear()


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def span(name: str, device=None):
    """Bracket a dependency of the current stream on communication (no-op when disabled or
    on CPU tensors)."""
    if not _enabled or not torch.cuda.is_available():
        yield
        return
    s = torch.cuda.current_stream(device)
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(s)
    try:
        yield
    finally:
        b.record(s)
        _spans.append((name, a, b))


def collect(reset: bool = True) -> Dict[str, float]:
    """Sum of the recorded spans in ms, by name (synchronises on the recorded events)."""
    out: Dict[str, float] = defaultdict(float)
    for name, a, b in _spans:
        b.synchronize()
        out[name] += a.elapsed_time(b)
    if reset:
        _spans.clear()
    return dict(out)
