"""Stream-accurate timing (HIP events) and summary statistics.

The reference times with host ``chrono``/``perf_counter`` around a device sync
(src/benchmark.cpp:25-40, python/test.py:100-110); events on the stream exclude host noise.
"""
from __future__ import annotations

import math
import time
from typing import Callable, Dict, List

import torch


def summarize(ms: List[float]) -> Dict[str, float]:
    """mean / std (population, as src/benchmark.cpp:42-53) / min / max / median in ms."""
    if not ms:
        return {"mean": math.nan, "std": math.nan, "min": math.nan, "max": math.nan, "median": math.nan}
    n = len(ms)
    mean = sum(ms) / n
    std = math.sqrt(sum((x - mean) ** 2 for x in ms) / n)
    s = sorted(ms)
    med = s[n // 2] if n % 2 else 0.5 * (s[n // 2 - 1] + s[n // 2])
    return {"mean": mean, "std": std, "min": s[0], "max": s[-1], "median": med}


def time_fn(fn: Callable[[], object], iters: int = 20, warmup: int = 3) -> List[float]:
    """Per-iteration milliseconds of ``fn`` (events on the current stream; host clock on CPU)."""
    for _ in range(warmup):
        fn()
    out = []
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        for _ in range(iters):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            out.append(a.elapsed_time(b))
    else:
        for _ in range(iters):
            t = time.perf_counter()
            fn()
            out.append((time.perf_counter() - t) * 1e3)
    return out
