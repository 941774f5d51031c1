"""GPU memory tracking (reference ``GPUMemoryTracker`` at python/test.py:25-40).

The reference logs ``memory_allocated``/``memory_reserved`` in MB per step and dumps
``memory_profile.json``. This version also records the peak per tracked region (reset with
``reset_peak_memory_stats``), which is what shows that no O((2N)^2) fp32 buffer is created,
and is safe to use on a CPU-only box (records zeros).
"""
from __future__ import annotations

import json
import time
from contextlib import contextmanager
from pathlib import Path
from typing import Callable, Dict, List, Optional

import torch

MB = 1024.0 * 1024.0


def _cuda() -> bool:
    return torch.cuda.is_available()


class GPUMemoryTracker:
    """Per-step memory log: ``tracker.log("step 3")``; ``tracker.region("fwd")`` for peaks."""

    def __init__(self, device: Optional[int] = None):
        self.device = device if device is not None else (torch.cuda.current_device() if _cuda() else 0)
        self.records: List[Dict] = []

    def snapshot(self) -> Dict[str, float]:
        if not _cuda():
            return {"allocated_mb": 0.0, "reserved_mb": 0.0, "peak_mb": 0.0}
        return {
            "allocated_mb": torch.cuda.memory_allocated(self.device) / MB,
            "reserved_mb": torch.cuda.memory_reserved(self.device) / MB,
            "peak_mb": torch.cuda.max_memory_allocated(self.device) / MB,
        }

    def log(self, tag: str, **extra) -> Dict:
        rec = {"tag": tag, "time": time.time(), **self.snapshot(), **extra}
        self.records.append(rec)
        return rec

    @contextmanager
    def region(self, tag: str, **extra):
        """Records the peak allocated above the region's starting point."""
        if _cuda():
            torch.cuda.synchronize(self.device)
            torch.cuda.reset_peak_memory_stats(self.device)
            base = torch.cuda.memory_allocated(self.device)
        else:
            base = 0
        yield
        if _cuda():
            torch.cuda.synchronize(self.device)
            peak = (torch.cuda.max_memory_allocated(self.device) - base) / MB
        else:
            peak = 0.0
        self.log(tag, region_peak_mb=peak, **extra)

    def dump(self, path: str | Path) -> Path:
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        path.write_text(json.dumps(self.records, indent=2))
        return path


def measure_peak(fn: Callable[[], object], device: Optional[int] = None) -> float:
    """Peak bytes allocated by ``fn()`` above the current allocation (0 on CPU)."""
    if not _cuda():
        fn()
        return 0.0
    dev = device if device is not None else torch.cuda.current_device()
    torch.cuda.synchronize(dev)
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    fn()
    torch.cuda.synchronize(dev)
    return float(torch.cuda.max_memory_allocated(dev) - base)
