"""Utilities: device checks, GPU memory tracking, timing, tracing, checkpoints."""
from .checkpoint import latest_checkpoint, load_checkpoint, save_checkpoint  # noqa: F401
from .device import arch_name, device_summary, is_gfx950, require_gfx950  # noqa: F401
from .memory import GPUMemoryTracker, measure_peak  # noqa: F401
from .timing import summarize, time_fn  # noqa: F401
from .trace import trace_range  # noqa: F401
