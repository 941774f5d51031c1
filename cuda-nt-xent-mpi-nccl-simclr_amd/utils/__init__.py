"""Utilities: device checks, GPU memory tracking, timing."""
from .device import arch_name, device_summary, is_gfx950, require_gfx950  # noqa: F401
