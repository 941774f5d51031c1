"""Device checks (reference ``verify_gpu_requirements`` at python/test.py:42-55 required
CUDA cc >= 7.0 and was never called; here the requirement is gfx950 / MI355X)."""
from __future__ import annotations

import torch


def arch_name(device: int = 0) -> str:
    if not torch.cuda.is_available():
        return ""
    return getattr(torch.cuda.get_device_properties(device), "gcnArchName", "")


def is_gfx950(device: int = 0) -> bool:
    return arch_name(device).startswith("gfx950")


def require_gfx950(device: int = 0) -> None:
    """Raise unless a ROCm build of torch sees an MI355X-class (gfx950) device."""
    if torch.version.hip is None:
        raise RuntimeError("ntxent-mi355x needs a ROCm build of PyTorch")
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device visible")
    if not is_gfx950(device):
        raise RuntimeError(f"device {device} is {arch_name(device)!r}, expected gfx950 (MI355X)")


def device_summary(device: int = 0) -> dict:
    info = {"torch": torch.__version__, "hip": torch.version.hip, "available": torch.cuda.is_available()}
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(device)
        info.update(name=p.name, arch=arch_name(device), cus=p.multi_processor_count,
                    total_mem_gb=round(p.total_memory / 2**30, 1))
    return info
