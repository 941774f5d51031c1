"""Batched SimCLR augmentations on the GPU (no per-image host work, no torchvision).

The SimCLR view pipeline — random resized crop, horizontal flip, colour jitter, random
grayscale (Chen et al., 2020, Appendix A) — applied to a whole NCHW batch with a handful of
kernels: one affine ``grid_sample`` covers crop + resize + flip, colour ops are broadcasted
per-sample scalars. Two independent calls give the two views.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


@dataclass
class AugmentConfig:
    out_size: int = 32
    scale: Tuple[float, float] = (0.2, 1.0)       # crop area fraction
    ratio: Tuple[float, float] = (3 / 4, 4 / 3)   # crop aspect ratio
    flip_p: float = 0.5
    jitter_p: float = 0.8
    brightness: float = 0.4
    contrast: float = 0.4
    saturation: float = 0.4
    gray_p: float = 0.2


def _uniform(n, lo, hi, g, device):
    return torch.rand(n, generator=g, device=device) * (hi - lo) + lo


def random_resized_crop_flip(x: torch.Tensor, cfg: AugmentConfig, g: Optional[torch.Generator] = None) -> torch.Tensor:
    n, _, _, _ = x.shape
    dev = x.device
    area = _uniform(n, cfg.scale[0], cfg.scale[1], g, dev)
    logr = _uniform(n, math.log(cfg.ratio[0]), math.log(cfg.ratio[1]), g, dev)
    r = torch.exp(logr)
    sw = torch.sqrt(area * r).clamp(max=1.0)   # crop width / image width
    sh = torch.sqrt(area / r).clamp(max=1.0)
    cx = (torch.rand(n, generator=g, device=dev) * 2 - 1) * (1 - sw)
    cy = (torch.rand(n, generator=g, device=dev) * 2 - 1) * (1 - sh)
    flip = torch.where(torch.rand(n, generator=g, device=dev) < cfg.flip_p, -1.0, 1.0)
    theta = torch.zeros(n, 2, 3, device=dev, dtype=x.dtype)
    theta[:, 0, 0] = sw * flip
    theta[:, 0, 2] = cx
    theta[:, 1, 1] = sh
    theta[:, 1, 2] = cy
    grid = F.affine_grid(theta, (n, x.shape[1], cfg.out_size, cfg.out_size), align_corners=False)
    return F.grid_sample(x, grid, mode="bilinear", padding_mode="reflection", align_corners=False)


def color_jitter_gray(x: torch.Tensor, cfg: AugmentConfig, g: Optional[torch.Generator] = None) -> torch.Tensor:
    n = x.shape[0]
    dev = x.device
    apply = (torch.rand(n, generator=g, device=dev) < cfg.jitter_p).to(x.dtype).view(n, 1, 1, 1)
    b = _uniform(n, 1 - cfg.brightness, 1 + cfg.brightness, g, dev).to(x.dtype).view(n, 1, 1, 1)
    c = _uniform(n, 1 - cfg.contrast, 1 + cfg.contrast, g, dev).to(x.dtype).view(n, 1, 1, 1)
    s = _uniform(n, 1 - cfg.saturation, 1 + cfg.saturation, g, dev).to(x.dtype).view(n, 1, 1, 1)
    y = x * b
    mean = y.mean(dim=(1, 2, 3), keepdim=True)
    y = (y - mean) * c + mean
    gray = (0.299 * y[:, 0:1] + 0.587 * y[:, 1:2] + 0.114 * y[:, 2:3]) if x.shape[1] == 3 else y.mean(1, keepdim=True)
    y = (y - gray) * s + gray
    y = apply * y + (1 - apply) * x
    to_gray = (torch.rand(n, generator=g, device=dev) < cfg.gray_p).to(x.dtype).view(n, 1, 1, 1)
    gy = (0.299 * y[:, 0:1] + 0.587 * y[:, 1:2] + 0.114 * y[:, 2:3]).expand_as(y) if x.shape[1] == 3 else y
    return (to_gray * gy + (1 - to_gray) * y).clamp(0.0, 1.0)


def simclr_view(x: torch.Tensor, cfg: Optional[AugmentConfig] = None, g: Optional[torch.Generator] = None) -> torch.Tensor:
    cfg = cfg or AugmentConfig(out_size=x.shape[-1])
    return color_jitter_gray(random_resized_crop_flip(x, cfg, g), cfg, g)


def two_views(x: torch.Tensor, cfg: Optional[AugmentConfig] = None, g: Optional[torch.Generator] = None):
    return simclr_view(x, cfg, g), simclr_view(x, cfg, g)
