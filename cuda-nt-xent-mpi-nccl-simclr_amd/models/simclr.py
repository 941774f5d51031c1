"""SimCLR model family: ResNet encoder + MLP projection head.

The reference repository is named after SimCLR but ships only the loss op.
This module provides the model the loss is meant for (Chen et al., 2020): an encoder f(.)
producing representations h and a 2-layer MLP head g(.) producing the embeddings z fed to
NT-Xent. Layout choices for MI355X: channels_last activations (MIOpen's NHWC convolution
kernels), bf16 autocast in the trainer, and no torchvision dependency (not installed here).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.short = None
        if stride != 1 or cin != cout:
            self.short = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)), inplace=True)
        out = self.bn2(self.conv2(out))
        return F.relu(out + (x if self.short is None else self.short(x)), inplace=True)


class ResNetEncoder(nn.Module):
    """ResNet-{18,34}-style encoder. ``cifar_stem`` uses a 3x3 stride-1 stem (SimCLR's
    CIFAR-10 variant); otherwise the ImageNet 7x7/2 stem + max-pool."""

    def __init__(self, layers: Sequence[int] = (2, 2, 2, 2), width: int = 64, in_ch: int = 3, cifar_stem: bool = True):
        super().__init__()
        if cifar_stem:
            self.stem = nn.Sequential(nn.Conv2d(in_ch, width, 3, 1, 1, bias=False), nn.BatchNorm2d(width), nn.ReLU(inplace=True))
        else:
            self.stem = nn.Sequential(nn.Conv2d(in_ch, width, 7, 2, 3, bias=False), nn.BatchNorm2d(width),
                                      nn.ReLU(inplace=True), nn.MaxPool2d(3, 2, 1))
        blocks: List[nn.Module] = []
        cin = width
        for i, n in enumerate(layers):
            cout = width * (2 ** i)
            for j in range(n):
                blocks.append(BasicBlock(cin, cout, stride=2 if (j == 0 and i > 0) else 1))
                cin = cout
        self.blocks = nn.Sequential(*blocks)
        self.out_dim = cin

    def forward(self, x):
        x = self.blocks(self.stem(x))
        return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


def resnet18(width: int = 64, cifar_stem: bool = True) -> ResNetEncoder:
    return ResNetEncoder((2, 2, 2, 2), width, cifar_stem=cifar_stem)


def resnet34(width: int = 64, cifar_stem: bool = True) -> ResNetEncoder:
    return ResNetEncoder((3, 4, 6, 3), width, cifar_stem=cifar_stem)


class ProjectionHead(nn.Module):
    """g(h) = W2 ReLU(BN(W1 h)) (SimCLR v1); ``layers=3`` gives the SimCLR v2 head."""

    def __init__(self, in_dim: int, hidden_dim: int = 2048, out_dim: int = 128, layers: int = 2, bn: bool = True):
        super().__init__()
        mods: List[nn.Module] = []
        d = in_dim
        for _ in range(layers - 1):
            mods += [nn.Linear(d, hidden_dim, bias=not bn)]
            if bn:
                mods += [nn.BatchNorm1d(hidden_dim)]
            mods += [nn.ReLU(inplace=True)]
            d = hidden_dim
        mods += [nn.Linear(d, out_dim)]
        self.net = nn.Sequential(*mods)

    def forward(self, h):
        return self.net(h)


class SimCLR(nn.Module):
    """z = g(f(x)). ``forward(x1, x2)`` returns the stacked embeddings [z1; z2] that the NT-Xent
    loss consumes (positive pair i <-> i + N), plus the representations h if asked."""

    def __init__(self, encoder: Optional[nn.Module] = None, proj_hidden: int = 2048, proj_out: int = 128,
                 proj_layers: int = 2):
        super().__init__()
        self.encoder = encoder if encoder is not None else resnet18()
        feat = getattr(self.encoder, "out_dim", None)
        if feat is None:
            raise ValueError("encoder must expose out_dim")
        self.head = ProjectionHead(feat, proj_hidden, proj_out, proj_layers)

    def forward(self, x1: torch.Tensor, x2: Optional[torch.Tensor] = None, return_features: bool = False):
        x = x1 if x2 is None else torch.cat([x1, x2], 0)
        h = self.encoder(x)
        z = self.head(h)
        return (z, h) if return_features else z


class MLPEncoder(nn.Module):
    """Tiny encoder for vector inputs (tests, synthetic embedding-space experiments)."""

    def __init__(self, in_dim: int, hidden: int = 256, out_dim: int = 256):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(in_dim, hidden), nn.ReLU(inplace=True), nn.Linear(hidden, out_dim))
        self.out_dim = out_dim

    def forward(self, x):
        return self.net(x.flatten(1))


def param_groups_for_lars(model: nn.Module, weight_decay: float) -> Tuple[dict, dict]:
    """Biases and normalisation parameters get no weight decay and no LARS adaptation."""
    decay, no_decay = [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (no_decay if p.ndim <= 1 else decay).append(p)
    return ({"params": decay, "weight_decay": weight_decay, "lars": True},
            {"params": no_decay, "weight_decay": 0.0, "lars": False})
