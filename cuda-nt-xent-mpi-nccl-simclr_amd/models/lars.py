"""LARS (You et al., 2017), the optimiser SimCLR trains with at large batch.

Per-parameter trust ratio eta * ||w|| / (||g|| + wd * ||w||) scales SGD-momentum updates;
param groups with ``lars=False`` (biases, BN) skip adaptation and weight decay, as in SimCLR.
The update is written with ``torch._foreach`` ops so a step is a few fused kernels rather
than one launch per tensor.
"""
from __future__ import annotations

from typing import Iterable

import torch


class LARS(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 0.3, momentum: float = 0.9, weight_decay: float = 1e-6,
                 eta: float = 1e-3, eps: float = 1e-9):
        defaults = dict(lr=lr, momentum=momentum, weight_decay=weight_decay, eta=eta, eps=eps, lars=True)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            grads = [p.grad for p in params]
            wd, lr, mom = group["weight_decay"], group["lr"], group["momentum"]
            if wd:
                grads = torch._foreach_add(grads, params, alpha=wd)
            if group.get("lars", True):
                pn = torch._foreach_norm(params)
                gn = torch._foreach_norm(grads)
                scales = []
                for w, gnorm in zip(pn, gn):
                    trust = torch.where((w > 0) & (gnorm > 0), group["eta"] * w / (gnorm + group["eps"]),
                                        torch.ones_like(w))
                    scales.append(trust)
                grads = [g * s for g, s in zip(grads, scales)]
            bufs = []
            for p, g in zip(params, grads):
                st = self.state[p]
                if "momentum_buffer" not in st:
                    st["momentum_buffer"] = torch.clone(g).detach()
                else:
                    st["momentum_buffer"].mul_(mom).add_(g)
                bufs.append(st["momentum_buffer"])
            torch._foreach_add_(params, bufs, alpha=-lr)
        return loss
