"""Pure-PyTorch NT-Xent oracle (CPU or GPU, any dtype; fp64 for gradchecks).

This is the *correct* SimCLR NT-Xent that the reference intends. The
reference itself computes something else (self-similarity diagonal of a scrambled GEMM,
``src/ntxent_kernel.cu:117,161-173``) and its backward ignores ``grad_out``
(``src/ntxent_kernel.cu:221``), so parity targets these formulas, not its outputs.

Notation: ``h = [h1; h2]`` of shape ``[2N, d]``; ``z = h / max(||h||, eps)``;
``S = z z^T / tau`` with the diagonal masked; positive ``p(i) = (i + N) mod 2N``;
``lse_i = log sum_{j != i} exp S_ij``; ``loss = mean_i (lse_i - S_{i,p(i)})``.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch

EPS = 1e-12


def normalize(h: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Return (z, inv_norm) with z = h * inv_norm, inv_norm = 1/max(||h||, eps)."""
    inv = 1.0 / h.norm(dim=1).clamp_min(EPS)
    return h * inv.unsqueeze(1), inv


def positive_index(rows: int, device=None) -> torch.Tensor:
    n = rows // 2
    return (torch.arange(rows, device=device) + n) % rows


def logits(h: torch.Tensor, temperature: float) -> torch.Tensor:
    z, _ = normalize(h)
    S = z @ z.t() / temperature
    mask = torch.eye(h.shape[0], dtype=torch.bool, device=h.device)
    return S.masked_fill(mask, float("-inf"))


def ntxent_loss(h: torch.Tensor, temperature: float = 0.07) -> torch.Tensor:
    """Autograd-capable NT-Xent on stacked views ``h = [h1; h2]``."""
    if h.dim() != 2 or h.shape[0] % 2:
        raise ValueError("h must be [2N, d] with stacked views")
    S = logits(h, temperature)
    pos = positive_index(h.shape[0], h.device)
    return torch.nn.functional.cross_entropy(S, pos, reduction="mean")


def ntxent_loss_pair(z1: torch.Tensor, z2: torch.Tensor, temperature: float = 0.07) -> torch.Tensor:
    return ntxent_loss(torch.cat([z1, z2], 0), temperature)


def ntxent_stats(h: torch.Tensor, temperature: float = 0.07):
    """(loss, lse[2N], pos_logit[2N]) in the dtype of h."""
    S = logits(h, temperature)
    lse = torch.logsumexp(S, dim=1)
    pos = positive_index(h.shape[0], h.device)
    pl = S.gather(1, pos.unsqueeze(1)).squeeze(1)
    return (lse - pl).mean(), lse, pl


def ntxent_backward_analytic(h: torch.Tensor, temperature: float, grad_out: float | torch.Tensor = 1.0,
                             lse: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Closed-form gradient via the symmetric trick (what the HIP backward implements).

    C = P + P^T - 2 I_pos, dL/dz = C z / (2N tau), dL/dh = inv (dz - z (z . dz)).
    """
    R = h.shape[0]
    z, inv = normalize(h)
    S = logits(h, temperature)
    if lse is None:
        lse = torch.logsumexp(S, dim=1)
    P = torch.exp(S - lse.unsqueeze(1))
    pos = positive_index(R, h.device)
    C = P + P.t()
    C[torch.arange(R, device=h.device), pos] -= 2.0
    dz = (C @ z) * (torch.as_tensor(grad_out, dtype=h.dtype, device=h.device) / (R * temperature))
    dot = (z * dz).sum(1, keepdim=True)
    return inv.unsqueeze(1) * (dz - z * dot)


# ---------------------------------------------------------------------------------------
# Data-parallel layout: rank r holds h_r = [h1_r; h2_r] (2n rows); positives are rank-local.
# ---------------------------------------------------------------------------------------
def global_pair_order(shards: Sequence[torch.Tensor]) -> torch.Tensor:
    """Re-stack per-rank shards into the single-process [view1; view2] layout (same pairs)."""
    n = shards[0].shape[0] // 2
    v1 = torch.cat([s[:n] for s in shards], 0)
    v2 = torch.cat([s[n:] for s in shards], 0)
    return torch.cat([v1, v2], 0)


def sharded_forward_backward(shards: Sequence[torch.Tensor], temperature: float,
                             grad_out: float = 1.0) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """Simulate the W-rank algorithm in one process: each rank uses only its rows, the
    gathered normalised embeddings and the gathered LSE (no column-gradient exchange)."""
    W = len(shards)
    R = shards[0].shape[0]
    n = R // 2
    zs, invs = zip(*[normalize(s) for s in shards])
    z_all = torch.cat(zs, 0)
    N2 = W * R
    lses, losses = [], []
    for r in range(W):
        S = zs[r] @ z_all.t() / temperature
        own = torch.arange(R, device=S.device) + r * R
        S[torch.arange(R), own] = float("-inf")
        lse = torch.logsumexp(S, 1)
        pos = (torch.arange(R) + n) % R + r * R
        losses.append((lse - S[torch.arange(R), pos]).sum())
        lses.append(lse)
    lse_all = torch.cat(lses)
    loss = torch.stack(losses).sum() / N2
    grads = []
    for r in range(W):
        S = zs[r] @ z_all.t() / temperature
        own = torch.arange(R) + r * R
        Pr = torch.exp(S - lses[r].unsqueeze(1))
        Pc = torch.exp(S - lse_all.unsqueeze(0))
        C = Pr + Pc
        C[torch.arange(R), own] = 0.0
        pos = (torch.arange(R) + n) % R + r * R
        C[torch.arange(R), pos] -= 2.0
        dz = C @ z_all * (grad_out / (N2 * temperature))
        z = zs[r]
        dot = (z * dz).sum(1, keepdim=True)
        grads.append(invs[r].unsqueeze(1) * (dz - z * dot))
    return loss, grads


# ---------------------------------------------------------------------------------------
# What the reference computes as written (for documentation / contrast tests only).
# ---------------------------------------------------------------------------------------
def reference_as_written_forward(z: torch.Tensor, T: float) -> torch.Tensor:
    """Emulates src/ntxent_kernel.cu:160-200 (column-major cuBLAS with lda=2B on row-major
    data, self-diagonal target). Kept to document why parity targets the correct math."""
    B, D = z.shape
    zc = torch.cat([z, z], 0)  # :161
    A = zc.reshape(-1)[: 2 * B * D].reshape(D, 2 * B).t()  # lda=2B read of row-major memory
    L = A @ A.t() / T
    P = torch.softmax(L, dim=1)
    return -torch.log(torch.diagonal(P)).mean()


def flops_fwd_bwd(rows_local: int, rows_global: int, dim: int, symmetric_local: bool = True,
                  symmetric_global: bool = False) -> float:
    """MFMA FLOPs of one rank's fwd+bwd (store mode): fwd S GEMM (upper-triangular in the
    own-rank block; with ``symmetric_global`` each cross-rank block counted once per pair, i.e.
    half per rank, as parallel/symmetric.py executes it) + dZ GEMM. For TFLOP/s reporting."""
    own = rows_local * rows_local * dim * 2.0
    remote = rows_local * (rows_global - rows_local) * dim * 2.0
    fwd = (own / 2 if symmetric_local else own) + (remote / 2 if symmetric_global else remote)
    bwd = rows_local * rows_global * dim * 2.0
    return fwd + bwd


def expected_random_loss(rows: int) -> float:
    """Loss of an uninformative model: log(2N - 1)."""
    return math.log(rows - 1)
