"""Single-GPU emulation of the W-rank data-parallel NT-Xent (testing / debugging aid).

Runs every virtual rank's stage ops (the same HIP kernels and per-rank plans the RCCL path
uses: own-rank upper-triangular tiles, remote column blocks with global column indices,
per-rank LSE slot, rank-local symmetric backward) sequentially on one device. The
collectives are replaced by construction: each rank's ``prep``/``transpose`` writes into its
slot of the shared gathered buffers, and each rank's LSE lands in its slot of ``lse2_all``.
This is what lets a 1-GPU box verify the multi-GPU math bit-for-bit (the real path differs
only in who fills the other slots).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from ..ops import _ext
from ..ops.ntxent import resolve_compute


def emulated_dist_forward_backward(shards: Sequence[torch.Tensor], temperature: float, *, compute: str = "auto",
                                   keep_logits: bool = True, grad_out: float = 1.0
                                   ) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """Loss (global mean over all W*R rows) and per-rank dL/dh_r for shards h_r = [h1_r; h2_r]."""
    C = _ext.load()
    W = len(shards)
    R, d = shards[0].shape
    dev = shards[0].device
    comp = resolve_compute(shards[0].dtype, False, compute)
    plans = [C.get_plan(R, d, W, r, float(temperature), comp, dev.index) for r in range(W)]
    P0 = plans[0]
    Rpad = P0.rows_pad
    f8 = P0.compute_dtype == "fp8"
    keep_logits = keep_logits or f8  # fp8 plans always keep their (fp16) cosines
    cdt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[P0.backward_dtype]
    zq_all = torch.empty((W * Rpad, P0.ld_k), dtype=cdt, device=dev)
    zqt_all = torch.empty((W, P0.dim_n, P0.ld_t), dtype=cdt, device=dev)
    zq8_all = torch.empty((W * Rpad, P0.ld_k8), dtype=torch.uint8, device=dev) if f8 else None
    invs, yposs = [], []
    for r in range(W):  # "all-gather" of Zq / ZqT: every rank writes its own slot
        zq = zq_all[r * Rpad:(r + 1) * Rpad]
        zq8 = zq8_all[r * Rpad:(r + 1) * Rpad] if f8 else None
        _, inv, ypos, _ = C.prep(shards[r].contiguous(), plans[r], zq, zq8)
        C.transpose(zq, plans[r], zqt_all[r])
        invs.append(inv)
        yposs.append(ypos)
    fwd_all = zq8_all if f8 else zq_all  # forward GEMM operand
    lse2_all = torch.empty((W * Rpad,), dtype=torch.float32, device=dev)
    loss = torch.zeros((), dtype=torch.float32, device=dev)
    scs, cposs = [], []
    for r in range(W):
        P = plans[r]
        part = torch.empty((P.col_tiles, Rpad, 2), dtype=torch.float32, device=dev)
        sc = torch.empty((P.n_fwd_tiles * 256 * 256,), dtype=cdt, device=dev) if keep_logits else None
        C.fwd_stats_range(fwd_all[r * Rpad:(r + 1) * Rpad], fwd_all, P, part, sc, 0, P.n_fwd_tiles)
        cpos = torch.empty((Rpad,), dtype=torch.float32, device=dev)
        loss = loss + C.lse(part, yposs[r], lse2_all, cpos, P)  # "all-gather" of LSE + "all-reduce"
        scs.append(sc)
        cposs.append(cpos)
    go = torch.tensor([grad_out], dtype=torch.float32, device=dev)
    grads = []
    for r in range(W):
        P = plans[r]
        zq = zq_all[r * Rpad:(r + 1) * Rpad]
        cb = C.coef(scs[r], lse2_all, cposs[r], P) if keep_logits else C.coef_gemm(zq, zq_all, lse2_all, cposs[r], P)
        slabs = C.dz(cb, zqt_all, P)
        grads.append(C.norm_bwd(slabs, shards[r].contiguous(), invs[r], go, P))
    return loss, grads


def emulated_ring_forward_backward(shards: Sequence[torch.Tensor], temperature: float, *, compute: str = "auto",
                                   grad_out: float = 1.0) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """The ring-negatives stage ops (:mod:`parallel.ring`) for W virtual ranks on one device:
    every rank r visits the column blocks q = r, r-1, ... with rank q's rows as the chunk."""
    from .ring import block_tiles

    C = _ext.load()
    W = len(shards)
    R, d = shards[0].shape
    dev = shards[0].device
    comp = resolve_compute(shards[0].dtype, False, compute)
    plans = [C.get_plan(R, d, W, r, float(temperature), comp, dev.index) for r in range(W)]
    Rpad, rt = plans[0].rows_pad, plans[0].row_tiles
    preps = [C.prep(shards[r].contiguous(), plans[r]) for r in range(W)]
    zqs = [p[0] for p in preps]
    lse2_all = torch.empty((W * Rpad,), dtype=torch.float32, device=dev)
    loss = torch.zeros((), dtype=torch.float32, device=dev)
    cposs = []
    for r in range(W):
        P = plans[r]
        tiles = block_tiles(C, P, dev)
        part = torch.empty((P.col_tiles, Rpad, 2), dtype=torch.float32, device=dev)
        for s in range(W):
            q = (r - s) % W
            C.fwd_stats_tiles(zqs[r], zqs[q], q * rt, tiles[q], P, part)
        cpos = torch.empty((Rpad,), dtype=torch.float32, device=dev)
        loss = loss + C.lse(part, preps[r][2], lse2_all, cpos, P)
        cposs.append(cpos)
    go = torch.tensor([grad_out], dtype=torch.float32, device=dev)
    grads = []
    for r in range(W):
        P = plans[r]
        tiles = block_tiles(C, P, dev)
        acc = None
        for s in range(W):
            q = (r - s) % W
            cb = C.coef_gemm_tiles(zqs[r], zqs[q], q * rt, tiles[q], lse2_all, cposs[r], P, rt, q * rt)
            slabs = C.dz_block(cb, C.transpose(zqs[q], P), P)
            acc = slabs if acc is None else acc + slabs
        grads.append(C.norm_bwd(acc, shards[r].contiguous(), preps[r][1], go, P))
    return loss, grads


def emulated_sym_forward_backward(shards: Sequence[torch.Tensor], temperature: float, *, compute: str = "auto",
                                  grad_out: float = 1.0) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """The symmetric data-parallel stage ops (:mod:`parallel.symmetric`) for W virtual ranks on
    one device: each rank computes only its assigned cross blocks; the point-to-point
    exchanges (column partials, partner gradient contributions) become copies."""
    from .symmetric import (sym_coef, sym_grad_slabs, sym_jobs, sym_norm_bwd, sym_own_grad, sym_partner_grads,
                            sym_tiles)

    C = _ext.load()
    W = len(shards)
    R, d = shards[0].shape
    dev = shards[0].device
    comp = resolve_compute(shards[0].dtype, False, compute)
    plans = [C.get_plan(R, d, W, r, float(temperature), comp, dev.index) for r in range(W)]
    P0 = plans[0]
    Rpad, rt = P0.rows_pad, P0.row_tiles
    f8 = P0.compute_dtype == "fp8"
    cdt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[P0.backward_dtype]
    zq_all = torch.empty((W * Rpad, P0.ld_k), dtype=cdt, device=dev)
    zqt_all = torch.empty((W, P0.dim_n, P0.ld_t), dtype=cdt, device=dev)
    zq8_all = torch.empty((W * Rpad, P0.ld_k8), dtype=torch.uint8, device=dev) if f8 else None
    invs, yposs = [], []
    for r in range(W):
        zq = zq_all[r * Rpad:(r + 1) * Rpad]
        _, inv, ypos, _ = C.prep(shards[r].contiguous(), plans[r], zq, zq8_all[r * Rpad:(r + 1) * Rpad] if f8 else None)
        C.transpose(zq, plans[r], zqt_all[r])
        invs.append(inv)
        yposs.append(ypos)
    fwd_all = zq8_all if f8 else zq_all
    parts, parts_x, scs, tiles = [], [], [], []
    for r in range(W):
        P = plans[r]
        t, n = sym_tiles(C, P, dev)
        part = torch.empty((P.col_tiles, Rpad, 2), dtype=torch.float32, device=dev)
        part_x = torch.empty_like(part)
        sc = torch.empty((n * 256 * 256,), dtype=cdt, device=dev)
        C.fwd_stats_sym(fwd_all[r * Rpad:(r + 1) * Rpad], fwd_all, t, P, part, part_x, sc, 0, n)
        parts.append(part)
        parts_x.append(part_x)
        scs.append(sc)
        tiles.append(t)
    for r in range(W):  # "send" column partials to their owners
        for (q, m0, m1, k0, k1) in sym_jobs(W, r, rt):
            parts[q][r * rt + m0:r * rt + m1, k0 * 256:k1 * 256].copy_(parts_x[r][q * rt + m0:q * rt + m1, k0 * 256:k1 * 256])
    lse2_all = torch.empty((W * Rpad,), dtype=torch.float32, device=dev)
    loss = torch.zeros((), dtype=torch.float32, device=dev)
    cposs = []
    for r in range(W):
        cpos = torch.empty((Rpad,), dtype=torch.float32, device=dev)
        loss = loss + C.lse(parts[r], yposs[r], lse2_all, cpos, plans[r])
        cposs.append(cpos)
    go = torch.tensor([grad_out], dtype=torch.float32, device=dev)
    bufs = [sym_coef(C, plans[r], W, tiles[r], scs[r], lse2_all, cposs[r]) for r in range(W)]
    sent = [sym_partner_grads(C, plans[r], W, r, bufs[r][1], zqt_all) for r in range(W)]
    grads = []
    for r in range(W):
        own, recv, views = sym_grad_slabs(plans[r], W, r, dev)
        sym_own_grad(C, plans[r], W, r, bufs[r][0], zqt_all, own[0])
        for p, view in views.items():  # "receive"
            view.copy_(sent[p][r])
        grads.append(sym_norm_bwd(C, plans[r], own, recv, shards[r].contiguous(), invs[r], go))
    return loss, grads
