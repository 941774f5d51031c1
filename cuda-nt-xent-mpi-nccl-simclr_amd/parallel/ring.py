"""Ring-negatives NT-Xent: global-batch negatives with O(local) memory.

The all-gather path (``parallel.distributed``) holds every rank's normalised rows, the kept
cosines and the coefficient matrix for all W*R columns: O(R * W R) per GPU, which 288 GB of
HBM3E covers up to about a hundred 8192-row ranks. Past that, this mode passes one rank's rows
around the ring at a time (ring-attention analogue over the negatives axis): at step s rank r
holds the rows of rank q = (r - s) mod W, sends them on to r + 1 and receives the next block
from r - 1 while the MFMA kernels consume the current one. Per block:

* forward: the similarity tiles of column block q (the upper triangle for q = r) fold their
  per-tile (max, sum) partials into the per-column-tile LSE state; nothing of size W R x R
  is stored. After the ring: LSE merge, LSE all-gather (W * Rpad floats), loss all-reduce.
* backward: the ring runs again; each block's coefficients C_{r,q} are recomputed from the
  rows (MFMA GEMM with the coefficient epilogue) into a compact R x R buffer, Z_q is
  transposed locally, and dZ += C_{r,q} Z_q accumulates in fp32.

Peak extra memory: two ring buffers of R x d, one R x R coefficient block, the fp32 dZ.
Compute is the all-gather path's recompute mode plus one transpose per block; the ring's
point-to-point sends use one xGMI link per step, so prefer the all-gather path whenever its
buffers fit. The reference has no multi-GPU code at all; the math is
``reference.sharded_forward_backward`` (tests compare against the fp64 oracle).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..ops import _ext
from ..ops.ntxent import resolve_compute
from .commstats import comm_reserve_cus, span
from .distributed import _all_gather_into, _is_gloo, _world

_TILE_CACHE: Dict[tuple, Dict[int, torch.Tensor]] = {}


def block_tiles(C, plan, device) -> Dict[int, torch.Tensor]:
    """Forward tiles of the plan grouped by column block (rank): {q: int32 [n, 4] on device}.
    The own block keeps its upper triangle (diagonal / mirrored kinds)."""
    key = (plan.rows, plan.dim, plan.world, plan.rank, device.index)
    hit = _TILE_CACHE.get(key)
    if hit is not None:
        return hit
    rt = plan.row_tiles
    per: Dict[int, List[Tuple[int, int, int, int]]] = {q: [] for q in range(plan.world)}
    for ti, tj, kind in C.fwd_tile_list(plan.rows, plan.dim, plan.world, plan.rank):
        per[tj // rt].append((ti, tj, kind, 0))
    out = {q: torch.tensor(v, dtype=torch.int32).reshape(-1, 4).to(device) for q, v in per.items()}
    _TILE_CACHE[key] = out
    return out


def _exchange(send: torch.Tensor, recv: torch.Tensor, group):
    """Send ``send`` to rank r+1 and receive rank r-1's block into ``recv``. Returns work
    handles to wait on (RCCL: asynchronous on the communicator's stream)."""
    W, r = _world(group)
    nxt, prv = (r + 1) % W, (r - 1) % W
    g_nxt = dist.get_global_rank(group, nxt) if group is not None else nxt
    g_prv = dist.get_global_rank(group, prv) if group is not None else prv
    if _is_gloo(group):  # host staging: gloo point-to-point moves CPU tensors only
        s_cpu, r_cpu = send.detach().cpu(), torch.empty(recv.shape, dtype=recv.dtype)
        if r % 2 == 0:
            dist.send(s_cpu, g_nxt, group=group)
            dist.recv(r_cpu, g_prv, group=group)
        else:
            dist.recv(r_cpu, g_prv, group=group)
            dist.send(s_cpu, g_nxt, group=group)
        recv.copy_(r_cpu)
        return []
    ops = [dist.P2POp(dist.isend, send, g_nxt, group), dist.P2POp(dist.irecv, recv, g_prv, group)]
    return dist.batch_isend_irecv(ops)


def _ring(zq: torch.Tensor, group, fn):
    """Calls fn(q, rows_of_q, reserve_cus) for q = r, r-1, ..., r-W+1 while the next block
    travels; reserve_cus = the CUs its GEMMs leave free for the transfer in flight."""
    W, r = _world(group)
    bufs = [torch.empty_like(zq), torch.empty_like(zq)] if W > 1 else []
    cur = zq
    for s in range(W):
        q = (r - s) % W
        works = []
        nxt = None
        if s < W - 1:
            nxt = bufs[s % 2]
            works = _exchange(cur, nxt, group)
        fn(q, cur, comm_reserve_cus(dist.get_backend(group)) if works else 0)
        with span("ring_rows"):
            for w in works:
                w.wait()
        if nxt is not None:
            cur = nxt


class RingNTXentFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h: torch.Tensor, temperature: float, compute: str, group):
        C = _ext.load()
        W, r = _world(group)
        h = h.contiguous()
        R, d = h.shape
        plan = C.get_plan(R, d, W, r, float(temperature), compute, h.device.index)
        if plan.compute_dtype == "fp8":
            raise ValueError("ring negatives run fp32/fp16/bf16 compute (fp8 keeps cosines: use the all-gather path)")
        Rpad, rt = plan.rows_pad, plan.row_tiles
        zq, inv, ypos, _ = C.prep(h, plan)
        tiles = block_tiles(C, plan, h.device)
        part = torch.empty((plan.col_tiles, Rpad, 2), dtype=torch.float32, device=h.device)
        _ring(zq, group, lambda q, rows, res: C.fwd_stats_tiles(zq, rows, q * rt, tiles[q], plan, part, reserve_cus=res))
        lse2_all = torch.empty((W * Rpad,), dtype=torch.float32, device=h.device)
        cpos = torch.empty((Rpad,), dtype=torch.float32, device=h.device)
        loss = C.lse(part, ypos, lse2_all, cpos, plan)
        if W > 1:
            mine = lse2_all[r * Rpad:(r + 1) * Rpad].clone()
            with span("lse_loss"):
                _all_gather_into(lse2_all, mine, group)
                dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=group)
        ctx.plan, ctx.group = plan, group
        ctx.save_for_backward(h, zq, inv, lse2_all, cpos)
        return loss

    @staticmethod
    def backward(ctx, grad_out: torch.Tensor):
        C = _ext.load()
        h, zq, inv, lse2_all, cpos = ctx.saved_tensors
        plan, group = ctx.plan, ctx.group
        rt = plan.row_tiles
        tiles = block_tiles(C, plan, h.device)
        acc: List[Optional[torch.Tensor]] = [None]

        def block(q, rows, res):
            cb = C.coef_gemm_tiles(zq, rows, q * rt, tiles[q], lse2_all, cpos, plan, rt, q * rt, reserve_cus=res)
            slabs = C.dz_block(cb, C.transpose(rows, plan), plan, reserve_cus=res)
            acc[0] = slabs if acc[0] is None else acc[0].add_(slabs)

        _ring(zq, group, block)
        dh = C.norm_bwd(acc[0], h, inv, grad_out.reshape(1), plan)
        return dh, None, None, None


def ring_ntxent_loss(h_local: torch.Tensor, temperature: float = 0.07, *, group=None, compute: str = "auto",
                     use_mixed_precision: bool = False) -> torch.Tensor:
    """Global NT-Xent over the group with ring-passed negatives (O(local) memory); same value
    and gradient as :func:`parallel.distributed.dist_ntxent_loss`."""
    if not h_local.is_cuda:
        from .distributed import cpu_dist_ntxent_loss

        return cpu_dist_ntxent_loss(h_local, temperature, group=group)
    comp = resolve_compute(h_local.dtype, use_mixed_precision, compute)
    return RingNTXentFunction.apply(h_local, float(temperature), comp, group)
