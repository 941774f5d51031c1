"""Symmetric global-batch negatives: every rank pair's similarity block is computed ONCE.

The all-gather path (``parallel.distributed``) has every rank r compute its full row block
S_{r,:} = Z_r Z_all^T / tau, so each off-diagonal block S_{r,q} is computed twice in the group
(once as S_{r,q} by r, once as S_{q,r} = S_{r,q}^T by q). Here the W(W-1)/2 off-diagonal
blocks are split evenly: rank r computes the blocks (r, r+1), ..., (r, r+(W-1)//2) (mod W) in
full and, for even W, half of the block (r, r + W/2) (the pair shares it by row tiles). For
each tile of a block it computes, the forward GEMM epilogue emits the row partials (for r's
rows) AND the column partials (for q's rows), and the kept cosines give both coefficient
blocks C_{r,q} and C_{q,r} = C_{r,q}^T. This is the north star's "reduce-scatter of
embedding grads on the backward" (BASELINE.json), done point to point over xGMI:

* forward: prep -> Zq sent point-to-point to the ranks that compute against it (half of an
  all-gather's traffic: 4 x 32 MiB per rank at W = 8, one grouped batch so every peer's
  transfer runs on its own link at once) while the own upper-triangular tiles run -> the
  assigned cross tiles -> column partials (2 MiB per block at B=4096) sent to their owners ->
  LSE -> LSE all-gather + loss all-reduce.
* backward: partners' ZqT blocks transposed locally; coefficient pass (own tiles mirrored in
  place, cross tiles mirrored into a
  per-partner buffer) -> the partners' gradient contributions C_{q,r} Z_r (MFMA dZ GEMMs),
  sent point-to-point as soon as they exist (fp16 for reduced-precision plans: 32 MiB per
  block) -> this rank's own
  contributions C_{r,q} Z_q accumulate in the dZ epilogue while the sends run -> received
  contributions added -> L2-normalisation backward.

Per GPU at W = 8 (B = 4096/view, d = 2048) the forward similarity work drops from 7.5 to 4
blocks of 8192 x 8192 x 2048 and the coefficient pass from 7.5 to 4 blocks; the dZ GEMMs stay
at 8 blocks (half of them produce the partners' contributions). Traffic: 3.5 x 32 MiB of fp16
dZ contributions per rank, each to a different peer (one xGMI link each), overlapped with the
own-row dZ GEMMs.

The reference has no multi-GPU code at all; the math is SURVEY.md §2.2.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.distributed as dist

from ..ops import _ext, reference
from ..ops.ntxent import resolve_compute
from .commstats import comm_reserve_cus, span
from .distributed import _all_gather_into, _is_gloo, _world

Job = Tuple[int, int, int, int, int]  # (q, m0, m1, k0, k1): my row tiles [m0,m1) x q's row tiles [k0,k1)


def sym_jobs(world: int, rank: int, row_tiles: int) -> List[Job]:
    """Blocks rank ``rank`` computes: (q, m0, m1, k0, k1) = its row tiles [m0, m1) against
    rank q's row tiles [k0, k1). Every unordered pair {r, q} (r != q) is covered exactly once
    across the group; for even W the pair at distance W/2 is split by the lower rank's row
    tiles (lower rank: its tiles [0, h); upper rank: all its tiles x the lower rank's [h, rt))."""
    W, r, rt = world, rank, row_tiles
    jobs: List[Job] = []
    for d in range(1, (W - 1) // 2 + 1):
        jobs.append(((r + d) % W, 0, rt, 0, rt))
    if W % 2 == 0 and W > 1:
        q = (r + W // 2) % W
        h = (rt + 1) // 2
        job = (q, 0, h, 0, rt) if r < q else (q, 0, rt, h, rt)
        if job[1] < job[2] and job[3] < job[4]:
            jobs.append(job)
    return jobs


def sym_incoming(world: int, rank: int, row_tiles: int) -> List[Job]:
    """Jobs of OTHER ranks that involve ``rank``'s rows: (p, m0, m1, k0, k1) with rank p
    computing its row tiles [m0, m1) against this rank's row tiles [k0, k1)."""
    out: List[Job] = []
    for p in range(world):
        if p == rank:
            continue
        for (q, m0, m1, k0, k1) in sym_jobs(world, p, row_tiles):
            if q == rank:
                out.append((p, m0, m1, k0, k1))
    return out


def sym_chunk_bounds(row_tiles: int, nchunks: int) -> List[Tuple[int, int]]:
    """Row-tile ranges of the forward exchange chunks (as build_sym_fwd_tiles)."""
    return [(row_tiles * c // nchunks, row_tiles * (c + 1) // nchunks) for c in range(nchunks)]


def sym_num_chunks(row_tiles: int) -> int:
    """Forward rows travel in up to 4 chunks (8 MiB each at B=4096, d=2048): the cross tiles of
    chunk c start while chunk c+1 is on the wire."""
    return max(1, min(4, row_tiles))


def sym_chunk_segments(plan, jobs: List[Job], nchunks: int) -> List[Tuple[int, int]]:
    """(first, count) of each chunk's cross tiles in the symmetric forward tile list."""
    out, first = [], plan.n_own_tiles
    for (c0, c1) in sym_chunk_bounds(plan.row_tiles, nchunks):
        n = sum((m1 - m0) * max(0, min(k1, c1) - max(k0, c0)) for (_, m0, m1, k0, k1) in jobs)
        out.append((first, n))
        first += n
    return out


def sym_work_blocks(world: int, row_tiles: int) -> List[float]:
    """Cross-block tiles per rank in units of full blocks (balance check)."""
    return [sum((m1 - m0) * (k1 - k0) for (_, m0, m1, k0, k1) in sym_jobs(world, r, row_tiles)) / row_tiles ** 2
            for r in range(world)]


def _grank(group, r: int) -> int:
    return dist.get_global_rank(group, r) if group is not None else r


def _p2p(sends, recvs, group):
    """Point-to-point exchange: ``sends`` = [(tensor, dst)], ``recvs`` = [(tensor, src)] (group
    ranks). RCCL: one grouped batch on the communicator's stream, returns work handles. gloo
    (CPU transport for the 1-GPU rehearsals): host-staged isend/irecv, completed on return."""
    if not sends and not recvs:
        return []
    if _is_gloo(group):
        reqs, back = [], []
        for t, dst in sends:
            c = t.detach().contiguous().cpu()
            back.append(c)  # keep alive until sent
            reqs.append(dist.isend(c, _grank(group, dst), group=group))
        for t, src in recvs:
            c = torch.empty(t.shape, dtype=t.dtype)
            reqs.append(dist.irecv(c, _grank(group, src), group=group))
            back.append((t, c))
        for q in reqs:
            q.wait()
        for item in back:
            if isinstance(item, tuple):
                item[0].copy_(item[1])
        return []
    ops = [dist.P2POp(dist.isend, t, _grank(group, dst), group) for t, dst in sends]
    ops += [dist.P2POp(dist.irecv, t, _grank(group, src), group) for t, src in recvs]
    return dist.batch_isend_irecv(ops)


_TILES: Dict[tuple, Tuple[torch.Tensor, int]] = {}


def sym_tiles(C, plan, device) -> Tuple[torch.Tensor, int]:
    key = (plan.rows, plan.dim, plan.world, plan.rank, device.index)
    hit = _TILES.get(key)
    if hit is None:
        jobs = sym_jobs(plan.world, plan.rank, plan.row_tiles)
        t = C.sym_fwd_tiles(plan, jobs, sym_num_chunks(plan.row_tiles))
        hit = (t, int(t.shape[0]))
        _TILES[key] = hit
    return hit


class SymNTXentFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h: torch.Tensor, temperature: float, compute: str, group):
        C = _ext.load()
        W, r = _world(group)
        h = h.contiguous()
        R, d = h.shape
        plan = C.get_plan(R, d, W, r, float(temperature), compute, h.device.index)
        Rpad, rt = plan.rows_pad, plan.row_tiles
        f8 = plan.compute_dtype == "fp8"
        cdt = {"fp32": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}[plan.backward_dtype]
        dev = h.device
        zq_all = torch.empty((W * Rpad, plan.ld_k), dtype=cdt, device=dev)
        zqt_all = torch.empty((W, plan.dim_n, plan.ld_t), dtype=cdt, device=dev)
        zq = zq_all[r * Rpad:(r + 1) * Rpad]
        fwd_all = torch.empty((W * Rpad, plan.ld_k8), dtype=torch.uint8, device=dev) if f8 else zq_all
        fwd = fwd_all[r * Rpad:(r + 1) * Rpad]
        _, inv, ypos, _ = C.prep(h, plan, zq, fwd if f8 else None)
        C.transpose(zq, plan, zqt_all[r])
        # rows travel only where a block needs them: to the ranks that compute against this
        # rank's rows (only the row tiles they use) and from the ranks this one computes
        # against -- half of an all-gather's traffic. Chunk c of the rows is one grouped batch
        # (RCCL runs a group's peers concurrently over their own xGMI links; the chunks follow
        # each other on the communicator's stream), and the cross tiles of chunk c run while
        # chunk c+1 is on the wire. The partners' ZqT blocks are transposed locally in the
        # backward.
        jobs = sym_jobs(W, r, rt)
        inc = sym_incoming(W, r, rt)
        nch = sym_num_chunks(rt)
        works = []
        for (c0, c1) in sym_chunk_bounds(rt, nch):
            sends, recvs = [], []
            for (p, m0, m1, k0, k1) in inc:  # p uses my row tiles [k0, k1)
                a0, a1 = max(k0, c0), min(k1, c1)
                if a0 < a1:
                    sends.append((fwd[a0 * 256:a1 * 256], p))
            for (q, m0, m1, k0, k1) in jobs:  # I use q's row tiles [k0, k1)
                a0, a1 = max(k0, c0), min(k1, c1)
                if a0 < a1:
                    recvs.append((fwd_all[q * Rpad + a0 * 256:q * Rpad + a1 * 256], q))
            works.append(_p2p(sends, recvs, group))
        if f8:  # the backward runs on the fp16 rows: after the forward chunks
            works_f16 = _p2p([(zq[k0 * 256:k1 * 256], p) for (p, m0, m1, k0, k1) in inc],
                             [(zq_all[q * Rpad + k0 * 256:q * Rpad + k1 * 256], q) for (q, m0, m1, k0, k1) in jobs], group)
        else:
            works_f16 = []
        tiles, ntiles = sym_tiles(C, plan, dev)
        part = torch.empty((plan.col_tiles, Rpad, 2), dtype=torch.float32, device=dev)
        part_x = torch.empty_like(part)
        sc = torch.empty((ntiles * 256 * 256,), dtype=cdt, device=dev)
        reserve = comm_reserve_cus(dist.get_backend(group))
        # chunk 0 of the rows is on the wire
        C.fwd_stats_sym(fwd, fwd_all, tiles, plan, part, part_x, sc, 0, plan.n_own_tiles, reserve_cus=reserve)
        segs = sym_chunk_segments(plan, jobs, nch)
        for c, (ws, (first, count)) in enumerate(zip(works, segs)):
            with span("fwd_rows"):
                for w in ws:
                    w.wait()
            # the next chunk (or the fp16 rows of an fp8 plan) is still on the wire
            more = c + 1 < len(works) and bool(works[c + 1]) or bool(works_f16)
            C.fwd_stats_sym(fwd, fwd_all, tiles, plan, part, part_x, sc, first, count,
                            reserve_cus=reserve if more else 0)
        with span("fwd_rows"):
            for w in works_f16:
                w.wait()
        # column partials of the cross tiles -> their rows' owners (part slots [r*rt + m0, r*rt + m1))
        sends = [(part_x[q * rt + m0:q * rt + m1, k0 * 256:k1 * 256].contiguous(), q) for (q, m0, m1, k0, k1) in jobs]
        recvs = [(torch.empty((m1 - m0, (k1 - k0) * 256, 2), dtype=torch.float32, device=dev), p)
                 for (p, m0, m1, k0, k1) in inc]
        with span("fwd_col_partials"):
            for w in _p2p(sends, recvs, group):
                w.wait()
        for (buf, _), (p, m0, m1, k0, k1) in zip(recvs, inc):
            part[p * rt + m0:p * rt + m1, k0 * 256:k1 * 256].copy_(buf)
        lse2_all = torch.empty((W * Rpad,), dtype=torch.float32, device=dev)
        cpos = torch.empty((Rpad,), dtype=torch.float32, device=dev)
        loss = C.lse(part, ypos, lse2_all, cpos, plan)
        mine = lse2_all[r * Rpad:(r + 1) * Rpad].clone()
        with span("lse_loss"):
            _all_gather_into(lse2_all, mine, group)
            dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=group)
        ctx.plan, ctx.group = plan, group
        ctx.sc = sc
        ctx.save_for_backward(h, inv, zq_all, zqt_all, lse2_all, cpos, tiles)
        return loss

    @staticmethod
    def backward(ctx, grad_out: torch.Tensor):
        C = _ext.load()
        h, inv, zq_all, zqt_all, lse2_all, cpos, tiles = ctx.saved_tensors
        plan, group = ctx.plan, ctx.group
        sc, ctx.sc = ctx.sc, None
        if sc is None:
            raise RuntimeError("symmetric NT-Xent: backward called twice (kept cosines already consumed)")
        W, r = _world(group)
        Rpad = plan.rows_pad
        for (q, *_) in sym_jobs(W, r, plan.row_tiles):  # partners' B operands of the own dZ GEMMs
            C.transpose(zq_all[q * Rpad:(q + 1) * Rpad], plan, zqt_all[q])
        dh = sym_backward_local(C, plan, W, r, h, inv, zqt_all, lse2_all, cpos, tiles, sc, grad_out, group)
        return dh, None, None, None


def _split_jobs(jobs: List[Job], rt: int):
    """(full jobs, split job or None): full jobs come first in slot order (partners r+1, r+2, ...)."""
    full = [j for j in jobs if (j[1], j[2], j[3], j[4]) == (0, rt, 0, rt)]
    rest = [j for j in jobs if (j[1], j[2], j[3], j[4]) != (0, rt, 0, rt)]
    assert jobs[:len(full)] == full and len(rest) <= 1
    return full, (rest[0] if rest else None)


def sym_coef(C, plan, W, tiles, sc, lse2_all, cpos):
    """Kept cosines -> (cbuf: this rank's coefficient tiles, compact [row_tiles][plan.sym_c_ld]:
    column block r + d at column slots [d * rt, (d + 1) * rt) for d = 0 .. W/2, the only blocks a
    rank writes (5 of 8 at W = 8: 640 instead of 1024 MiB at B = 4096, d = 2048);
    mbuf: the partners' mirrored blocks [slots][row_tiles][row_tiles], slot = job order)."""
    rt = plan.row_tiles
    nslot = max(1, W // 2)  # partner slots (q - r - 1) mod W = 0 .. W/2 - 1
    cbuf = torch.empty((rt * plan.sym_c_ld * 65536,), dtype=sc.dtype, device=sc.device)
    mbuf = torch.empty((nslot * rt * rt * 65536,), dtype=sc.dtype, device=sc.device)
    C.coef_sym(sc, tiles, lse2_all, cpos, plan, cbuf, mbuf)
    return cbuf, mbuf


def contrib_dtype(plan) -> torch.dtype:
    """dtype of the partner gradient contributions on the wire: fp16 for the reduced-precision
    plans (half the xGMI bytes; the contributions are O(1) sums, fp16's 11-bit mantissa is
    finer than the bf16/fp16 gradient they end up in), fp32 for exact-fp32 plans."""
    return torch.float32 if plan.backward_dtype == "fp32" else torch.float16


def sym_partner_grad(C, plan, W, r, mbuf, zqt_all, job):
    """One partner's gradient contribution: rows = C_{q,r}[q's tiles k0..k1, my tiles m0..m1)
    Z_r[m0..m1), [(k1 - k0) * 256, dim_n] in :func:`contrib_dtype`, destined for q's rows
    k0*256... The job's mirror slot is (q - r - 1) mod W."""
    Rpad, rt = plan.rows_pad, plan.row_tiles
    q, m0, m1, k0, k1 = job
    slot = (q - r - 1) % W
    out = torch.empty((Rpad, plan.dim_n), dtype=contrib_dtype(plan), device=mbuf.device)
    C.dz_view(mbuf, slot * rt * rt + m0, rt, zqt_all, r, m0 * 256, m1 - m0, k0, k1, out, False, plan)
    return out[k0 * 256:k1 * 256]


def sym_partner_grads(C, plan, W, r, mbuf, zqt_all):
    """All partners' contributions {q: rows}. The full blocks (slots 0 .. nfull-1, partners
    r+1 .. r+nfull) are ONE GEMM: a tall A of nfull x row_tiles row panels against Z_r."""
    Rpad, rt = plan.rows_pad, plan.row_tiles
    jobs = sym_jobs(W, r, rt)
    full = [j for j in jobs if (j[1], j[2], j[3], j[4]) == (0, rt, 0, rt)]
    assert jobs[:len(full)] == full
    out = {}
    if full:
        buf = torch.empty((len(full) * Rpad, plan.dim_n), dtype=contrib_dtype(plan), device=mbuf.device)
        C.dz_view(mbuf, 0, rt, zqt_all, r, 0, rt, 0, len(full) * rt, buf, False, plan)
        out.update({q: buf[i * Rpad:(i + 1) * Rpad] for i, (q, *_) in enumerate(full)})
    for job in jobs[len(full):]:
        out[job[0]] = sym_partner_grad(C, plan, W, r, mbuf, zqt_all, job)
    return out


def sym_grad_slabs(plan, W, r, device):
    """(own, received, views): own = fp32 [1, Rpad, dim_n] for this rank's contributions;
    received = [incoming, Rpad, dim_n] in :func:`contrib_dtype`, slab i = what incoming job i
    (sym_incoming order) sends, rows outside its range zeroed; views = {sender: receive view}.
    The normalisation backward sums them all while reading."""
    inc = sym_incoming(W, r, plan.row_tiles)
    own = torch.empty((1, plan.rows_pad, plan.dim_n), dtype=torch.float32, device=device)
    recv = torch.empty((len(inc), plan.rows_pad, plan.dim_n), dtype=contrib_dtype(plan), device=device)
    views = {}
    for i, (p, m0, m1, k0, k1) in enumerate(inc):
        sl = recv[i]
        sl[:k0 * 256].zero_()
        sl[k1 * 256:].zero_()
        views[p] = sl[k0 * 256:k1 * 256]
    return own, recv, views


def sym_norm_bwd(C, plan, own, recv, h, inv, grad_out):
    if recv.dtype == torch.float32:  # exact-fp32 plans: one fp32 stack
        return C.norm_bwd_slabs(torch.cat([own, recv], 0), h, inv, grad_out.reshape(1), plan)
    return C.norm_bwd_slabs(own, h, inv, grad_out.reshape(1), plan, recv)


def sym_own_grad(C, plan, W, r, cbuf, zqt_all, out, reserve_cus=0):
    """This rank's own contributions into ``out`` [Rpad, dim_n]: C_{r,r} Z_r + the full blocks
    C_{r,q} Z_q (one GEMM over the consecutive rank blocks r..r+nfull, two if they wrap) + the
    split block's rows. The GEMMs leave ``reserve_cus`` CUs free for transfers in flight.
    ``cbuf`` is the compact layout of :func:`sym_coef` (block r + d at column slots d * rt...)."""
    rt, cld = plan.row_tiles, plan.sym_c_ld
    full, split = _split_jobs(sym_jobs(W, r, rt), rt)
    nb = 1 + len(full)  # blocks r, r+1, ..., r+nfull (mod W)
    first = min(nb, W - r)
    C.dz_view(cbuf, 0, cld, zqt_all, r, 0, first * rt, 0, rt, out, False, plan, reserve_cus=reserve_cus)
    if nb > first:
        C.dz_view(cbuf, first * rt, cld, zqt_all, 0, 0, (nb - first) * rt, 0, rt, out, True, plan,
                  reserve_cus=reserve_cus)
    if split is not None:
        q, m0, m1, k0, k1 = split
        C.dz_view(cbuf, ((q - r) % W) * rt + k0, cld, zqt_all, q, k0 * 256, k1 - k0, m0, m1, out, True, plan,
                  reserve_cus=reserve_cus)


def sym_backward_local(C, plan, W, r, h, inv, zqt_all, lse2_all, cpos, tiles, sc, grad_out, group):
    """Backward of one rank: the partners' contributions first (one stacked GEMM), sent in one
    grouped batch (concurrent over the peers' links) while this rank's own dZ GEMMs run;
    received contributions land in their own slabs, summed by the normalisation backward."""
    cbuf, mbuf = sym_coef(C, plan, W, tiles, sc, lse2_all, cpos)
    del sc
    contrib = sym_partner_grads(C, plan, W, r, mbuf, zqt_all)
    own, recv, views = sym_grad_slabs(plan, W, r, h.device)
    works = _p2p([(t, q) for q, t in contrib.items()], [(v, p) for p, v in views.items()], group)
    sym_own_grad(C, plan, W, r, cbuf, zqt_all, own[0], comm_reserve_cus(dist.get_backend(group)) if works else 0)
    with span("bwd_partner_grads"):
        for w in works:
            w.wait()
    del contrib, cbuf, mbuf
    return sym_norm_bwd(C, plan, own, recv, h, inv, grad_out)


def sym_ntxent_loss(h_local: torch.Tensor, temperature: float = 0.07, *, group=None, compute: str = "auto",
                    use_mixed_precision: bool = False) -> torch.Tensor:
    """Global NT-Xent over the group with each rank pair's similarity block computed once;
    same value and gradient as :func:`parallel.distributed.dist_ntxent_loss`."""
    W, _ = _world(group)
    if not h_local.is_cuda:
        return cpu_sym_ntxent_loss(h_local, temperature, group=group)
    comp = resolve_compute(h_local.dtype, use_mixed_precision, compute)
    if W == 1:
        from ..ops.ntxent import ntxent_loss

        return ntxent_loss(h_local, temperature, compute=comp)
    return SymNTXentFunction.apply(h_local, float(temperature), comp, group)


# ---------------------------------------------------------------------------------------
# CPU / gloo path: the same block assignment and exchanges with torch ops, at a configurable
# tile size (tests use small tiles so that the split pair and partial ranges are exercised).
# ---------------------------------------------------------------------------------------
class _CpuSymFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, temperature, group, tile):
        W, r = _world(group)
        R = h.shape[0]
        n = R // 2
        rt = -(-R // tile)
        Rp = rt * tile
        z, inv = reference.normalize(h)
        zp = torch.zeros((Rp, z.shape[1]), dtype=z.dtype)
        zp[:R] = z
        if W > 1:
            parts = [torch.empty_like(zp) for _ in range(W)]
            dist.all_gather(parts, zp, group=group)
        else:
            parts = [zp]
        valid = torch.arange(Rp) < R
        ninf = float("-inf")
        S_own = zp @ zp.t() / temperature
        S_own[~valid] = ninf
        S_own[:, ~valid] = ninf
        S_own.fill_diagonal_(ninf)
        lse_terms = [torch.logsumexp(S_own, 1)]
        jobs = sym_jobs(W, r, rt)
        inc = sym_incoming(W, r, rt)
        blocks = []
        col_sends = []
        for (q, m0, m1, k0, k1) in jobs:
            rows = slice(m0 * tile, m1 * tile)
            cols = slice(k0 * tile, k1 * tile)
            S = zp[rows] @ parts[q][cols].t() / temperature
            S[~valid[rows]] = ninf
            S[:, ~valid[cols]] = ninf
            blocks.append(S)
            t = torch.full((Rp,), ninf, dtype=S.dtype)
            t[rows] = torch.logsumexp(S, 1)
            lse_terms.append(t)
            col_sends.append((torch.logsumexp(S, 0), q))
        col_recvs = [(torch.empty(((k1 - k0) * tile,), dtype=z.dtype), p) for (p, m0, m1, k0, k1) in inc]
        _p2p(col_sends, col_recvs, group)
        for (buf, _), (p, m0, m1, k0, k1) in zip(col_recvs, inc):
            t = torch.full((Rp,), ninf, dtype=z.dtype)
            t[k0 * tile:k1 * tile] = buf
            lse_terms.append(t)
        lse = torch.logsumexp(torch.stack(lse_terms), 0)[:R]
        ar = torch.arange(R)
        pos = (ar + n) % R
        ypos = (z[ar] * z[pos]).sum(1) / temperature
        loss = (lse - ypos).sum() / (W * R)
        if W > 1:
            lparts = [torch.empty_like(lse) for _ in range(W)]
            dist.all_gather(lparts, lse.contiguous(), group=group)
            dist.all_reduce(loss, group=group)
        else:
            lparts = [lse]
        ctx.save_for_backward(z, inv)
        ctx.meta = (temperature, W, r, tile, group, parts, blocks, lparts, S_own)
        return loss

    @staticmethod
    def backward(ctx, g):
        z, inv = ctx.saved_tensors
        temperature, W, r, tile, group, parts, blocks, lparts, S_own = ctx.meta
        R = z.shape[0]
        n = R // 2
        rt = -(-R // tile)
        Rp = rt * tile

        def padl(l):
            out = torch.full((Rp,), float("inf"), dtype=l.dtype)  # exp(S - inf) = 0 on padding
            out[:R] = l
            return out

        lse_all = [padl(l) for l in lparts]
        lr = lse_all[r]
        Cown = torch.exp(S_own - lr[:, None]) + torch.exp(S_own - lr[None, :])
        ar = torch.arange(R)
        Cown[ar, (ar + n) % R] -= 2.0
        dz = Cown @ parts[r]
        jobs = sym_jobs(W, r, rt)
        inc = sym_incoming(W, r, rt)
        sends = []
        for (q, m0, m1, k0, k1), S in zip(jobs, blocks):
            rows = slice(m0 * tile, m1 * tile)
            cols = slice(k0 * tile, k1 * tile)
            Cb = torch.exp(S - lr[rows, None]) + torch.exp(S - lse_all[q][None, cols])
            dz[rows] += Cb @ parts[q][cols]
            sends.append((Cb.t() @ parts[r][rows], q))
        recvs = [(torch.empty(((k1 - k0) * tile, z.shape[1]), dtype=z.dtype), p) for (p, m0, m1, k0, k1) in inc]
        _p2p(sends, recvs, group)
        for (buf, _), (p, m0, m1, k0, k1) in zip(recvs, inc):
            dz[k0 * tile:k1 * tile] += buf
        dz = dz[:R] * (g / (W * R * temperature))
        dot = (z * dz).sum(1, keepdim=True)
        return inv.unsqueeze(1) * (dz - z * dot), None, None, None


def cpu_sym_ntxent_loss(h_local: torch.Tensor, temperature: float = 0.07, group=None, tile: int = 256) -> torch.Tensor:
    return _CpuSymFn.apply(h_local, float(temperature), group, int(tile))
