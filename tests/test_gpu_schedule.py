"""The similarity-GEMM schedules at the shapes that select them, against a GPU fp64 oracle.

Each schedule of launch_fwd_stats / launch_dz is the only one compiled for its shapes (the
A/B alternatives of earlier rounds are deleted), so these tests pin each against the fp64
oracle of the same loss, plus determinism (bitwise-equal repeated runs):

* operand streaming across whole-tile items (>= 2 rounds per block: 2N >= 8192 rows), fp16 /
  bf16 / fp32 kept cosines (fp32: the 32-store epilogue);
* the diagonal remainder after the whole rounds (diag_up_kernel): the headline's 16 tiles at one
  block per CU, config 5's 32 tiles at two, fp32 cosines, and the per-tile-max epilogue (T = 0.02);
* piece-major split-K forward (fp16 partial tiles for 2-byte plans, fp32 for fp32 / fp8) and
  split-K dZ (fp32 slabs) for tile-starved shapes.

Kept cosines are also checked against a torch fp32 GEMM of the same normalised rows.
Reference intent: the GEMM + row kernels of /root/reference/src/ntxent_kernel.cu:160-200 and the
backward SGEMM :228-236, at the sizes the benchmark runs.
"""
import math

import pytest
import torch

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _views(rows, dim, seed, dtype=torch.bfloat16, noise=0.5):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = rows // 2
    base = torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    v1 = base + noise * torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    v2 = base + noise * torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    return torch.cat([v1, v2], 0).to(dtype)


def _oracle(h, T):
    x = h.detach().double().requires_grad_(True)
    loss = R.ntxent_loss(x, T)
    (g,) = torch.autograd.grad(loss, x)
    return loss.item(), g


def _run(h, T, compute):
    import ntxent_amd

    x = h.clone().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, T, compute=compute)
    (g,) = torch.autograd.grad(loss, x)
    torch.cuda.synchronize()
    return loss.detach(), g


# loss rel err, grad max-abs err / max |grad| (fp8: the e4m3 forward's own quantisation error)
# (bf16: measured 8.5e-6 / 7.9e-3 at 16384 x 1024 and 12288 x 512, profiles/r4/gpu_tests.log)
TOL = {"fp16": (2e-6, 1e-2), "bf16": (2e-5, 2e-2), "fp32": (1e-7, 2e-5), "fp8": (5e-2, 2.5e-1)}


def _check(h, T, compute, tol=None):
    lt, gt = tol or TOL[compute]
    la, ga = _run(h, T, compute)
    lb, gb = _run(h, T, compute)
    assert torch.equal(la, lb) and torch.equal(ga, gb), "schedule is not deterministic"
    lref, gref = _oracle(h, T)
    l = la.item()
    assert math.isfinite(l) and torch.isfinite(ga).all()
    lerr = abs(l - lref) / max(1.0, abs(lref))
    gerr = (ga.double() - gref).abs().max().item() / gref.abs().max().item()
    print(f"SCHED rows={h.shape[0]} dim={h.shape[1]} compute={compute} T={T} loss_err={lerr:.2e} grad_err={gerr:.2e}")
    assert lerr <= lt, (l, lref)
    assert gerr <= gt, gerr


@pytest.mark.parametrize("rows,dim,compute", [
    (8192, 256, "fp16"),     # 2 whole-tile rounds per block, streamed hand-over
    (12288, 512, "bf16"),    # 4 rounds + remainder
    (8192, 128, "fp32"),     # f32 kept cosines: 32 epilogue stores per wave
])
def test_streamed_forward_matches_fp64(ext, rows, dim, compute):
    h = _views(rows, dim, 31, torch.float32 if compute == "fp32" else torch.bfloat16)
    plan = ext.get_plan(rows, dim, 1, 0, 0.07, compute, 0)
    assert not plan.small
    _check(h, 0.07, compute)


@pytest.mark.parametrize("rows,dim,compute", [(8192, 256, "fp16"), (8192, 128, "fp32")])
def test_kept_cosines_match_torch_gemm(ext, rows, dim, compute):
    """Kept cosine tiles (canonical fragment order) of every forward tile, diagonal remainder
    included, against torch's fp32 GEMM of the same normalised rows."""
    h = _views(rows, dim, 33, torch.float32 if compute == "fp32" else torch.bfloat16)
    plan = ext.get_plan(rows, dim, 1, 0, 0.07, compute, 0)
    zq, inv, ypos, _ = ext.prep(h, plan)
    part, sc = ext.fwd_stats(zq, zq, plan, True)
    torch.cuda.synchronize()
    z = zq[:, :dim].float()
    S = z @ z.t()
    tiles = plan.fwd_tiles.cpu().tolist()
    sc = sc.view(len(tiles), 256, 256)
    tol = 2e-3 if compute != "fp32" else 1e-5
    for k in (0, len(tiles) // 2, len(tiles) - 1):  # first, middle, last (a diagonal tile)
        ti, tj = tiles[k][0], tiles[k][1]
        ref = S[ti * 256:(ti + 1) * 256, tj * 256:(tj + 1) * 256]
        got = _unfragment(sc[k].float(), compute)
        if tiles[k][2] == 1:  # diagonal tile: only the upper 64x64 regions are kept
            for a in range(4):
                for b in range(a, 4):
                    r = slice(64 * a, 64 * a + 64)
                    c = slice(64 * b, 64 * b + 64)
                    assert (got[r, c] - ref[r, c]).abs().max().item() <= tol
        else:
            assert (got - ref).abs().max().item() <= tol


def _unfragment(t, compute):
    """Canonical fragment order -> row-major 256 x 256 (sim_gemm.h sc_unit / fp32 layout)."""
    lane = torch.arange(64, device=t.device)
    out = torch.empty(256, 256, device=t.device)
    flat = t.reshape(-1)
    for rb in range(0, 256, 16):
        for cb in range(0, 256, 16):
            rows = rb + 4 * (lane >> 4)
            cols = cb + (lane & 15)
            if compute == "fp32":
                base = (((rb >> 4) * 16 + (cb >> 4)) * 64 + lane) * 4
                off = 0
            else:
                base = (((rb >> 4) * 8 + (cb >> 5)) * 64 + lane) * 8
                off = 4 if (cb & 16) else 0
            for r in range(4):
                out[rows + r, cols] = flat[base + off + r]
    return out


@pytest.mark.parametrize("rows,dim,compute,T", [
    (8192, 2048, "fp16", 0.07),   # headline: 2 rounds + 16 diagonal tiles (one block per CU)
    (16384, 1024, "bf16", 0.07),  # config 5 shape: 32 diagonal tiles (two blocks per CU)
    (8192, 1024, "fp32", 0.07),   # f32 kept cosines
    (8192, 1024, "fp16", 0.02),   # per-tile-max epilogue (no fixed shift)
])
def test_diagonal_remainder_matches_fp64(ext, rows, dim, compute, T):
    # T = 0.02 on noisy views (positive cosine ~0.1): an O(1) loss; at noise 0.5 it would saturate at
    # ~1e-14, below the fp16 coefficient range
    h = _views(rows, dim, 43, torch.float32 if compute == "fp32" else torch.bfloat16, 3.0 if T < 0.05 else 0.5)
    plan = ext.get_plan(rows, dim, 1, 0, T, compute, 0)
    n_main = plan.n_fwd_tiles - plan.n_fwd_tiles % 256
    assert 0 < plan.n_fwd_tiles - n_main <= plan.row_tiles, "shape must leave a diagonal remainder"
    tol = TOL[compute] if T >= 0.05 or compute == "fp32" else (2e-6, 6e-2)  # kept fp16 cosines at 1/T = 50
    _check(h, T, compute, tol)


def test_large_diagonal_remainder_runs_diag_up(ext):
    """A remainder of 48 diagonal tiles (2N = 24576: 4656 own tiles = 18 rounds + 48 on 256 CUs)
    runs as diag_up regions: round 4 sized the ticket region for at most 36 remainder tiles and
    sent larger ones to the stream-K third round; the counter region now holds 14
    tickets per CU."""
    rows, dim = 24576, 256  # >= 4 K-steps per tile (the remainder path's minimum)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rt = rows // 256
    n_own = rt * (rt + 1) // 2
    nk = dim * 2 // 128
    rem = n_own % cus
    assert ext.fwd_diag_remainder(n_own, nk, cus, rt) == rem
    if cus == 256:
        assert rem == 48
    plan = ext.get_plan(rows, dim, 1, 0, 0.07, "fp16", 0)
    assert plan.n_fwd_tiles == n_own and not plan.small
    h = _views(rows, dim, 53)
    _check(h, 0.07, "fp16")


@pytest.mark.parametrize("rows,dim,compute", [
    (2048, 8192, "fp16"),   # config 4: split-K forward (fp16 slabs) + split-K dZ
    (1024, 4096, "bf16"),
    (2048, 8192, "fp32"),   # fp32 slabs
    (2048, 4096, "fp8"),    # fp8 forward: fp32 slabs
    (8192, 512, "fp16"),    # config 2: split-K dZ only
])
def test_splitk_matches_fp64(ext, rows, dim, compute):
    nk = (dim * (1 if compute == "fp8" else (4 if compute == "fp32" else 2))) // 128
    n_own = (rows // 256) * (rows // 256 + 1) // 2
    if rows < 8192:
        assert ext.fwd_splitk_pieces(n_own, nk, 256, rows // 256) > 0
    h = _views(rows, dim, 47, torch.float32 if compute == "fp32" else torch.bfloat16)
    _check(h, 0.07, compute)
