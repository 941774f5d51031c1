"""Forward similarity GEMM with operand streaming across work items (sim_gemm_kernel, MODE
kModeFwd: the trailing stages of one whole-tile item stage the next item's first two K-steps
and its epilogue runs with them in flight) vs the drained schedule (set_fwd_stream(False)).

Each tile's MFMA order is the same either way, so the LSE partials, the kept cosines, the loss
and the gradient must agree bitwise; shapes with >= 2 whole-tile rounds per block (2N >= 8192
rows: 528+ tiles on 256 CUs) exercise the hand-over, fp32 operands the 32-store epilogue.
"""
import pytest
import torch

from test_gpu_kernels import _inputs

pytestmark = pytest.mark.gpu


def _with_stream(C, on, fn):
    old = C.fwd_stream_enabled()
    C.set_fwd_stream(on)
    try:
        out = fn()
        torch.cuda.synchronize()
        return out
    finally:
        C.set_fwd_stream(old)


@pytest.mark.parametrize("rows,dim,compute", [
    (8192, 256, "fp16"),     # 2 whole-tile rounds per block
    (12288, 512, "bf16"),    # 4 rounds + remainder
    (8192, 128, "fp32"),     # f32 kept cosines: 32 epilogue stores per wave
    (8192, 2048, "fp16"),    # headline shape
])
def test_fwd_stream_stats_bitwise(ext, rows, dim, compute):
    C = ext
    assert C.fwd_stream_enabled(), "streaming is the default"
    _, h = _inputs(rows, dim, torch.float32 if compute == "fp32" else torch.bfloat16, seed=31)
    plan = C.get_plan(rows, dim, 1, 0, 0.07, compute, 0)
    assert not plan.small
    zq, inv, ypos, _ = C.prep(h, plan)

    def fwd():
        part, sc = C.fwd_stats(zq, zq, plan, True)
        return part.clone(), sc.clone()

    a = _with_stream(C, True, fwd)
    b = _with_stream(C, False, fwd)
    assert torch.equal(a[1], b[1]), "kept cosines differ"
    assert torch.equal(a[0], b[0]), "LSE partials differ"


@pytest.mark.parametrize("rows,dim,compute", [(8192, 512, "fp16"), (16384, 256, "bf16")])
def test_fwd_stream_loss_grad_bitwise(ext, rows, dim, compute):
    import ntxent_amd

    _, h = _inputs(rows, dim, torch.bfloat16, seed=37)

    def step():
        x = h.clone().requires_grad_(True)
        loss = ntxent_amd.ntxent_loss(x, 0.07, compute=compute)
        (g,) = torch.autograd.grad(loss, x)
        return loss.detach(), g

    la, ga = _with_stream(ext, True, step)
    lb, gb = _with_stream(ext, False, step)
    assert torch.equal(la, lb)
    assert torch.equal(ga, gb)


@pytest.mark.parametrize("rows,dim,compute", [(2048, 8192, "fp16"), (1024, 4096, "bf16"), (2048, 4096, "fp8"),
                                              (8192, 512, "fp16")])  # last: split-K dZ only
def test_splitk_piece_major_matches_tile_major(ext, rows, dim, compute):
    """Tile-starved forward and dZ (split-K + reduce launch): the piece-major aligned split against the
    tile-major straddling one (different K pieces, so equal to fp32 rounding) and the loss
    against the fp64 oracle."""
    import ntxent_amd
    from test_gpu_kernels import _oracle

    _, h = _inputs(rows, dim, torch.bfloat16, seed=41)
    old, old_half = ext.splitk_piece_major(), ext.splitk_half()
    ext.set_splitk_half(False)  # fp32 slabs both ways (the fp16 slabs: test_splitk_half_slabs)
    ext.set_splitk_dz_half(False)
    outs = {}
    try:
        for pm in (True, False):
            ext.set_splitk_piece_major(pm)
            x = h.clone().requires_grad_(True)
            loss = ntxent_amd.ntxent_loss(x, 0.07, compute=compute)
            (g,) = torch.autograd.grad(loss, x)
            torch.cuda.synchronize()
            outs[pm] = (loss.item(), g.float())
    finally:
        ext.set_splitk_piece_major(old)
        ext.set_splitk_half(old_half)
        ext.set_splitk_dz_half(False)
    (la, ga), (lb, gb) = outs[True], outs[False]
    assert abs(la - lb) <= 1e-5 * abs(lb)
    scale = gb.abs().max().item()
    assert (ga - gb).abs().max().item() <= 1e-2 * scale
    if compute != "fp8":
        lo, _ = _oracle(h, 0.07)
        assert abs(la - lo) <= 2e-4 * abs(lo)


@pytest.mark.parametrize("rows,dim,compute", [(2048, 8192, "fp16"), (1024, 4096, "bf16"), (2048, 8192, "fp32"),
                                              (2048, 4096, "fp8"), (8192, 512, "fp16"), (8192, 512, "bf16")])
def test_splitk_half_slabs(ext, rows, dim, compute):
    """Piece-major split-K forward and dZ with fp16 partial tiles (the default for 2-byte plans)
    against fp32 slabs: each piece is rounded once to fp16 before the fp32 sum, so the kept cosines
    and dZ move by a few fp16 ulps at most. fp32 and fp8 plans keep fp32 slabs (bitwise equal
    either way). 8192 x 512 splits only the dZ."""
    import ntxent_amd
    from test_gpu_kernels import _oracle

    assert ext.splitk_half() and not ext.splitk_dz_half(), "fp16 forward slabs are the default, dZ opt-in"
    _, h = _inputs(rows, dim, torch.float32 if compute == "fp32" else torch.bfloat16, seed=43)
    outs = {}
    try:
        for half in (True, False):
            ext.set_splitk_half(half)
            ext.set_splitk_dz_half(half)
            x = h.clone().requires_grad_(True)
            loss = ntxent_amd.ntxent_loss(x, 0.07, compute=compute)
            (g,) = torch.autograd.grad(loss, x)
            torch.cuda.synchronize()
            outs[half] = (loss.item(), g.float())
    finally:
        ext.set_splitk_half(True)
        ext.set_splitk_dz_half(False)
    (la, ga), (lb, gb) = outs[True], outs[False]
    if compute in ("fp32", "fp8"):
        assert la == lb and torch.equal(ga, gb), "fp32 / fp8 plans must not use fp16 slabs"
        return
    assert abs(la - lb) <= 1e-4 * abs(lb)
    assert (ga - gb).abs().max().item() <= 1e-2 * gb.abs().max().item()
    lo, go = _oracle(h, 0.07)
    assert abs(la - lo) <= 2e-4 * abs(lo)
    # the gradient error against the fp64 oracle stays within 25 % of the fp32-slab one
    ea = (ga.double().cpu() - go).abs().max().item()
    eb = (gb.double().cpu() - go).abs().max().item()
    assert ea <= 1.25 * eb + 1e-6, (ea, eb)


@pytest.mark.parametrize("rows,dim,compute,T", [
    (8192, 2048, "fp16", 0.07),   # headline: 16 diagonal tiles in the remainder
    (16384, 1024, "bf16", 0.07),  # config 5 shape: 32 diagonal tiles (2 blocks per CU)
    (8192, 1024, "fp32", 0.07),   # f32 kept cosines
    (8192, 1024, "fp16", 0.02),   # per-tile-max epilogue (no fixed shift)
])
def test_diag_upper_matches_full_subtiles(ext, rows, dim, compute, T):
    """The forward's diagonal remainder from the upper 64x64 regions only (diag_up_kernel; the
    coefficient pass mirrors the rest) against all 16 regions over the whole K (diag_sub_kernel):
    partials to fp32 rounding (the off-diagonal regions sum two K halves), loss and gradient."""
    import ntxent_amd

    _, h = _inputs(rows, dim, torch.float32 if compute == "fp32" else torch.bfloat16, seed=43)
    plan = ext.get_plan(rows, dim, 1, 0, T, compute, 0)
    zq, inv, ypos, _ = ext.prep(h, plan)
    old = ext.diag_upper_enabled()
    outs = {}
    try:
        for up in (True, False):
            ext.set_diag_upper(up)
            part, _ = ext.fwd_stats(zq, zq, plan, True)
            x = h.clone().requires_grad_(True)
            loss = ntxent_amd.ntxent_loss(x, T, compute=compute)
            (g,) = torch.autograd.grad(loss, x)
            torch.cuda.synchronize()
            outs[up] = (part.clone(), loss.item(), g.float())
    finally:
        ext.set_diag_upper(old)
    (pa, la, ga), (pb, lb, gb) = outs[True], outs[False]
    # (max, sum) partials: same max (fixed shift) / sums to fp32 rounding
    torch.testing.assert_close(pa, pb, rtol=2e-5, atol=0)
    assert abs(la - lb) <= 2e-6 * abs(lb)
    scale = gb.abs().max().item()
    assert (ga - gb).abs().max().item() <= 4e-3 * scale


@pytest.mark.parametrize("rows,dim,compute", [(8192, 2048, "fp16"), (16384, 1024, "bf16")])
def test_superblock_order_bitwise(ext, rows, dim, compute):
    """Own-block tiles in 8-panel superblocks (default) vs Z-order: every tile's work and every
    merge order (partials per column tile, coefficient tiles by slot) are independent of the list
    order, so loss and gradient agree bitwise (the order is part of the plan-cache key)."""
    import ntxent_amd

    _, h = _inputs(rows, dim, torch.bfloat16, seed=53)
    old = ext.superblock_order_enabled()
    outs = {}
    try:
        for sb in (True, False):
            ext.set_superblock_order(sb)
            x = h.clone().requires_grad_(True)
            loss = ntxent_amd.ntxent_loss(x, 0.07, compute=compute)
            (g,) = torch.autograd.grad(loss, x)
            torch.cuda.synchronize()
            outs[sb] = (loss.detach(), g)
    finally:
        ext.set_superblock_order(old)
    assert torch.equal(outs[True][0], outs[False][0])
    assert torch.equal(outs[True][1], outs[False][1])
