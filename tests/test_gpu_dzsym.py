"""dZ GEMM on the upper-triangular coefficient matrix and Zq itself (launch_dz_sym) vs the
round-2 backward (mirrored coefficient tiles + ZqT transpose + launch_dz) and vs the fp64
oracle, on the large-problem pipeline (shapes past the one-launch small path).

The mirrored K-steps (column tiles below the own diagonal) are read as transposes of the stored
upper tiles, so every shape here exercises both the direct and the transposed operand paths.
"""
import pytest
import torch

from test_gpu_kernels import TOL, _inputs, _oracle

pytestmark = pytest.mark.gpu


def _run(h, T, compute, keep, sym):
    import ntxent_amd

    C = ntxent_amd.ops._ext.load()
    old = C.dz_sym_enabled()
    C.set_dz_sym(sym)
    try:
        x = h.clone().requires_grad_(True)
        loss = ntxent_amd.ntxent_loss(x, T, compute=compute, keep_logits=keep)
        (g,) = torch.autograd.grad(loss, x)
        torch.cuda.synchronize()
        return loss.item(), g
    finally:
        C.set_dz_sym(old)


@pytest.mark.parametrize("rows,dim,compute,keep", [
    (4096, 512, "fp16", True),     # 16 row tiles: 120 mirrored (tile, K-tile) pairs
    (3000, 256, "bf16", True),     # padded rows (Rpad 3072), bf16 operands
    (2048, 1024, "fp16", False),   # recompute flow (coefficient GEMM) + split-K dZ pieces
    (2560, 512, "fp8", True),      # fp8 forward, fp16 backward
])
def test_dz_sym_matches_transpose_path_and_oracle(ext, rows, dim, compute, keep):
    plan = ext.get_plan(rows, dim, 1, 0, 0.1, "fp16" if compute == "fp8" else compute, 0)
    assert plan.dz_sym and not plan.small
    _, h = _inputs(rows, dim, torch.float32, seed=rows + dim)
    l1, g1 = _run(h, 0.1, compute, keep, True)
    l0, g0 = _run(h, 0.1, compute, keep, False)
    assert l1 == l0  # the forward is unchanged (the LSE launch just skips the transpose)
    scale = g0.abs().max().item()
    diff = (g1 - g0).abs().max().item()
    print(f"DZSYM rows={rows} dim={dim} compute={compute} keep={keep} max|g_sym - g_old|/max|g|={diff / scale:.3e} "
          f"bitwise={torch.equal(g1, g0)}")
    # same coefficients, same K order: at most output rounding apart
    assert diff <= 1e-3 * scale
    if compute != "fp8":
        lref, gref = _oracle(h, 0.1)
        err = (g1.double().cpu() - gref).abs().max().item()
        assert err <= TOL[compute][1] * gref.abs().max().item(), err


def test_dz_sym_native_raw_backward(ext):
    """The reference-API backward (coefficient GEMM, no kept cosines) takes the same path."""
    _, h = _inputs(4096, 256, torch.float32, seed=11)
    go = torch.tensor(1.0, device=h.device)
    C = ext
    old = C.dz_sym_enabled()
    try:
        C.set_dz_sym(True)
        g1, _ = C.backward(h, torch.empty(0, device=h.device), go, 0.07, True)
        C.set_dz_sym(False)
        g0, _ = C.backward(h, torch.empty(0, device=h.device), go, 0.07, True)
    finally:
        C.set_dz_sym(old)
    scale = g0.abs().max().item()
    assert (g1 - g0).abs().max().item() <= 1e-3 * scale


@pytest.mark.parametrize("rows,dim,compute,keep,sym", [
    (4096, 512, "fp16", True, True),
    (3000, 256, "bf16", True, True),     # padded rows: the fused epilogue's row guard
    (2048, 1024, "fp16", False, True),   # coefficient-GEMM flow (dot partials in the recompute epilogue)
    (2560, 512, "fp16", True, False),    # launch_dz path (no dz_sym) with the fused epilogue
    (2560, 512, "fp8", True, False),     # fp8 plans: never fused (bitwise the unfused result)
    (4096, 520, "bf16", True, True),     # d % 256 != 0: partial last column tile
    (8192, 1024, "fp16", True, True),    # enough dZ tiles for whole-tile rounds (epilogue, not split-K reduce)
])
def test_norm_fuse_matches_unfused(ext, rows, dim, compute, keep, sym):
    """The normalisation backward fused into the dZ epilogue (dot_i from the coefficient pass)
    against the separate norm_bwd launch, and against the oracle."""
    C = ext
    old = C.norm_fuse_enabled()
    _, h = _inputs(rows, dim, torch.float32, seed=rows + 7 * dim)
    hb = h.to(torch.bfloat16) if compute == "bf16" else h
    try:
        C.set_norm_fuse(True)
        l1, g1 = _run(hb, 0.1, compute, keep, sym)
        C.set_norm_fuse(False)
        l0, g0 = _run(hb, 0.1, compute, keep, sym)
    finally:
        C.set_norm_fuse(old)
    assert l1 == l0
    g1, g0 = g1.float(), g0.float()
    scale = g0.abs().max().item()
    diff = (g1 - g0).abs().max().item()
    print(f"NORMFUSE rows={rows} dim={dim} compute={compute} keep={keep} sym={sym} rel diff={diff / scale:.3e}")
    if compute == "fp8":
        assert torch.equal(g1, g0)
    assert diff <= (1e-2 if compute == "bf16" else 2e-3) * scale
    if compute != "fp8" and rows * rows * dim <= 2 ** 34:  # (host fp64 oracle)
        lref, gref = _oracle(hb.float(), 0.1)
        err = (g1.double().cpu() - gref).abs().max().item()
        assert err <= TOL[compute][1] * gref.abs().max().item(), err
