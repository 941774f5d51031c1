"""Half C: the coefficient pass writes only the upper coefficient tiles and the dZ GEMM stages a
lower K tile C_IJ (J < I) from C_JI through a transposing LDS image (SimParams::c_half,
sim_gemm.h read_a_tr). The mirrored C holds the same values as C_JI^T, bit for bit, and the dZ
accumulates in the same K order, so the gradient must be BITWISE the full-C gradient; and both
within the usual tolerance of an fp64 oracle. Shapes: the headline (32 row panels), config 4 (8
row panels, d = 8192), config 5 (64 row panels); config 2 (d = 512: split-K dZ) is not eligible
and must fall back to the full C. Reference intent: /root/reference/src/ntxent_kernel.cu:232-262
(the backward's gradient).
"""
import pytest
import torch

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _views(rows, dim, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = rows // 2
    base = torch.randn(n, dim, device="cuda", generator=g)
    v1 = base + 0.7 * torch.randn(n, dim, device="cuda", generator=g)
    v2 = base + 0.7 * torch.randn(n, dim, device="cuda", generator=g)
    return torch.cat([v1, v2], 0).to(torch.bfloat16)


def _grad(h, T, compute="auto"):
    import ntxent_amd

    x = h.clone().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, T, compute=compute)
    (g,) = torch.autograd.grad(loss, x)
    torch.cuda.synchronize()
    return loss.detach(), g


@pytest.mark.parametrize("rows,dim", [(8192, 2048), (2048, 8192), (16384, 1024), (8192, 512)])
def test_half_c_gradient_bitwise_equal_to_full_c(ext, rows, dim):
    h = _views(rows, dim, seed=rows + dim)
    old = ext.half_c_enabled()
    try:
        ext.set_half_c(False)
        l0, g0 = _grad(h, 0.07)
        ext.set_half_c(True)
        l1, g1 = _grad(h, 0.07)
    finally:
        ext.set_half_c(old)
    assert l0.item() == l1.item()
    assert torch.equal(g0, g1), f"max diff {(g0.float() - g1.float()).abs().max().item()}"


def test_half_c_gradient_vs_fp64_oracle(ext):
    h = _views(8192, 2048, seed=7)
    old = ext.half_c_enabled()
    try:
        ext.set_half_c(True)
        _, g = _grad(h, 0.1)
    finally:
        ext.set_half_c(old)
    x = h.double().requires_grad_(True)
    (gr,) = torch.autograd.grad(R.ntxent_loss(x, 0.1), x)
    scale = gr.abs().max().item()
    assert (g.double() - gr).abs().max().item() <= 8e-3 * scale


def test_half_c_engine_matches_full_c(ext):
    # the native Engine's world-1 backward takes the same half-C decision
    h = _views(8192, 2048, seed=3)
    old = ext.half_c_enabled()
    outs = []
    try:
        for on in (False, True):
            ext.set_half_c(on)
            eng = ext.NativeEngine(8192, 2048, 0.07, "bf16", "auto")
            loss, dh = eng.step(h)
            torch.cuda.synchronize()
            outs.append((loss.item(), dh.clone()))
            del eng
    finally:
        ext.set_half_c(old)
    assert outs[0][0] == outs[1][0]
    assert torch.equal(outs[0][1], outs[1][1])
