"""Raw-operand forward (RawRows): the forward GEMM reads the input rows h themselves (bf16 input
-> bf16 MFMA operands, exact; fp16 -> fp16) and normalises in its epilogue, the LSE launch writes
Z^T = (h inv)^T, and the row prologue only computes inv and the positive logits.

Pinned against the fp64 oracle at the shapes that select each forward schedule (whole rounds +
diagonal remainder, two blocks per CU, split-K), against the unit-row (zq) forward of the same
plan, for determinism, and for the second backward (retain_graph), which rebuilds the unit rows
the raw forward never wrote. Reference intent: /root/reference/src/ntxent_kernel.cu:160-200
(forward GEMM + row kernels), tests/test_forward.cpp (batch sweep).
"""
import math

import pytest
import torch

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _views(rows, dim, seed, dtype=torch.bfloat16, noise=0.5, scale=1.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = rows // 2
    base = torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    v1 = base + noise * torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    v2 = base + noise * torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    return (scale * torch.cat([v1, v2], 0)).to(dtype)


def _run(ext, h, T, compute, raw):
    import ntxent_amd

    old = ext.raw_forward_enabled()
    ext.set_raw_forward(raw)
    try:
        x = h.clone().requires_grad_(True)
        loss = ntxent_amd.ntxent_loss(x, T, compute=compute)
        (g,) = torch.autograd.grad(loss, x)
        torch.cuda.synchronize()
        return loss.detach(), g
    finally:
        ext.set_raw_forward(old)


def _oracle(h, T):
    x = h.detach().double().requires_grad_(True)
    loss = R.ntxent_loss(x, T)
    (g,) = torch.autograd.grad(loss, x)
    return loss.item(), g


@pytest.mark.parametrize("rows,dim,dtype,compute", [
    (8192, 2048, torch.bfloat16, "fp16"),   # headline: 2 rounds + 16 diagonal tiles, bf16 operands / fp16 cosines
    (16384, 1024, torch.bfloat16, "fp16"),  # config 5 shape: diagonal remainder at two blocks per CU
    (2048, 8192, torch.bfloat16, "fp16"),   # config 4: split-K forward (fp16 slabs of normalised pieces)
    (8192, 512, torch.float16, "fp16"),     # fp16 rows: fp16 operands
    (4096, 1024, torch.bfloat16, "bf16"),   # bf16 plan: bf16 operands and cosines
])
def test_raw_forward_matches_fp64_and_zq_path(ext, rows, dim, dtype, compute):
    h = _views(rows, dim, 71, dtype)
    plan = ext.get_plan(rows, dim, 1, 0, 0.07, compute, 0)
    assert not plan.small
    out = ext.fused_forward(h, 0.07, compute, True)
    assert out[1].numel() == 0, "the raw-operand forward did not run"
    la, ga = _run(ext, h, 0.07, compute, True)
    lb, gb = _run(ext, h, 0.07, compute, True)
    assert torch.equal(la, lb) and torch.equal(ga, gb), "raw forward is not deterministic"
    lz, gz = _run(ext, h, 0.07, compute, False)
    lref, gref = _oracle(h, 0.07)
    scale = gref.abs().max().item()
    e_raw = (ga.double() - gref).abs().max().item() / scale
    e_zq = (gz.double() - gref).abs().max().item() / scale
    l_raw = abs(la.item() - lref) / max(1.0, abs(lref))
    l_zq = abs(lz.item() - lref) / max(1.0, abs(lref))
    print(f"RAWFWD rows={rows} dim={dim} {dtype} {compute}: loss err raw {l_raw:.2e} zq {l_zq:.2e}; "
          f"grad err raw {e_raw:.2e} zq {e_zq:.2e}")
    lt, gt = (2e-5, 2e-2) if compute == "bf16" else (2e-6, 1e-2)
    assert math.isfinite(la.item()) and l_raw <= lt, (la.item(), lref)
    assert e_raw <= gt, e_raw
    # exact inputs: the raw forward is no less accurate than normalising into fp16 first
    assert l_raw <= 2 * l_zq + 1e-7


@pytest.mark.parametrize("scale", [1e-4, 1e3])
def test_raw_forward_input_scale(ext, scale):
    """Rows far from unit norm: the raw accumulators carry |h|^2 (fp32), the epilogue divides it
    out; the loss is scale-invariant (the reference's stability grid scales the inputs too,
    /root/reference/python/test.py:57-79)."""
    h = _views(4096, 512, 73, scale=scale)
    l1, g1 = _run(ext, h, 0.07, "fp16", True)
    lref, gref = _oracle(h, 0.07)
    assert abs(l1.item() - lref) <= 2e-6 * max(1.0, abs(lref))
    assert (g1.double() - gref).abs().max().item() <= 1e-2 * gref.abs().max().item()


def test_raw_forward_second_backward(ext):
    """retain_graph: the second backward has no kept cosines and recomputes S from unit rows,
    which the raw forward never wrote (the backward rebuilds them)."""
    import ntxent_amd

    h = _views(8192, 256, 79)
    x = h.clone().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, 0.07)
    (g1,) = torch.autograd.grad(loss, x, retain_graph=True)
    (g2,) = torch.autograd.grad(loss, x)
    torch.cuda.synchronize()
    assert (g1.float() - g2.float()).abs().max().item() <= 2e-2 * g1.float().abs().max().item()
