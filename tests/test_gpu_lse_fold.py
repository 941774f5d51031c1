"""The LSE launch folded into the diagonal remainder's launch (LseFold, sim_gemm.h
lse_fold_group): when the remainder is exactly the diagonal tiles of the second half of the rows
(the headline and config 2: 16 of 32 panels), each completed 64-row group's block merges its 64
positive pairs and adds its loss to the LSE launch's fixed-point ticket, and no LSE launch runs.
Pinned against the unfolded path (same value up to the merge order and the per-block partial
sums) and against the fp64 oracle; shapes where the fold does not apply must be unaffected.
Reference intent: /root/reference/src/ntxent_kernel.cu:202-215 (compute_loss).
"""
import pytest
import torch

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _views(rows, dim, seed, noise=0.7):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = rows // 2
    base = torch.randn(n, dim, device="cuda", generator=g)
    v1 = base + noise * torch.randn(n, dim, device="cuda", generator=g)
    v2 = base + noise * torch.randn(n, dim, device="cuda", generator=g)
    return torch.cat([v1, v2], 0).to(torch.bfloat16)


def _run(ext, h, T, fold):
    old = ext.lse_fold_enabled()
    try:
        ext.set_lse_fold(fold)
        out = ext.fused_forward(h, T, "fp16", True)
        torch.cuda.synchronize()
    finally:
        ext.set_lse_fold(old)
    return out[0].item(), out[4].clone(), out[6].clone()


@pytest.mark.parametrize("rows,dim,T", [(8192, 2048, 0.07), (8192, 512, 0.07), (8192, 2048, 0.02),
                                        (16384, 1024, 0.07), (6144, 256, 0.07)])
def test_folded_lse_matches_lse_launch(ext, rows, dim, T):
    h = _views(rows, dim, seed=rows + dim)
    l0, lse0, c0 = _run(ext, h, T, False)
    l1, lse1, c1 = _run(ext, h, T, True)
    ref = R.ntxent_loss(h.double(), T).item()
    assert abs(l1 - l0) <= 1e-6 * abs(l0) + 1e-7, (l0, l1)
    assert abs(l1 - ref) <= 2e-6 * abs(ref) + 1e-7, (l1, ref)
    R2 = rows
    assert (lse1[:R2] - lse0[:R2]).abs().max().item() <= 2e-5
    assert (c1[:R2] - c0[:R2]).abs().max().item() <= 1e-5


def test_folded_lse_repeatable_and_gradient(ext):
    import ntxent_amd

    h = _views(8192, 2048, seed=9)
    old = ext.lse_fold_enabled()
    try:
        ext.set_lse_fold(True)
        a = ntxent_amd.ntxent_loss(h, 0.1).item()
        b = ntxent_amd.ntxent_loss(h, 0.1).item()
        x = h.clone().requires_grad_(True)
        (g,) = torch.autograd.grad(ntxent_amd.ntxent_loss(x, 0.1), x)
    finally:
        ext.set_lse_fold(old)
    assert a == b
    xd = h.double().requires_grad_(True)
    (gr,) = torch.autograd.grad(R.ntxent_loss(xd, 0.1), xd)
    assert (g.double() - gr).abs().max().item() <= 8e-3 * gr.abs().max().item()


def test_folded_lse_nonfinite_gives_nan(ext):
    import ntxent_amd

    h = _views(8192, 2048, seed=4)
    h[5000, 3] = float("nan")  # a second-half row: its pair's group carries the non-finite count
    old = ext.lse_fold_enabled()
    try:
        ext.set_lse_fold(True)
        loss = ntxent_amd.ntxent_loss(h, 0.07)
    finally:
        ext.set_lse_fold(old)
    assert torch.isnan(loss).item()


def test_engine_fold_matches(ext):
    h = _views(8192, 2048, seed=13)
    old = ext.lse_fold_enabled()
    outs = []
    try:
        for on in (False, True):
            ext.set_lse_fold(on)
            eng = ext.NativeEngine(8192, 2048, 0.07, "bf16", "auto")
            loss, dh = eng.step(h)
            torch.cuda.synchronize()
            outs.append((loss.item(), dh.float().clone()))
            del eng
    finally:
        ext.set_lse_fold(old)
    assert abs(outs[0][0] - outs[1][0]) <= 1e-6 * abs(outs[0][0])
    assert (outs[0][1] - outs[1][1]).abs().max().item() <= 1e-2 * outs[0][1].abs().max().item()
