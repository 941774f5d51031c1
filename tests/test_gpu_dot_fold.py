"""Dot reduce folded into the dZ GEMM (SimParams::dot_cnt, sim_gemm.h dz_dot_fold / dz_dot).

dot_i = z_i . g_i = sum_j C_ij cos_ij (the normalisation backward's radial term) is summed from
the coefficient pass's slot partials. Unfolded, a separate dot_reduce launch does it; folded, every
block of the dZ's persistent grid sums its share of the rows before its first item and publishes
them through a counter that the epilogues poll. Both use the same additions in the same order
(dot_slot_sum), so the gradient must be BITWISE the unfolded one, at every shape: the headline,
config 5 (16384 rows), config 4 (d = 8192), a padded row count (6000 rows: 192 dZ tiles on 256
CUs, stream-K items), and config 2 (d = 512: split-K dZ pieces fold for the reduce launch).
Repeated steps check that the counters clean themselves.
Reference intent: /root/reference/src/ntxent_kernel.cu:232-262 (the backward's gradient).
"""
import pytest
import torch

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _views(rows, dim, seed, dtype=torch.bfloat16):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = rows // 2
    base = torch.randn(n, dim, device="cuda", generator=g)
    v1 = base + 0.7 * torch.randn(n, dim, device="cuda", generator=g)
    v2 = base + 0.7 * torch.randn(n, dim, device="cuda", generator=g)
    return torch.cat([v1, v2], 0).to(dtype)


def _grad(h, T):
    import ntxent_amd

    x = h.clone().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, T)
    (g,) = torch.autograd.grad(loss, x)
    torch.cuda.synchronize()
    return loss.detach(), g


def _both(ext, fn):
    old = ext.dot_fold_enabled()
    try:
        ext.set_dot_fold(False)
        a = fn()
        ext.set_dot_fold(True)
        b = fn()
    finally:
        ext.set_dot_fold(old)
    return a, b


@pytest.mark.parametrize("rows,dim,dtype", [(8192, 2048, torch.bfloat16), (16384, 1024, torch.bfloat16),
                                            (2048, 8192, torch.bfloat16), (6000, 2048, torch.float16),
                                            (8192, 512, torch.bfloat16)])
def test_dot_fold_gradient_bitwise(ext, rows, dim, dtype):
    h = _views(rows, dim, seed=rows + dim, dtype=dtype)
    (l0, g0), (l1, g1) = _both(ext, lambda: _grad(h, 0.07))
    assert l0.item() == l1.item()
    assert torch.equal(g0, g1), f"max diff {(g0.float() - g1.float()).abs().max().item()}"


def test_dot_fold_repeated_steps_and_oracle(ext):
    # the counters return to zero at every kernel exit: later steps see a fresh count
    h = _views(8192, 2048, seed=11)
    old = ext.dot_fold_enabled()
    try:
        ext.set_dot_fold(True)
        outs = [_grad(h, 0.1)[1] for _ in range(4)]
    finally:
        ext.set_dot_fold(old)
    for g in outs[1:]:
        assert torch.equal(outs[0], g)
    x = h.double().requires_grad_(True)
    (gr,) = torch.autograd.grad(R.ntxent_loss(x, 0.1), x)
    scale = gr.abs().max().item()
    assert (outs[0].double() - gr).abs().max().item() <= 8e-3 * scale


def test_dot_fold_engine_bitwise(ext):
    # the native Engine's world-1 backward takes the same fold decision
    h = _views(8192, 2048, seed=5)

    def run():
        eng = ext.NativeEngine(8192, 2048, 0.07, "bf16", "auto")
        res = []
        for _ in range(2):
            loss, dh = eng.step(h)
            torch.cuda.synchronize()
            res.append((loss.item(), dh.clone()))
        del eng
        return res

    a, b = _both(ext, run)
    for (la, ga), (lb, gb) in zip(a, b):
        assert la == lb
        assert torch.equal(ga, gb)
    assert torch.equal(b[0][1], b[1][1])


@pytest.mark.parametrize("rows,dim", [(8192, 2048), (6000, 2048)])
def test_dot_fold_fallback_bitwise(ext, rows, dim):
    # every epilogue skips the poll and sums its rows' dot from the slots itself (the path a grid
    # whose blocks are not all resident would take): the same additions, the same bits
    h = _views(rows, dim, seed=rows + 3, dtype=torch.bfloat16)
    spin = ext.dot_fold_spin()
    try:
        ext.set_dot_fold_spin(0)
        (l0, g0), (l1, g1) = _both(ext, lambda: _grad(h, 0.07))
    finally:
        ext.set_dot_fold_spin(spin)
    assert l0.item() == l1.item()
    assert torch.equal(g0, g1), f"max diff {(g0.float() - g1.float()).abs().max().item()}"
