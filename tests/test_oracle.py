"""CPU tests of the pure-PyTorch NT-Xent oracle.

The oracle is what every HIP kernel test compares against, so it is pinned here first:
fp64 gradcheck, the closed-form symmetric backward vs autograd, closed-form values, the
reference's stability grid (python/test.py:57-79) and the sharded (data-parallel) math.
"""
import math

import pytest
import torch

from ntxent_amd.ops import reference as ref


def _emb(rows, dim, seed=0, dtype=torch.float64, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(rows, dim, generator=g, dtype=torch.float64) * scale).to(dtype)


@pytest.mark.parametrize("rows,dim", [(4, 3), (8, 16), (16, 5), (32, 128)])
@pytest.mark.parametrize("T", [0.07, 0.5])
def test_gradcheck_fp64(rows, dim, T):
    h = _emb(rows, dim, seed=rows * dim).requires_grad_(True)
    assert torch.autograd.gradcheck(lambda x: ref.ntxent_loss(x, T), (h,), eps=1e-6, atol=1e-5)


@pytest.mark.parametrize("rows,dim", [(4, 3), (10, 7), (64, 128)])
@pytest.mark.parametrize("T", [0.01, 0.07, 1.0])
@pytest.mark.parametrize("grad_out", [1.0, 0.37, -2.0])
def test_analytic_backward_matches_autograd(rows, dim, T, grad_out):
    h = _emb(rows, dim, seed=7).requires_grad_(True)
    loss = ref.ntxent_loss(h, T)
    (g_auto,) = torch.autograd.grad(loss, h, torch.tensor(grad_out, dtype=h.dtype))
    g_an = ref.ntxent_backward_analytic(h.detach(), T, grad_out)
    torch.testing.assert_close(g_an, g_auto, rtol=1e-9, atol=1e-12)


def test_closed_form_orthogonal_views():
    # 2N orthonormal rows: every off-diagonal logit is 0 -> loss = log(2N - 1).
    rows = 8
    h = torch.eye(rows, dtype=torch.float64)
    assert math.isclose(ref.ntxent_loss(h, 0.5).item(), ref.expected_random_loss(rows), rel_tol=1e-12)


def test_closed_form_identical_views():
    # views identical and mutually orthogonal pairs: positive logit 1/T, negatives 0.
    n, T = 4, 0.25
    v = torch.eye(n, dtype=torch.float64)
    h = torch.cat([v, v], 0)
    R = 2 * n
    expect = math.log(math.exp(1 / T) + (R - 2)) - 1 / T
    assert math.isclose(ref.ntxent_loss(h, T).item(), expect, rel_tol=1e-12)


def test_pair_api_and_stats():
    z1, z2 = _emb(6, 9, 1), _emb(6, 9, 2)
    h = torch.cat([z1, z2])
    a = ref.ntxent_loss_pair(z1, z2, 0.1)
    loss, lse, pl = ref.ntxent_stats(h, 0.1)
    torch.testing.assert_close(a, loss)
    torch.testing.assert_close((lse - pl).mean(), a)
    assert lse.shape == (12,) and pl.shape == (12,)


def test_scale_invariance():
    h = _emb(16, 32, 3)
    torch.testing.assert_close(ref.ntxent_loss(h, 0.07), ref.ntxent_loss(h * 1e3, 0.07))


@pytest.mark.parametrize("scale", [1e-5, 1.0, 1e5])
@pytest.mark.parametrize("T", [0.01, 0.07, 1.0])
def test_stability_grid_fp32(scale, T):
    # python/test.py:57-79 grid (B=128, D=256), fp32, loss and grads finite.
    h = _emb(256, 256, 5, dtype=torch.float32, scale=scale).requires_grad_(True)
    loss = ref.ntxent_loss(h, T)
    loss.backward()
    assert torch.isfinite(loss) and torch.isfinite(h.grad).all()


def test_zero_rows_are_finite():
    h = _emb(8, 4, 9)
    h[1] = 0
    h[6] = 0
    g = ref.ntxent_backward_analytic(h, 0.07)
    assert torch.isfinite(ref.ntxent_loss(h, 0.07)) and torch.isfinite(g).all()
    # below the eps clamp z = h / eps, so a zero row gets dz / eps (as F.normalize does)
    hh = h.clone().requires_grad_(True)
    (g_auto,) = torch.autograd.grad(ref.ntxent_loss(hh, 0.07), hh)
    torch.testing.assert_close(g, g_auto, rtol=1e-9, atol=1e-6)


def test_input_validation():
    with pytest.raises(ValueError):
        ref.ntxent_loss(torch.randn(5, 3))
    with pytest.raises(ValueError):
        ref.ntxent_loss(torch.randn(4))


def test_reference_as_written_differs():
    # The reference's as-written forward (self-diagonal target, scrambled GEMM) is not NT-Xent;
    # documented so nobody "fixes" parity towards it.
    z = torch.nn.functional.normalize(_emb(8, 16, 11), dim=1)
    written = ref.reference_as_written_forward(z, 0.07)
    correct = ref.ntxent_loss(torch.cat([z, z]), 0.07)
    assert torch.isfinite(written) and not torch.isclose(written, correct)


@pytest.mark.parametrize("W", [1, 2, 4])
@pytest.mark.parametrize("n,dim", [(2, 3), (8, 16), (5, 33)])
def test_sharded_math_equals_unsharded(W, n, dim):
    shards = [_emb(2 * n, dim, seed=100 + r) for r in range(W)]
    loss, grads = ref.sharded_forward_backward(shards, 0.2, grad_out=0.8)
    hg = ref.global_pair_order(shards).requires_grad_(True)
    l_ref = ref.ntxent_loss(hg, 0.2)
    (g_ref,) = torch.autograd.grad(l_ref, hg, torch.tensor(0.8, dtype=hg.dtype))
    torch.testing.assert_close(loss, l_ref, rtol=1e-10, atol=1e-12)
    # map per-rank rows back to the global [view1; view2] order
    N = W * n
    for r, g in enumerate(grads):
        torch.testing.assert_close(g[:n], g_ref[r * n:(r + 1) * n], rtol=1e-9, atol=1e-12)
        torch.testing.assert_close(g[n:], g_ref[N + r * n:N + (r + 1) * n], rtol=1e-9, atol=1e-12)


def test_flops_model():
    # B=4096 per view, d=2048, 1 GPU: upper-triangular fwd (half of 2*R^2*d) + full dZ GEMM.
    R, d = 8192, 2048
    f = ref.flops_fwd_bwd(R, R, d)
    assert f == pytest.approx(R * R * d * 2.0 * 1.5)
    assert ref.flops_fwd_bwd(R, 8 * R, d) > 8 * f / 1.5 * 0.9
