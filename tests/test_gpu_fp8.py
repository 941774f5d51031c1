"""fp8 (e4m3) forward path on gfx950 — BASELINE config 5.

The forward GEMM runs on the CDNA4 block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 with each
row quantised as e4m3(z * 2^e_i), e_i its amax-derived power of two (row amax -> [224, 448]),
and the E8M0 scales applied by the MFMA; the backward runs in fp16 on the forward's kept cosines. Exact reference: the fp64 NT-Xent of
the fp8-QUANTISED rows (torch.float8_e4m3fn, OCP, round-to-nearest-even) — tight parity.
Accuracy study: versus the unquantised loss at tau = 0.07 (documented tolerance).
"""
import math

import pytest
import torch

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _rows(rows, dim, seed, noise=0.3):
    g = torch.Generator().manual_seed(seed)
    n = rows // 2
    base = torch.randn(n, dim, generator=g, dtype=torch.float64)
    return torch.cat([base + noise * torch.randn(n, dim, generator=g, dtype=torch.float64),
                      base + noise * torch.randn(n, dim, generator=g, dtype=torch.float64)], 0)


def _quantised(h64):
    """Per-row amax scaling as prep does: e = floor(log2(448 / amax)) clamped to [0, 126]."""
    z = torch.nn.functional.normalize(h64.float(), dim=1).double()
    amax = z.abs().amax(1, keepdim=True).float()
    _, E = torch.frexp(448.0 / amax)  # 448 / amax = m * 2^E, m in [0.5, 1)
    sc = torch.ldexp(torch.ones_like(amax), (E - 1).clamp(0, 126)).double()
    return (z * sc).to(torch.float8_e4m3fn).double() / sc


@pytest.mark.parametrize("rows,dim", [(64, 128), (512, 256), (600, 200), (1024, 1024)])
def test_fp8_loss_matches_quantised_oracle(rows, dim):
    import ntxent_amd

    h64 = _rows(rows, dim, seed=rows + dim)
    x = h64.float().cuda()
    loss = ntxent_amd.ntxent_loss(x, 0.07, compute="fp8")
    q = _quantised(h64)
    # q rows are not exactly unit-norm: the GEMM sees q_i . q_j, as does this oracle
    S = q @ q.t() / 0.07
    S.fill_diagonal_(float("-inf"))
    pos = R.positive_index(rows)
    ref = torch.nn.functional.cross_entropy(S, pos).item()
    assert abs(loss.item() - ref) < 1e-4 * max(1.0, ref), (loss.item(), ref)


@pytest.mark.parametrize("T", [0.07, 0.5])
def test_fp8_accuracy_vs_exact(T):
    import ntxent_amd

    h64 = _rows(2048, 1024, seed=11)
    x = h64.float().cuda().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, T, compute="fp8")
    (g,) = torch.autograd.grad(loss, x)
    h = h64.clone().requires_grad_(True)
    lref = R.ntxent_loss(h, T)
    (gref,) = torch.autograd.grad(lref, h)
    assert math.isfinite(loss.item())
    assert abs(loss.item() - lref.item()) < 2e-2 * max(1.0, lref.item()), (loss.item(), lref.item())
    rel = ((g.double().cpu() - gref).norm() / gref.norm()).item()
    assert rel < 0.1, rel


def test_fp8_emulated_ranks():
    from ntxent_amd.parallel.emulate import emulated_dist_forward_backward

    shards = [_rows(256, 128, seed=40 + r) for r in range(2)]
    loss, grads = emulated_dist_forward_backward([s.float().cuda() for s in shards], 0.1, compute="fp8")
    qs = [_quantised(s) for s in shards]
    q = R.global_pair_order(qs)
    S = q @ q.t() / 0.1
    S.fill_diagonal_(float("-inf"))
    ref = torch.nn.functional.cross_entropy(S, R.positive_index(q.shape[0])).item()
    assert abs(loss.item() - ref) < 1e-4 * max(1.0, ref), (loss.item(), ref)
    assert all(torch.isfinite(g).all() for g in grads)


@pytest.mark.parametrize("W", [2, 3])
def test_fp8_emulated_symmetric_ranks(W):
    """Symmetric data-parallel mode with the fp8 forward: same quantised-oracle loss as the
    all-gather mode, and the same gradients up to the fp16 backward's rounding."""
    from ntxent_amd.parallel.emulate import emulated_dist_forward_backward, emulated_sym_forward_backward

    shards = [_rows(300, 128, seed=50 + r) for r in range(W)]
    dev = [s.float().cuda() for s in shards]
    loss, grads = emulated_sym_forward_backward(dev, 0.1, compute="fp8")
    qs = [_quantised(s) for s in shards]
    q = R.global_pair_order(qs)
    S = q @ q.t() / 0.1
    S.fill_diagonal_(float("-inf"))
    ref = torch.nn.functional.cross_entropy(S, R.positive_index(q.shape[0])).item()
    assert abs(loss.item() - ref) < 1e-4 * max(1.0, ref), (loss.item(), ref)
    l2, g2 = emulated_dist_forward_backward(dev, 0.1, compute="fp8")
    for a, b in zip(grads, g2):
        rel = ((a.double() - b.double()).norm() / b.double().norm()).item()
        assert rel < 2e-3, rel
