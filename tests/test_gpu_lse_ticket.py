"""LSE launch's loss sum as one 64-bit fixed-point ticket per block (lse_block, lse_loss_fx) and the
Z^T side job of the diagonal remainder (DiagSideZt).

The fixed-point sum must stay within fp32 rounding of the fp64 oracle at temperatures that move
its scale (F from log(2N) + 2/tau + 1 per row), be bitwise repeatable, and still turn a
non-finite input into a NaN loss (the ticket's non-finite count). The side-job Z^T is pinned by the
gradient of the paths that read it, against the LSE-launch transpose of the unit-row forward.
Reference intent: /root/reference/src/ntxent_kernel.cu:202-215 (compute_loss).
"""
import pytest
import torch

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _views(rows, dim, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = rows // 2
    base = torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    v1 = base + 0.5 * torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    v2 = base + 0.5 * torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    return torch.cat([v1, v2], 0).to(torch.bfloat16)


@pytest.mark.parametrize("rows,dim,T", [(4096, 512, 0.07), (8192, 256, 0.02), (4096, 256, 1.0)])
def test_ticket_loss_matches_fp64_and_repeats(ext, rows, dim, T):
    import ntxent_amd

    h = _views(rows, dim, seed=rows + dim)
    a = ntxent_amd.ntxent_loss(h, T).item()
    b = ntxent_amd.ntxent_loss(h, T).item()
    ref = R.ntxent_loss(h.double(), T).item()
    assert a == b
    assert abs(a - ref) <= 2e-6 * abs(ref) + 1e-7


@pytest.mark.parametrize("bad", [float("nan"), float("inf")])
def test_nonfinite_input_gives_nan_loss(ext, bad):
    import ntxent_amd

    h = _views(4096, 512, seed=3)
    h[7, 3] = bad
    loss = ntxent_amd.ntxent_loss(h, 0.07)
    assert torch.isnan(loss).item()


def test_side_job_zt_gradient_matches_unit_row_path(ext):
    # 8192 rows x d 2048: 16 diagonal remainder tiles on one block per CU -> Z^T from the side job;
    # the unit-row forward transposes in the LSE launch instead
    import ntxent_amd

    h = _views(8192, 2048, seed=11)
    grads = []
    old = ext.raw_forward_enabled()
    try:
        for raw in (True, False):
            ext.set_raw_forward(raw)
            x = h.clone().requires_grad_(True)
            loss = ntxent_amd.ntxent_loss(x, 0.07, compute="fp16")
            (g,) = torch.autograd.grad(loss, x)
            grads.append(g.float())
    finally:
        ext.set_raw_forward(old)
    scale = grads[1].abs().max().item()
    assert (grads[0] - grads[1]).abs().max().item() <= 1e-2 * scale


def _low_loss_views(rows, dim, rank, noise, seed):
    # views of points on a rank-`rank` subspace: positives nearly identical, the nearest negatives
    # close enough that tau = 0.01 leaves a small but nonzero loss (~0.04 at rank 8, noise 0.1)
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = rows // 2
    basis = torch.randn(rank, dim, device="cuda", generator=g, dtype=torch.float64)
    base = torch.randn(n, rank, device="cuda", generator=g, dtype=torch.float64) @ basis / rank**0.5
    v1 = base + noise * torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    v2 = base + noise * torch.randn(n, dim, device="cuda", generator=g, dtype=torch.float64)
    return torch.cat([v1, v2], 0).to(torch.bfloat16)


@pytest.mark.parametrize("rows,dim", [(16384, 128), (16384, 512)])
def test_ticket_loss_low_loss_low_tau(ext, rows, dim):
    # the regime where the fixed-point quantum (sized from the worst-case bound log 2N + 2/tau + 1
    # per row) is largest relative to the sum: tau = 0.01, strongly correlated views, loss < 0.05
    import ntxent_amd

    h = _low_loss_views(rows, dim, rank=8, noise=0.1, seed=rows + dim)
    ref = R.ntxent_loss(h.double(), 0.01).item()
    assert 1e-4 < ref < 0.05, ref
    a = ntxent_amd.ntxent_loss(h, 0.01).item()
    assert a == ntxent_amd.ntxent_loss(h, 0.01).item()
    assert abs(a - ref) <= 1e-6 * abs(ref), (a, ref, abs(a - ref) / ref)


@pytest.mark.parametrize("rows,dim", [(8192, 2048), (2048, 8192)])
@pytest.mark.parametrize("raw", [True, False])
def test_zt_exact_against_unit_rows(ext, raw, rows, dim):
    # Z^T (the dZ GEMM's B operand) element-wise: the raw-operand forward's side job (DiagSideZt,
    # beside the diagonal remainder at 8192 x 2048) or the LSE launch's raw transpose (split-K
    # forward at 2048 x 8192) writes fp16((h * inv)^T) from the returned inv; the unit-row
    # forward's LSE-launch transpose writes zq^T. Exact, padded rows/columns zero.
    h = _views(rows, dim, seed=5)
    old = ext.raw_forward_enabled()
    try:
        ext.set_raw_forward(raw)
        out = ext.fused_forward(h, 0.07, "fp16", True)
    finally:
        ext.set_raw_forward(old)
    zq, zqt, inv = out[1], out[2], out[3]
    rows, dim = h.shape
    assert zqt.dtype == torch.float16 and zqt.shape[0] >= dim and zqt.shape[1] >= rows
    if raw:
        assert zq.numel() == 0  # nothing reads unit rows on the raw path
        want = (h.float() * inv[:, None]).to(torch.float16).t()
    else:
        want = zq[:rows, :dim].t()
    got = zqt[:dim, :rows]
    bad = (got != want).sum().item()
    assert bad == 0, f"{bad} mismatching Z^T elements, max diff {(got.float() - want.float()).abs().max().item()}"
    assert (zqt[dim:] == 0).all().item()
