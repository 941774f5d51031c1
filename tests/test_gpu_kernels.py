"""HIP kernel numerics vs the PyTorch fp64 oracle (run on an MI355X).

Covers the intents of the reference's GTest/pytest suites (tests/test_forward.cpp,
tests/test_backward.cpp, python/test.py) with value checks they never had.
"""
import math

import pytest
import torch

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu

# (loss rtol, grad max-abs err relative to max |grad|): 2x the largest errors measured over the
# shapes below on MI355X (profiles/r2/parity_kernels.log: fp32 8.5e-10 / 2.8e-6, fp16 6.0e-7 /
# 3.9e-3, bf16 3.1e-7 / 1.1e-2; the kernels are deterministic, so box-to-box these do not move)
TOL = {
    "fp32": (2e-9, 6e-6),
    "fp16": (1.2e-6, 8e-3),
    "bf16": (7e-7, 2.2e-2),
}


def _inputs(rows, dim, dtype, seed=0, noise=0.3):
    g = torch.Generator().manual_seed(seed)
    n = rows // 2
    base = torch.randn(n, dim, generator=g, dtype=torch.float64)
    v1 = base + noise * torch.randn(n, dim, generator=g, dtype=torch.float64)
    v2 = base + noise * torch.randn(n, dim, generator=g, dtype=torch.float64)
    h64 = torch.cat([v1, v2], 0)
    return h64, h64.to(dtype).cuda()


def _oracle(h_dev, T):
    h = h_dev.detach().double().cpu().requires_grad_(True)
    loss = R.ntxent_loss(h, T)
    (g,) = torch.autograd.grad(loss, h)
    return loss.item(), g


def _check(h_dev, T, compute, keep=True):
    import ntxent_amd

    x = h_dev.clone().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, T, compute=compute, keep_logits=keep)
    (g,) = torch.autograd.grad(loss, x)
    lref, gref = _oracle(h_dev, T)
    lt, gt = TOL[compute]
    assert math.isfinite(loss.item())
    assert abs(loss.item() - lref) <= lt * max(1.0, abs(lref)), (loss.item(), lref)
    err = (g.double().cpu() - gref).abs().max().item()
    scale = gref.abs().max().item()
    print(f"PARITY rows={h_dev.shape[0]} dim={h_dev.shape[1]} in={h_dev.dtype} compute={compute} T={T} "
          f"loss_rel_err={abs(loss.item() - lref) / max(1.0, abs(lref)):.3e} grad_rel_err={err / scale:.3e}")
    assert err <= gt * scale, (err, scale)
    return loss.item(), lref, err / scale


@pytest.mark.parametrize("compute", ["fp32", "fp16", "bf16"])
@pytest.mark.parametrize("rows,dim", [(64, 128), (34, 100), (512, 256), (600, 200), (1024, 512)])
def test_fwd_bwd_matches_oracle(ext, rows, dim, compute):
    _, h = _inputs(rows, dim, torch.float32, seed=rows + dim)
    _check(h, 0.07, compute)


@pytest.mark.parametrize("in_dtype", [torch.bfloat16, torch.float16])
def test_low_precision_inputs(ext, in_dtype):
    _, h = _inputs(768, 384, in_dtype, seed=7)
    _check(h, 0.1, "fp16")


@pytest.mark.parametrize("rows,dim", [(512, 256), (1030, 96)])
def test_recompute_equals_store(ext, rows, dim):
    import ntxent_amd

    _, h = _inputs(rows, dim, torch.float32, seed=3)
    out = []
    for keep in (True, False):
        x = h.clone().requires_grad_(True)
        loss = ntxent_amd.ntxent_loss(x, 0.07, compute="fp16", keep_logits=keep)
        (g,) = torch.autograd.grad(loss, x)
        out.append((loss.item(), g))
    assert out[0][0] == out[1][0]
    assert torch.allclose(out[0][1], out[1][1], rtol=1e-2, atol=1e-6 * out[0][1].abs().max().item() + 1e-9)


def test_grad_out_scaling(ext):
    import ntxent_amd

    _, h = _inputs(256, 64, torch.float32, seed=5)
    x = h.clone().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, 0.5, compute="fp32")
    (3.5 * loss).backward()
    _, gref = _oracle(h, 0.5)
    assert torch.allclose(x.grad.double().cpu(), 3.5 * gref, rtol=1e-3, atol=1e-7)


@pytest.mark.parametrize("scale", [1e-5, 1.0, 1e5])
@pytest.mark.parametrize("T", [0.01, 0.07, 1.0])
def test_numerical_stability_grid(ext, scale, T):
    """The reference harness's stability grid (python/test.py:57-79) with value checks."""
    import ntxent_amd

    g = torch.Generator().manual_seed(11)
    z = torch.nn.functional.normalize(torch.randn(256, 256, generator=g), dim=1) * scale
    x = z.cuda().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, T, compute="fp32")
    (gr,) = torch.autograd.grad(loss, x)
    assert torch.isfinite(loss) and torch.isfinite(gr).all()
    lref, gref = _oracle(z.cuda(), T)
    assert abs(loss.item() - lref) <= 1e-4 * max(1.0, abs(lref))
    assert (gr.double().cpu() - gref).abs().max() <= 1e-3 * gref.abs().max() + 1e-12


def test_zero_rows_are_finite(ext):
    import ntxent_amd

    _, h = _inputs(128, 64, torch.float32)
    h[3] = 0
    x = h.clone().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, 0.07, compute="fp32")
    (g,) = torch.autograd.grad(loss, x)
    assert torch.isfinite(loss) and torch.isfinite(g).all()


def test_deterministic(ext):
    import ntxent_amd

    _, h = _inputs(1024, 256, torch.bfloat16, seed=9)
    res = []
    for _ in range(3):
        x = h.clone().requires_grad_(True)
        loss = ntxent_amd.ntxent_loss(x, 0.07)
        (g,) = torch.autograd.grad(loss, x)
        res.append((loss.item(), g))
    for l, g in res[1:]:
        assert l == res[0][0]
        assert torch.equal(g, res[0][1])


def test_reference_api_forward_backward(ext):
    """forward / forward_with_stats / backward with the reference's names and kwargs."""
    _, h = _inputs(64, 128, torch.float32, seed=1)
    loss = ext.forward(h, 0.07)
    loss2, lse = ext.forward_with_stats(h, 0.07, use_mixed_precision=False)
    lref, lse_ref, _ = R.ntxent_stats(h.double().cpu(), 0.07)
    assert abs(loss.item() - lref.item()) < 1e-4
    assert torch.allclose(lse.double().cpu(), lse_ref, atol=1e-4)
    go = torch.tensor(1.0, device=h.device)
    gz, glog = ext.backward(h, lse, go, 0.07, want_grad_logits=True)
    gref = R.ntxent_backward_analytic(h.double().cpu(), 0.07)
    # with the caller's fp32 LSE the positive coefficient a_i = 1 - P_ip inherits the LSE's
    # rounding (~1e-6 absolute); these views are nearly saturated (P_ip -> 1, |grad| ~ 3e-6), so
    # the stats path is held to that absolute level, the recomputing path to 1e-4 relative
    assert (gz.double().cpu() - gref).abs().max() < 5e-3 * gref.abs().max() + 1e-9
    assert glog.shape == (64, 64)
    gz2, glog2 = torch.ops.ntxent_cuda.backward(h, torch.empty(64, 64, device=h.device), go, 0.07)
    assert (gz2.double().cpu() - gref).abs().max() < 1e-4 * gref.abs().max() + 1e-9
    assert glog2.numel() == 0  # grad_logits only on request
    assert torch.ops.ntxent_cuda.forward(h, 0.07).item() == pytest.approx(loss.item(), rel=1e-6)
    assert ext.check_tensor_core_support() is True


@pytest.mark.parametrize("rows,dim,mp", [(600, 200, False), (2048, 512, True)])
def test_raw_backward_with_stats_skips_forward(ext, rows, dim, mp):
    """backward(z, lse_from_forward_with_stats, ...) runs ONE similarity GEMM (coefficients from
    the given LSE) and matches the stateless path that recomputes the statistics."""
    _, h = _inputs(rows, dim, torch.float32, seed=rows)
    _, lse = ext.forward_with_stats(h, 0.1, use_mixed_precision=mp)
    go = torch.tensor(0.5, device=h.device)
    g1, _ = ext.backward(h, lse, go, 0.1, use_mixed_precision=mp)
    g2, _ = ext.backward(h, torch.empty(0, device=h.device), go, 0.1, use_mixed_precision=mp)
    scale = g2.abs().max().item()
    assert (g1 - g2).abs().max().item() <= (1e-5 if not mp else 2e-3) * scale
    gref = 0.5 * R.ntxent_backward_analytic(h.double().cpu(), 0.1)
    assert (g1.double().cpu() - gref).abs().max().item() <= (2e-4 if not mp else 2e-2) * gref.abs().max().item()


def test_raw_backward_ignores_stale_stats(ext):
    """An LSE is trusted only for the z tensor, T and precision forward_with_stats returned it
    for: after an in-place update of z, or at another temperature, the backward recomputes the
    statistics and matches the stateless path (stale stats gave silent errors)."""
    _, h = _inputs(600, 200, torch.float32, seed=3)
    _, lse = ext.forward_with_stats(h, 0.1)
    go = torch.tensor(1.0, device=h.device)
    # other temperature: ignored
    g1, _ = ext.backward(h, lse, go, 0.2)
    g2, _ = ext.backward(h, torch.empty(0, device=h.device), go, 0.2)
    assert torch.equal(g1, g2)
    # z changed in place after the forward: ignored
    h.mul_(1.5).add_(0.25)
    g3, _ = ext.backward(h, lse, go, 0.1)
    g4, _ = ext.backward(h, torch.empty(0, device=h.device), go, 0.1)
    assert torch.equal(g3, g4)
    # a copy of the LSE (not the returned tensor) is not trusted either
    _, lse2 = ext.forward_with_stats(h, 0.1)
    g5, _ = ext.backward(h, lse2.clone(), go, 0.1)
    assert torch.equal(g5, g4)


@pytest.mark.parametrize("B", [16, 32, 64, 128])
def test_different_batch_sizes(ext, B):
    """tests/test_forward.cpp:41-51 DifferentBatchSizes, with an oracle value check."""
    _, h = _inputs(2 * B, 128, torch.float32, seed=B)
    _check(h, 0.07, "fp32")


@pytest.mark.parametrize("keep", [True, False])
def test_peak_memory_accounting(ext, keep):
    """Peak memory = the design's buffers, no hidden quadratic fp32 allocations.

    Quadratic state is only the fp16 coefficient matrix C (2 B per logit) plus, in store mode,
    the upper-triangular fp16 cosine tiles; everything else is O(R*d) or O(#CUs) (stream-K
    scratch). The reference allocates three fp32 (2N)^2 buffers per step (logits, softmax,
    grad_logits: src/ntxent_kernel.cu:155-158,218), i.e. 12 B per logit.
    """
    import ntxent_amd

    rows, dim = 8192, 256
    _, h = _inputs(rows, dim, torch.bfloat16, seed=2)
    plan = ext.get_plan(rows, dim, 1, 0, 0.07, "fp16", 0)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    x = h.clone().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, 0.07, keep_logits=keep)
    (g,) = torch.autograd.grad(loss, x)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    Rp, tile = plan.rows_pad, 256 * 256
    quad = plan.row_tiles * plan.col_tiles * tile * 2 + (plan.n_fwd_tiles * tile * 2 if keep else 0)
    linear = Rp * plan.ld_k * 2 + plan.dim_n * plan.ld_t * 2 + Rp * plan.dim_n * 4 + plan.col_tiles * Rp * 8
    scratch = ext.gemm_workspace_bytes(max(plan.n_fwd_tiles, plan.n_dz_tiles), 256)
    expected = quad + linear + scratch + 2 * rows * dim * 2
    assert peak <= 1.1 * expected, (peak, expected)
    assert peak < 0.5 * 3 * rows * rows * 4, peak  # under half the reference's quadratic fp32 buffers


def test_torch_cuda_graph_capture_replay():
    """The autograd op (forward + backward, side-stream transpose included) captures into a
    torch.cuda.CUDAGraph (hipGraph) and replays bit-identically: what small batches need, where
    ~8 kernel launches per step dominate."""
    import ntxent_amd

    _, h = _inputs(512, 256, torch.bfloat16, seed=3)
    x = h.clone().requires_grad_(True)
    # warm up outside the capture: plans, tile lists and scratch are created on first use
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            loss = ntxent_amd.ntxent_loss(x, 0.07)
            (g,) = torch.autograd.grad(loss, x)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        loss_g = ntxent_amd.ntxent_loss(x, 0.07)
        (g_g,) = torch.autograd.grad(loss_g, x)
    eager_loss = ntxent_amd.ntxent_loss(x, 0.07)
    (eager_g,) = torch.autograd.grad(eager_loss, x)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    assert loss_g.item() == eager_loss.item()
    assert torch.equal(g_g, eager_g)
