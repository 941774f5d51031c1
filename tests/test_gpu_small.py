"""Small-problem path (kernels/small_kernels.hip) vs the fp64 oracle and vs the large-problem
pipeline, on an MI355X.

The reference benchmarks B in {32..1024} x D in {64,128,256} (src/benchmark.cpp:68-71) and
runs its stability grid at B=128, D=256 (python/test.py:57-79); those shapes now take one
forward and one backward launch after the row prologue.
"""
import math

import pytest
import torch

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu

# measured on MI355X (round 2): loss |err| <= ~3e-4 (fp16) / 2e-3 (bf16) relative; gradient
# max-abs error <= ~4e-3 (fp16) / 2e-2 (bf16) of max |grad|; tolerances are 2-3x that
TOL = {"fp16": (1e-3, 1e-2), "bf16": (6e-3, 4e-2)}


def _inputs(rows, dim, dtype, seed=0, noise=0.3):
    g = torch.Generator().manual_seed(seed)
    n = rows // 2
    base = torch.randn(n, dim, generator=g, dtype=torch.float64)
    h64 = torch.cat([base + noise * torch.randn(n, dim, generator=g, dtype=torch.float64),
                     base + noise * torch.randn(n, dim, generator=g, dtype=torch.float64)], 0)
    return h64.to(dtype).cuda()


def _run(h, T, compute, go=1.0):
    import ntxent_amd

    x = h.clone().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, T, compute=compute)
    (g,) = torch.autograd.grad(loss, x, torch.tensor(go, device=loss.device, dtype=loss.dtype))
    torch.cuda.synchronize()
    return loss.item(), g


def _oracle(h, T, go=1.0):
    x = h.detach().double().cpu().requires_grad_(True)
    loss = R.ntxent_loss(x, T)
    (g,) = torch.autograd.grad(loss, x, torch.tensor(go, dtype=torch.float64))
    return loss.item(), g


@pytest.fixture
def small_on(ext):
    ext.set_small_path(True)
    ext.set_small_splits(0)
    ext.set_small_fuse_rows(-1)
    yield ext
    ext.set_small_path(True)
    ext.set_small_splits(0)
    ext.set_small_fuse_rows(-1)


@pytest.mark.parametrize("fuse", [True, False])
@pytest.mark.parametrize("compute", ["fp16", "bf16"])
@pytest.mark.parametrize("in_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,dim", [(64, 128), (34, 100), (128, 256), (600, 200), (1024, 64), (2048, 256),
                                      (2048, 128), (66, 192)])
def test_small_path_matches_oracle(small_on, rows, dim, in_dtype, compute, fuse):
    """fuse: the forward normalises the rows itself (one launch) or runs after launch_prep."""
    small_on.set_small_fuse_rows(1 << 20 if fuse else 0)
    plan = small_on.get_plan(rows, dim, 1, 0, 0.07, compute, 0)
    assert plan.small and small_on.small_fwd_fused(plan) == fuse
    h = _inputs(rows, dim, in_dtype, seed=rows * 3 + dim)
    l, g = _run(h, 0.07, compute, go=0.7)
    lr, gr = _oracle(h, 0.07, go=0.7)
    lt, gt = TOL[compute]
    assert math.isfinite(l) and abs(l - lr) <= lt * max(1.0, abs(lr)), (l, lr)
    err = (g.double().cpu() - gr).abs().max().item() / gr.abs().max().item()
    assert err <= gt, err


@pytest.mark.parametrize("splits", [1, 2, 3, 8])
def test_small_backward_column_splits_agree(small_on, splits):
    h = _inputs(1024, 128, torch.float32, seed=5)  # fp32 dh: no output rounding flips
    small_on.set_small_splits(1)
    _, g1 = _run(h, 0.1, "fp16")
    small_on.set_small_splits(splits)
    _, gs = _run(h, 0.1, "fp16")
    err = (gs - g1).abs().max().item() / g1.abs().max().item()
    assert err <= 1e-5, err


def test_small_vs_large_pipeline(small_on):
    h = _inputs(512, 256, torch.bfloat16, seed=9)
    ls, gs = _run(h, 0.07, "fp16")
    small_on.set_small_path(False)
    ll, gl = _run(h, 0.07, "fp16")
    assert abs(ls - ll) <= 1e-3 * abs(ll)
    err = (gs.float() - gl.float()).abs().max().item() / gl.float().abs().max().item()
    assert err <= 1.5e-2, err


def test_small_path_deterministic(small_on):
    h = _inputs(1536, 192, torch.bfloat16, seed=11)
    l1, g1 = _run(h, 0.07, "fp16")
    l2, g2 = _run(h, 0.07, "fp16")
    assert l1 == l2 and torch.equal(g1, g2)


@pytest.mark.parametrize("scale", [1e-5, 1.0, 1e5])
@pytest.mark.parametrize("T", [0.01, 0.07, 1.0])
def test_small_path_stability_grid(small_on, scale, T):
    # python/test.py:57-79 grid (B=128, D=256), value-checked
    g = torch.Generator().manual_seed(0)
    z = torch.nn.functional.normalize(torch.randn(256, 256, generator=g, dtype=torch.float64), dim=1) * scale
    h = z.float().cuda()
    l, grad = _run(h, T, "fp16")
    lr, gr = _oracle(h, T)
    assert math.isfinite(l) and torch.isfinite(grad).all()
    assert abs(l - lr) <= 2e-2 * max(1.0, abs(lr)), (l, lr)
    err = (grad.double().cpu() - gr).abs().max().item() / max(gr.abs().max().item(), 1e-30)
    assert err <= 6e-2, err


@pytest.mark.parametrize("in_dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("rows,dim", [(256, 256), (130, 72), (1000, 128)])
def test_small_fused_prologue_vs_prep(small_on, rows, dim, in_dtype):
    """The one-launch forward (rows normalised in the kernel, positive logit taken from the MFMA
    tile holding the pair) against the forward after launch_prep: same rounded rows, so the loss
    agrees to accumulation order and the gradients (same backward) to output rounding (fp16 dh at
    this scale is subnormal: one ulp is 2^-24)."""
    h = _inputs(rows, dim, in_dtype, seed=rows + dim)
    small_on.set_small_fuse_rows(1 << 20)
    lf, gf = _run(h, 0.07, "fp16")
    small_on.set_small_fuse_rows(0)
    lp, gp = _run(h, 0.07, "fp16")
    assert abs(lf - lp) <= 1e-5 * abs(lp), (lf, lp)
    diff = (gf.float() - gp.float()).abs().max().item()
    assert diff <= max(2e-3 * gp.float().abs().max().item(), 2 * 2.0 ** -24), diff
