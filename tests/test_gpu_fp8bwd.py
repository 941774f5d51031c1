"""fp8 backward (FP8 plans): the coefficient matrix and Z^T enter the dZ GEMM as e4m3 (per-row
scale from the LSE pass's bound, Z^T scaled by 256) on the block-scaled MFMA, the positive term
added exactly in the dZ epilogue. Gradient error against the host fp64 oracle, next to the
fp8-forward / fp16-backward path of the same inputs (the error table in BASELINE.md comes from
these prints)."""
import pytest
import torch

from test_gpu_kernels import _inputs, _oracle

pytestmark = pytest.mark.gpu


def _grad(h, T, fp8_bwd):
    import ntxent_amd

    C = ntxent_amd.ops._ext.load()
    old = C.fp8_backward_enabled()
    C.set_fp8_backward(fp8_bwd)
    try:
        x = h.clone().requires_grad_(True)
        loss = ntxent_amd.ntxent_loss(x, T, compute="fp8", keep_logits=True)
        (g,) = torch.autograd.grad(loss, x)
        torch.cuda.synchronize()
        return loss.item(), g
    finally:
        C.set_fp8_backward(old)


@pytest.mark.parametrize("rows,dim,T", [
    (4096, 512, 0.07),
    (2048, 1024, 0.07),
    (3000, 256, 0.1),    # padded rows
    (4096, 256, 0.5),
])
def test_fp8_backward_error_vs_oracle(ext, rows, dim, T):
    _, h = _inputs(rows, dim, torch.bfloat16, seed=rows + dim)
    l8, g8 = _grad(h, T, True)
    l16, g16 = _grad(h, T, False)
    assert l8 == l16  # same forward
    lref, gref = _oracle(h, T)
    scale = gref.abs().max().item()
    e8 = (g8.double().cpu() - gref).abs().max().item() / scale
    e16 = (g16.double().cpu() - gref).abs().max().item() / scale
    # the backward's own quantisation error: same fp8 forward, e4m3 vs fp16 dZ operands
    eb = (g8.float() - g16.float()).abs().max().item() / g16.float().abs().max().item()
    print(f"FP8BWD rows={rows} dim={dim} T={T}: max|g - g64|/max|g64| fp8-bwd {e8:.3e}  fp16-bwd {e16:.3e}  "
          f"max|g8 - g16|/max|g16| {eb:.3e}")
    assert torch.isfinite(g8).all()
    assert not torch.equal(g8, g16)  # the e4m3 path ran
    # round 5: with the row scale taken from a bound on each row's largest negative (not the
    # fixed-shift M), the e4m3 operands cost less than the bf16 rounding of the gradient itself
    # (measured 5.3e-3 at rows=4096, d=512; 5.8e-3 at 16384 x 1024: one bf16 ulp of the largest
    # component); round 4's M-based scale gave 5e-2. Verdict r4 item 7: within 2x of the fp16
    # backward's error against the fp64 oracle.
    assert eb <= 1.6e-2, eb
    assert e8 <= 2 * e16 + 2e-3, (e8, e16)


def test_fp8_backward_is_default(ext):
    """FP8 plans take the e4m3 backward unless switched off (set_fp8_backward(False))."""
    assert ext.fp8_backward_enabled()
