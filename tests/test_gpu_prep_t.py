"""The fused row prologue + Z^T pass (prep_t_kernel) against the separate prep and transpose
launches it replaces: zq, 1/|h|, the positive logits and Z^T must be bit-identical (the same
rounding of the same products in the same order; only the data movement differs).

Reference intent: the row normalisation and positive-pair logits of
/root/reference/src/ntxent_kernel.cu:160-200 (the dZ operand layout is this framework's own).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,dim,in_dtype,compute", [
    (8192, 2048, torch.bfloat16, "fp16"),   # headline
    (8192, 512, torch.bfloat16, "bf16"),    # config 2, bf16 rows
    (16384, 1024, torch.bfloat16, "fp16"),  # config 5
    (4096, 256, torch.float32, "fp16"),     # fp32 input, one chunk per lane (half the lanes idle)
    (512, 768, torch.float16, "fp16"),      # 16 blocks; d = 768: a partial third 256-column block
])
def test_prep_t_matches_prep_and_transpose(ext, rows, dim, in_dtype, compute):
    plan = ext.get_plan(rows, dim, 1, 0, 0.07, compute, 0)
    if not ext.prep_t_eligible(plan):
        pytest.skip("plan not eligible for the fused prologue")
    g = torch.Generator(device="cuda").manual_seed(rows + dim)
    h = torch.randn(rows, dim, device="cuda", generator=g).to(in_dtype)
    zq, inv, ypos, zqt = ext.prep_t(h, plan)
    zq_ref, inv_ref, ypos_ref, _ = ext.prep(h, plan)
    zqt_ref = ext.transpose(zq_ref, plan)
    torch.cuda.synchronize()
    d = dim
    assert torch.equal(zq[:, :d], zq_ref[:, :d])
    assert torch.equal(inv, inv_ref)
    assert torch.equal(ypos, ypos_ref)
    assert torch.equal(zqt[:d, :rows], zqt_ref[:d, :rows])
    # and Z^T really is the transpose of the normalised rows
    assert torch.equal(zqt[:d, :rows].t(), zq[:rows, :d])


def test_prep_t_eligibility(ext):
    """fused_forward and the Engine take the fused prologue whenever the plan is eligible: the
    headline and configs 2 / 5 are; config 4 (d = 8192), fp32 plans and padded row counts are not."""
    assert ext.prep_t_eligible(ext.get_plan(8192, 2048, 1, 0, 0.07, "fp16", 0))
    assert ext.prep_t_eligible(ext.get_plan(8192, 512, 1, 0, 0.07, "bf16", 0))
    assert not ext.prep_t_eligible(ext.get_plan(2048, 8192, 1, 0, 0.07, "fp16", 0))
    assert not ext.prep_t_eligible(ext.get_plan(8192, 2048, 1, 0, 0.07, "fp32", 0))
    assert not ext.prep_t_eligible(ext.get_plan(8000, 2048, 1, 0, 0.07, "fp16", 0))
