"""SimCLR training steps on the MI355X (bf16 autocast encoder, HIP NT-Xent loss)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_simclr_trainer_gpu_steps(tmp_path):
    import ntxent_amd.models as M

    cfg = M.TrainConfig(steps=4, batch=64, width=16, proj_hidden=256, proj_out=128, log_every=0, warmup_steps=1,
                        ckpt_dir=str(tmp_path), ckpt_every=2)
    t = M.SimCLRTrainer(cfg)
    hist = t.fit()
    assert len(hist) == 4 and all(math.isfinite(r["loss"]) for r in hist)
    assert (tmp_path / "ckpt_4.pt").exists()
    assert t.mem is not None and t.mem.records


def test_loss_used_by_trainer_is_the_hip_op():
    import ntxent_amd

    z = torch.randn(128, 128, device="cuda", requires_grad=True)
    loss = ntxent_amd.NTXentLoss(0.5)(z)
    assert loss.grad_fn is not None and "NTXentFunction" in type(loss.grad_fn).__name__
