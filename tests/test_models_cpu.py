"""SimCLR model family, augmentations, LARS, trainer and checkpoint/resume on CPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ntxent_amd.models as M
from ntxent_amd.utils import GPUMemoryTracker, load_checkpoint, save_checkpoint, summarize, time_fn


def _cfg(**kw):
    base = dict(steps=6, batch=8, encoder="mlp", image_size=8, proj_hidden=32, proj_out=16, log_every=0,
                amp=False, warmup_steps=2, num_classes=4, optimizer="lars")
    base.update(kw)
    return M.TrainConfig(**base)


def test_simclr_shapes():
    m = M.SimCLR(M.resnet18(width=8), proj_hidden=64, proj_out=16)
    x1, x2 = torch.rand(3, 3, 16, 16), torch.rand(3, 3, 16, 16)
    z, h = m(x1, x2, return_features=True)
    assert z.shape == (6, 16) and h.shape == (6, 64)
    head = M.ProjectionHead(32, 64, 8, layers=3)
    assert head(torch.randn(5, 32)).shape == (5, 8)


def test_augment_range_shape_determinism():
    x = torch.rand(4, 3, 16, 16)
    g1, g2 = torch.Generator().manual_seed(3), torch.Generator().manual_seed(3)
    a, b = M.two_views(x, M.AugmentConfig(out_size=12), g1)
    c, _ = M.two_views(x, M.AugmentConfig(out_size=12), g2)
    assert a.shape == (4, 3, 12, 12) and float(a.min()) >= 0.0 and float(a.max()) <= 1.0
    assert torch.equal(a, c) and not torch.equal(a, b)


def test_lars_matches_sgd_without_adaptation():
    torch.manual_seed(0)
    w1 = torch.nn.Parameter(torch.randn(4, 4))
    w2 = torch.nn.Parameter(w1.detach().clone())
    o1 = M.LARS([{"params": [w1], "lars": False, "weight_decay": 0.0}], lr=0.1, momentum=0.9)
    o2 = torch.optim.SGD([w2], lr=0.1, momentum=0.9)
    for _ in range(3):
        for w, o in ((w1, o1), (w2, o2)):
            o.zero_grad()
            (w ** 2).sum().backward()
            o.step()
    torch.testing.assert_close(w1, w2)


def test_lars_trust_ratio_scales_update():
    w = torch.nn.Parameter(torch.ones(10))
    opt = M.LARS([w], lr=1.0, momentum=0.0, weight_decay=0.0, eta=1e-3)
    w.grad = torch.full((10,), 100.0)
    opt.step()
    # trust = eta * ||w|| / ||g|| -> update = lr * trust * g = 1e-3 * ||w|| * g/||g||
    torch.testing.assert_close(w.detach(), torch.ones(10) - 1e-3 * (10 ** 0.5) / 10 ** 0.5)


def test_trainer_runs_and_logs(tmp_path):
    cfg = _cfg(metrics_path=str(tmp_path / "m.jsonl"))
    hist = M.SimCLRTrainer(cfg).fit()
    assert len(hist) == 6 and all(torch.isfinite(torch.tensor(r["loss"])) for r in hist)
    assert (tmp_path / "m.jsonl").read_text().count("\n") == 6


def test_checkpoint_resume_is_exact(tmp_path):
    ref = M.SimCLRTrainer(_cfg()).fit()
    d = tmp_path / "ck"
    t1 = M.SimCLRTrainer(_cfg(ckpt_dir=str(d), ckpt_every=3))
    t1.fit(steps=3)
    assert (d / "ckpt_3.pt").exists()
    t2 = M.SimCLRTrainer(_cfg(ckpt_dir=str(d), ckpt_every=3))  # resumes from ckpt_3
    assert t2.step == 3
    rest = t2.fit()
    assert [round(r["loss"], 6) for r in rest] == [round(r["loss"], 6) for r in ref[3:]]


def test_checkpoint_roundtrip_weights_only(tmp_path):
    m = torch.nn.Linear(3, 2)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    p = save_checkpoint(tmp_path / "a.pt", model=m, optimizer=opt, step=7, extra={"k": 1})
    m2 = torch.nn.Linear(3, 2)
    st = load_checkpoint(p, model=m2, optimizer=torch.optim.SGD(m2.parameters(), lr=0.1))
    assert st["step"] == 7 and st["extra"] == {"k": 1}
    torch.testing.assert_close(m.weight, m2.weight)
    assert not (tmp_path / "a.pt.tmp").exists()


def test_utils_cpu_safe():
    t = GPUMemoryTracker()
    with t.region("x"):
        torch.ones(3)
    assert t.records[-1]["region_peak_mb"] == 0.0
    s = summarize(time_fn(lambda: torch.ones(10).sum(), iters=5, warmup=1))
    assert s["min"] <= s["mean"] <= s["max"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ddp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = M.SimCLRTrainer(_cfg(steps=3))
        hist = t.fit()
        w = next(t.model.parameters()).detach().clone()
        q.put((rank, [r["loss"] for r in hist], w.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_ddp_trainer_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=180) for _ in range(2)], key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    # identical global loss on both ranks, replicas stay in sync
    assert out[0][1] == pytest.approx(out[1][1], rel=1e-6)
    assert (out[0][2] == out[1][2]).all()
