"""The data-parallel paths on the real RCCL backend ("nccl" on ROCm), rehearsed on one GPU.

A one-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one device), so every
multi-rank test elsewhere runs on gloo with host staging. This file drives the RCCL-only
branches with a world-1 NCCL process group instead:

  * ``_p2p``'s ``dist.batch_isend_irecv`` branch (self send/recv in one grouped batch: RCCL
    runs it as a device kernel on the communicator's stream, like a peer transfer);
  * the RCCL CU reserve (``reserve_cus``: the GEMM leaves CUs free while a transfer is in
    flight) -- results must be bitwise those of the same launch without the transfer;
  * the all-gather / ring / symmetric data-parallel autograd functions end to end on RCCL
    collectives (world 1: every collective is a device-local copy), against the single-GPU op.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

from test_gpu_kernels import _inputs

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_group():
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", world_size=1, rank=0,
                            device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield dist.group.WORLD
    dist.barrier()
    dist.destroy_process_group()


def _upper_cosines(sc, rows):
    """Kept cosines (16-bit canonical fragment order) with the lower 64x64 regions of the own
    block's diagonal tiles (the last rows / 256 tiles) zeroed."""
    rt = (rows + 255) // 256
    t = sc.float().view(-1, 16, 8, 512).clone()  # [tile][16-row block][32-col pair][lane * 8]
    i = torch.arange(16, device=sc.device).view(16, 1)
    j = torch.arange(8, device=sc.device).view(1, 8)
    lower = (i >> 2) > (j >> 1)
    t[-rt:][:, lower] = 0
    return t


def test_p2p_batch_self_send_recv(nccl_group):
    from ntxent_amd.parallel.symmetric import _p2p

    g = torch.Generator(device="cuda").manual_seed(5)
    sends = [torch.randn(4096, 2048, device="cuda", generator=g).half() for _ in range(2)]  # 2 x 16 MiB
    recvs = [torch.empty_like(t) for t in sends]
    works = _p2p([(t, 0) for t in sends], [(t, 0) for t in recvs], nccl_group)
    assert works, "RCCL branch must return work handles (the gloo branch completes inline)"
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    for a, b in zip(sends, recvs):
        assert torch.equal(a, b)


def test_comm_overlap_reserve_is_bitwise_neutral(nccl_group, ext):
    """A forward GEMM launched under the RCCL CU reserve while a 256 MiB self-transfer is in
    flight gives exactly the results of the same launch without the transfer (the reserve
    changes the persistent schedule, hence the rounding of split tiles: against the unreserved
    launch it is held to rounding level)."""
    from ntxent_amd.parallel.commstats import comm_reserve_cus
    from ntxent_amd.parallel.symmetric import _p2p

    reserve = comm_reserve_cus("nccl")
    assert reserve > 0
    rows, dim = 8192, 1024
    _, h = _inputs(rows, dim, torch.bfloat16, seed=9)
    plan = ext.get_plan(rows, dim, 1, 0, 0.07, "fp16", 0)
    zq, inv, ypos, _ = ext.prep(h, plan)
    outs = {}
    for res, xfer in ((0, False), (reserve, False), (reserve, True)):
        big = torch.ones(64 * 1024 * 1024, dtype=torch.float32, device="cuda")
        dst = torch.empty_like(big)
        works = _p2p([(big, 0)], [(dst, 0)], nccl_group) if xfer else []
        part = torch.empty((plan.col_tiles, plan.rows_pad, 2), dtype=torch.float32, device="cuda")
        sc = torch.zeros((plan.n_fwd_tiles * 256 * 256,), dtype=torch.float16, device="cuda")
        ext.fwd_stats_range(zq, zq, plan, part, sc, 0, plan.n_fwd_tiles, reserve_cus=res)
        for w in works:
            w.wait()
        torch.cuda.synchronize()
        outs[(res, xfer)] = (part.clone(), sc.clone())
        if xfer:
            assert torch.equal(dst, big)
    a, b, c = outs[(0, False)], outs[(reserve, False)], outs[(reserve, True)]
    assert torch.equal(b[0], c[0]) and torch.equal(b[1], c[1])
    # the kept cosines do not depend on the schedule beyond rounding: the reserve moves diagonal
    # tiles between the whole-tile GEMM and the remainder kernel, which sums two K halves of the
    # upper regions and leaves the lower ones (mirrored by the coefficient pass) unwritten
    ka, kb = _upper_cosines(a[1], rows), _upper_cosines(b[1], rows)
    torch.testing.assert_close(ka, kb, rtol=0, atol=1e-3)
    torch.testing.assert_close(a[0], b[0], rtol=1e-5, atol=0)


@pytest.mark.parametrize("negatives", ["allgather", "ring", "symmetric"])
def test_dist_loss_on_rccl_world1(nccl_group, negatives):
    """Each data-parallel mode's autograd function on RCCL collectives equals the single-GPU op
    (symmetric mode is driven through its autograd function directly: the public entry point
    short-circuits to the single-GPU op at world size 1)."""
    import ntxent_amd
    from ntxent_amd.parallel import dist_ntxent_loss
    from ntxent_amd.parallel.symmetric import SymNTXentFunction

    _, h = _inputs(4096, 512, torch.bfloat16, seed=21)
    x0 = h.clone().requires_grad_(True)
    l0 = ntxent_amd.ntxent_loss(x0, 0.1, compute="fp16")
    (g0,) = torch.autograd.grad(l0, x0)
    x1 = h.clone().requires_grad_(True)
    if negatives == "symmetric":
        l1 = SymNTXentFunction.apply(x1, 0.1, "fp16", nccl_group)
    else:
        l1 = dist_ntxent_loss(x1, 0.1, group=nccl_group, compute="fp16", negatives=negatives)
    (g1,) = torch.autograd.grad(l1, x1)
    torch.cuda.synchronize()
    assert abs(l1.item() - l0.item()) <= 1e-5 * abs(l0.item())
    scale = g0.float().abs().max().item()
    assert (g1.float() - g0.float()).abs().max().item() <= 2e-2 * scale


def test_dist_loss_on_compute_stream(nccl_group):
    """The data-parallel step on a high-priority compute stream (use_compute_stream, as bench.py
    and the trainer run it): same loss / gradient as on the default stream, and the transfer's
    work handles order the compute stream correctly."""
    import ntxent_amd
    from ntxent_amd.parallel import use_compute_stream
    from ntxent_amd.parallel.symmetric import SymNTXentFunction

    _, h = _inputs(4096, 512, torch.bfloat16, seed=23)
    x0 = h.clone().requires_grad_(True)
    l0 = SymNTXentFunction.apply(x0, 0.1, "fp16", nccl_group)
    (g0,) = torch.autograd.grad(l0, x0)
    torch.cuda.synchronize()
    old = torch.cuda.current_stream()
    s = use_compute_stream()
    try:
        assert torch.cuda.current_stream() == s and s != torch.cuda.default_stream()
        x1 = h.clone().requires_grad_(True)
        l1 = SymNTXentFunction.apply(x1, 0.1, "fp16", nccl_group)
        (g1,) = torch.autograd.grad(l1, x1)
        torch.cuda.synchronize()
    finally:
        torch.cuda.set_stream(old)
    assert l1.item() == l0.item()
    assert torch.equal(g1, g0)
