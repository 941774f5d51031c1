"""Symmetric data-parallel mode (parallel/symmetric.py) on CPU: the block assignment covers
every rank pair's similarity block exactly once and balances the work; W gloo processes
running the torch implementation of the same exchanges (column partials forward, partner
gradient contributions backward) reproduce the single-process fp64 oracle."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ntxent_amd.parallel.symmetric import sym_incoming, sym_jobs, sym_work_blocks


@pytest.mark.parametrize("W", range(1, 10))
@pytest.mark.parametrize("rt", [1, 2, 3, 4, 7, 32])
def test_assignment_covers_each_pair_once(W, rt):
    cover = {}
    for r in range(W):
        for (q, m0, m1, k0, k1) in sym_jobs(W, r, rt):
            assert q != r and 0 <= q < W
            assert 0 <= m0 < m1 <= rt and 0 <= k0 < k1 <= rt
            for i in range(m0, m1):
                for j in range(k0, k1):
                    key = (min(r, q), max(r, q), i if r < q else j, j if r < q else i)
                    assert key not in cover, f"block tile {key} computed twice"
                    cover[key] = r
    assert len(cover) == W * (W - 1) // 2 * rt * rt
    work = sym_work_blocks(W, rt)
    if W > 1:
        assert max(work) - min(work) <= 1.0 / rt + 1e-9  # at most one row-tile panel apart
        assert abs(sum(work) - W * (W - 1) / 2) < 1e-9


@pytest.mark.parametrize("W", range(2, 9))
def test_incoming_mirrors_jobs(W):
    rt = 5
    for r in range(W):
        for (p, m0, m1, k0, k1) in sym_incoming(W, r, rt):
            assert (r, m0, m1, k0, k1) in sym_jobs(W, p, rt)
    n_msgs = sum(len(sym_jobs(W, r, rt)) for r in range(W))
    assert n_msgs == sum(len(sym_incoming(W, r, rt)) for r in range(W))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, dim, T, grad_out, tile, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ntxent_amd.parallel.symmetric import cpu_sym_ntxent_loss

        g = torch.Generator().manual_seed(2000 + rank)
        h = torch.randn(2 * n, dim, generator=g, dtype=torch.float64).requires_grad_(True)
        loss = cpu_sym_ntxent_loss(h, T, tile=tile)
        loss.backward(torch.tensor(grad_out, dtype=torch.float64))
        q.put((rank, loss.detach().numpy().copy(), h.detach().numpy().copy(), h.grad.detach().numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,dim,tile", [(2, 4, 8, 2), (2, 5, 7, 3), (3, 3, 6, 2), (4, 3, 5, 2), (4, 4, 6, 8)])
def test_gloo_symmetric_matches_oracle(world, n, dim, tile):
    from ntxent_amd.ops import reference as ref

    T, go = 0.1, 0.7
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, dim, T, go, tile, qu)) for r in range(world)]
    for p in procs:
        p.start()
    out = [qu.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = [(r, torch.from_numpy(l), torch.from_numpy(h), torch.from_numpy(g)) for r, l, h, g in sorted(out, key=lambda x: x[0])]
    shards = [r[2] for r in res]
    hg = ref.global_pair_order(shards).requires_grad_(True)
    l_ref = ref.ntxent_loss(hg, T)
    (g_ref,) = torch.autograd.grad(l_ref, hg, torch.tensor(go, dtype=hg.dtype))
    N = world * n
    for r, (_, loss, _, grad) in enumerate(res):
        torch.testing.assert_close(loss, l_ref.detach(), rtol=1e-10, atol=1e-12)
        torch.testing.assert_close(grad[:n], g_ref[r * n:(r + 1) * n], rtol=1e-9, atol=1e-12)
        torch.testing.assert_close(grad[n:], g_ref[N + r * n:N + (r + 1) * n], rtol=1e-9, atol=1e-12)
