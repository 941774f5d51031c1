"""Multi-process data-parallel NT-Xent on CPU (gloo), SURVEY.md §4.2 item 3.

Each rank holds its own [h1_r; h2_r]; the global loss and every rank's gradient must equal
the single-process oracle on the gathered batch. This exercises the same collective pattern
as the RCCL path (all-gather of normalised rows, all-gather of LSE, all-reduce of the loss).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, dim, T, grad_out, q, mode="symmetric"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ntxent_amd.parallel import dist_ntxent_loss

        g = torch.Generator().manual_seed(1000 + rank)
        h = torch.randn(2 * n, dim, generator=g, dtype=torch.float64).requires_grad_(True)
        loss = dist_ntxent_loss(h, T, backward_mode=mode)
        loss.backward(torch.tensor(grad_out, dtype=torch.float64))
        q.put((rank, loss.detach().numpy().copy(), h.detach().numpy().copy(), h.grad.detach().numpy().copy()))
    finally:
        dist.destroy_process_group()


def _run(world, n, dim, T=0.1, grad_out=1.0, mode="symmetric"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, dim, T, grad_out, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [(r, torch.from_numpy(l), torch.from_numpy(h), torch.from_numpy(g)) for r, l, h, g in sorted(out, key=lambda x: x[0])]


@pytest.mark.parametrize("world,n,dim,mode", [(2, 4, 8, "symmetric"), (2, 5, 17, "symmetric"), (3, 3, 6, "symmetric"),
                                              (2, 4, 8, "reduce_scatter"), (3, 3, 6, "reduce_scatter")])
def test_gloo_matches_oracle(world, n, dim, mode):
    from ntxent_amd.ops import reference as ref

    T, go = 0.1, 0.7
    res = _run(world, n, dim, T, go, mode)
    shards = [r[2] for r in res]
    hg = ref.global_pair_order(shards).requires_grad_(True)
    l_ref = ref.ntxent_loss(hg, T)
    (g_ref,) = torch.autograd.grad(l_ref, hg, torch.tensor(go, dtype=hg.dtype))
    N = world * n
    for r, (_, loss, _, grad) in enumerate(res):
        torch.testing.assert_close(loss, l_ref.detach(), rtol=1e-10, atol=1e-12)
        torch.testing.assert_close(grad[:n], g_ref[r * n:(r + 1) * n], rtol=1e-9, atol=1e-12)
        torch.testing.assert_close(grad[n:], g_ref[N + r * n:N + (r + 1) * n], rtol=1e-9, atol=1e-12)
