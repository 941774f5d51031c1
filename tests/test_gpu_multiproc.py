"""The real torch.distributed path (DistNTXentFunction: async gathers, own-tile / remote-tile
overlap, LSE all-gather, loss all-reduce, rank-local symmetric backward) with W processes.

On a 1-GPU box the W ranks share cuda:0 and talk over gloo (its collectives stage GPU tensors
through the host) or over RCCL itself (per-rank host ids, RCCL's socket transport); every HIP
kernel, plan and buffer is the one a W-GPU RCCL run uses. Results are checked against the fp64 oracle on the gathered batch.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shards(W, n, dim, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(W):
        base = torch.randn(n, dim, generator=g, dtype=torch.float64)
        out.append(torch.cat([base + 0.3 * torch.randn(n, dim, generator=g, dtype=torch.float64),
                              base + 0.3 * torch.randn(n, dim, generator=g, dtype=torch.float64)], 0))
    return out


def _worker(rank, W, port, n, dim, T, compute, keep, overlap, mode, q, negatives="allgather", backend="gloo"):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    if backend == "nccl":
        from ntxent_amd.parallel.commstats import rccl_shared_gpu_env

        rccl_shared_gpu_env(rank)
        dist.init_process_group("nccl", rank=rank, world_size=W, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=W)
    try:
        from ntxent_amd.parallel import dist_ntxent_loss

        h = _shards(W, n, dim, seed=11)[rank].float().cuda().requires_grad_(True)
        loss = dist_ntxent_loss(h, T, compute=compute, keep_logits=keep, overlap=overlap, backward_mode=mode,
                                negatives=negatives)
        (g,) = torch.autograd.grad(loss, h, torch.tensor(0.7, device=h.device))
        torch.cuda.synchronize()
        q.put((rank, loss.item(), g.double().cpu().numpy()))  # by value: no shared-memory fd hand-off
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("W,n,dim,compute,keep,overlap,mode,negatives", [
    (2, 256, 128, "fp32", True, True, "symmetric", "allgather"),
    (2, 300, 96, "fp16", False, True, "symmetric", "allgather"),
    (3, 128, 64, "fp16", True, False, "symmetric", "allgather"),
    (2, 128, 64, "fp32", True, True, "reduce_scatter", "allgather"),
    (2, 256, 128, "fp32", False, True, "symmetric", "ring"),
    (3, 150, 100, "fp16", False, True, "symmetric", "ring"),
    (2, 300, 96, "fp16", True, True, "symmetric", "symmetric"),
    (4, 256, 64, "fp32", True, True, "symmetric", "symmetric"),
    (3, 384, 80, "fp16", True, True, "symmetric", "symmetric"),
    (2, 2048, 64, "fp16", True, True, "symmetric", "symmetric"),  # 16 row tiles: 4 exchange chunks
    (8, 128, 64, "fp32", False, True, "symmetric", "ring"),        # W = 8 ring
])
def test_multiprocess_matches_oracle(W, n, dim, compute, keep, overlap, mode, negatives):
    _run_and_check(W, n, dim, compute, keep, overlap, mode, negatives, "gloo")


# RCCL itself at W > 1 on the 1-GPU box: per-rank NCCL_HOSTID makes RCCL accept two ranks on one
# device and connect them over its socket transport (commstats.rccl_shared_gpu_env), so the
# grouped batch_isend_irecv of the symmetric mode, the async all-gathers / reduce-scatter of the
# all-gather mode and the ring's exchanges run through RCCL's communicator and kernels, with the
# GEMMs' comm CU reserve active (only the wire is not xGMI).
@pytest.mark.parametrize("W,n,dim,compute,keep,overlap,mode,negatives", [
    (2, 512, 128, "fp16", False, True, "symmetric", "symmetric"),
    (2, 2048, 64, "fp16", True, True, "symmetric", "symmetric"),
    (3, 384, 80, "fp32", True, True, "symmetric", "symmetric"),
    (2, 300, 96, "fp16", False, True, "symmetric", "allgather"),
    (2, 128, 64, "fp32", True, True, "reduce_scatter", "allgather"),
    (2, 256, 128, "fp16", False, True, "symmetric", "ring"),
    # W = 8, the driver's scaling-run world size: 3 full partner blocks + a split pair per rank
    # (symmetric), 7 gathered blocks (all-gather); 8 processes sharing the GPU over sockets
    (8, 256, 64, "fp16", True, True, "symmetric", "symmetric"),
    (8, 256, 64, "fp16", False, True, "symmetric", "allgather"),
])
def test_multiprocess_rccl_matches_oracle(W, n, dim, compute, keep, overlap, mode, negatives):
    _run_and_check(W, n, dim, compute, keep, overlap, mode, negatives, "nccl")


def _run_and_check(W, n, dim, compute, keep, overlap, mode, negatives, backend):
    T = 0.1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, W, port, n, dim, T, compute, keep, overlap, mode, q, negatives,
                                               backend))
             for r in range(W)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(W):
        r, loss, g = q.get(timeout=240)
        res[r] = (loss, g)
    for p in procs:
        p.join(timeout=60)
    for r, (loss, g) in res.items():
        assert g is not None, f"rank {r} failed: {loss}"
        res[r] = (loss, torch.from_numpy(g))
    hg = R.global_pair_order([s.float().double() for s in _shards(W, n, dim, seed=11)]).requires_grad_(True)
    lref = R.ntxent_loss(hg, T)
    (gref,) = torch.autograd.grad(lref, hg, torch.tensor(0.7, dtype=torch.float64))
    lt, gt = {"fp32": (2e-5, 2e-4), "fp16": (3e-3, 2e-2)}[compute]
    scale = gref.abs().max().item()
    N = W * n
    for r in range(W):
        loss, g = res[r]
        assert abs(loss - lref.item()) <= lt * max(1.0, abs(lref.item())), (r, loss, lref.item())
        err = max((g[:n] - gref[r * n:(r + 1) * n]).abs().max().item(),
                  (g[n:] - gref[N + r * n:N + (r + 1) * n]).abs().max().item())
        assert err <= gt * scale, (r, err, scale)
