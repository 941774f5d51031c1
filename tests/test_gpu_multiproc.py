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


def _worker(rank, W, port, n, dim, T, compute, keep, overlap, mode, q, negatives="allgather", backend="gloo",
            impl="auto"):
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
        from ntxent_amd.parallel.engine_loss import cached_engine_bytes, release_engines

        loss = dist_ntxent_loss(h, T, compute=compute, keep_logits=keep, overlap=overlap, backward_mode=mode,
                                negatives=negatives, impl=impl)
        (g,) = torch.autograd.grad(loss, h, torch.tensor(0.7, device=h.device))
        torch.cuda.synchronize()
        used = "engine" if cached_engine_bytes() > 0 else "torch"
        release_engines()
        if impl != "auto" and used != impl:
            raise RuntimeError(f"asked impl={impl}, ran {used}")
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
# impl: "engine" = the native C++ engine behind autograd (parallel/engine_loss.py, the default of
# dist_ntxent_loss on RCCL); "torch" = the Python-driven stages over torch.distributed.
@pytest.mark.parametrize("W,n,dim,compute,keep,overlap,mode,negatives,impl", [
    (2, 512, 128, "fp16", False, True, "symmetric", "symmetric", "engine"),
    (2, 512, 128, "fp16", False, True, "symmetric", "symmetric", "torch"),
    (2, 2048, 64, "fp16", True, True, "symmetric", "symmetric", "engine"),
    (2, 2048, 64, "fp16", True, True, "symmetric", "symmetric", "torch"),
    (3, 384, 80, "fp32", True, True, "symmetric", "symmetric", "engine"),
    (3, 384, 80, "fp32", True, True, "symmetric", "symmetric", "torch"),
    (2, 300, 96, "fp16", False, True, "symmetric", "allgather", "engine"),
    (2, 300, 96, "fp16", False, True, "symmetric", "allgather", "torch"),
    (2, 256, 64, "fp8", True, True, "symmetric", "symmetric", "engine"),
    (2, 128, 64, "fp32", True, True, "reduce_scatter", "allgather", "torch"),
    (2, 256, 128, "fp16", False, True, "symmetric", "ring", "torch"),
    # W = 8, the driver's scaling-run world size: 3 full partner blocks + a split pair per rank
    # (symmetric), 7 gathered blocks (all-gather); 8 processes sharing the GPU over sockets
    (8, 256, 64, "fp16", True, True, "symmetric", "symmetric", "engine"),
    (8, 256, 64, "fp16", True, True, "symmetric", "symmetric", "torch"),
    (8, 256, 64, "fp16", False, True, "symmetric", "allgather", "engine"),
    (8, 256, 64, "fp16", False, True, "symmetric", "allgather", "torch"),
])
def test_multiprocess_rccl_matches_oracle(W, n, dim, compute, keep, overlap, mode, negatives, impl):
    _run_and_check(W, n, dim, compute, keep, overlap, mode, negatives, "nccl", impl)


def test_config3_shape_rccl_w4(tmp_path):
    """The SCALE run's per-rank shape (B = 4096 pairs/rank, d = 2048, bf16 inputs: 8192 rows x
    2048, 32 row tiles, 4 exchange chunks of 8 row tiles per peer, a split pair) at W = 4 over
    RCCL, both negatives modes on both implementations (tools/w8_full_check.py): symmetric ==
    all-gather loss, every gradient within 4e-3 of max|g| of an fp32 torch oracle of the global
    problem, and a per-rank HBM bound (torch allocator peak + the engine arena)."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    out = tmp_path / "c3.json"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        str(root / "tools" / "w8_full_check.py"), "--batch", "4096", "--dim", "2048", "--steps", "1",
                        "--grad-tol", "4e-3", "--impls", "engine,torch", "--json-out", str(out)],
                       capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    d = json.loads(out.read_text())
    assert d["ok"] and d["world"] == 4 and d["runs"] == ["symmetric/engine", "allgather/engine",
                                                          "symmetric/torch", "allgather/torch"]
    for p in d["per_rank"]:
        assert p["loss_rel_sym_vs_ag"] <= 1e-6, p
        assert p["grad_err_sym_vs_fp32"] <= 4e-3 and p["grad_err_ag_vs_fp32"] <= 4e-3, p
        assert 0 < p["peak_mib_symmetric"] <= 3072 and 0 < p["peak_mib_allgather"] <= 3072, p
    assert d["loss_rel_err_vs_fp32"] <= 1e-5


def _run_and_check(W, n, dim, compute, keep, overlap, mode, negatives, backend, impl="auto"):
    T = 0.1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, W, port, n, dim, T, compute, keep, overlap, mode, q, negatives,
                                               backend, impl))
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
    lt, gt = {"fp32": (2e-5, 2e-4), "fp16": (3e-3, 2e-2), "fp8": (5e-2, 0.3)}[compute]  # fp8: e4m3 rows vs the unquantised oracle
    scale = gref.abs().max().item()
    N = W * n
    for r in range(W):
        loss, g = res[r]
        assert abs(loss - lref.item()) <= lt * max(1.0, abs(lref.item())), (r, loss, lref.item())
        err = max((g[:n] - gref[r * n:(r + 1) * n]).abs().max().item(),
                  (g[n:] - gref[N + r * n:N + (r + 1) * n]).abs().max().item())
        assert err <= gt * scale, (r, err, scale)
