"""The native C++ Engine driven from Python (ntxent_amd.parallel.native.NativeNTXent): one GPU
against the autograd op and the fp64 oracle, hipGraph capture/replay, and W processes with the
engine's own RcclComm (per-rank NCCL_HOSTID: RCCL's socket transport on the one GPU)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from ntxent_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _h(rows, dim, seed, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(rows, dim, generator=g).to("cuda", dtype)


@pytest.mark.parametrize("rows,dim,dtype", [(512, 128, torch.bfloat16), (4096, 512, torch.bfloat16),
                                            (2048, 256, torch.float32)])
def test_native_engine_matches_autograd_and_oracle(rows, dim, dtype):
    import ntxent_amd
    from ntxent_amd.parallel.native import NativeNTXent

    T = 0.07
    h = _h(rows, dim, 3, dtype)
    eng = NativeNTXent(rows, dim, T, dtype=dtype)
    loss, dh = eng.step(h)
    torch.cuda.synchronize()
    x = h.clone().requires_grad_(True)
    ref_loss = ntxent_amd.ntxent_loss(x, T)
    ref_loss.backward()
    hd = h.double().cpu().requires_grad_(True)
    lo = R.ntxent_loss(hd, T)
    (go,) = torch.autograd.grad(lo, hd)
    scale = go.abs().max().item()
    assert abs(loss.item() - lo.item()) <= 2e-3 * max(1.0, abs(lo.item())), (loss.item(), lo.item())
    assert abs(loss.item() - ref_loss.item()) <= 1e-4 * max(1.0, abs(ref_loss.item()))
    assert (dh.double().cpu() - go).abs().max().item() <= 2e-2 * scale
    assert (dh.float() - x.grad.float()).abs().max().item() <= 1e-2 * scale
    assert eng.device_bytes > 0


def test_native_engine_graph_replay_matches_step():
    from ntxent_amd.parallel.native import NativeNTXent

    rows, dim = 4096, 256
    h = _h(rows, dim, 5)
    eng = NativeNTXent(rows, dim, 0.1)
    loss, dh = eng.step(h)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()  # stream capture needs a non-default stream
    with torch.cuda.stream(side):
        gdh = eng.capture(h)
        for _ in range(3):
            gl = eng.replay()
    side.synchronize()
    assert torch.equal(gdh, dh), "graph replay differs from the eager step"
    assert gl.item() == loss.item()


def test_native_engine_graph_keeps_captured_input_alive():
    """The graph holds the captured h's device pointer: the engine keeps that tensor alive itself,
    so capture(h); del h; step(h2); replay() still replays the captured step (no read of freed
    memory), and a multi-rank capture is refused."""
    from ntxent_amd.parallel.native import NativeNTXent

    rows, dim = 4096, 256
    eng = NativeNTXent(rows, dim, 0.1)
    h = _h(rows, dim, 5)
    ref_loss, ref_dh = eng.step(h)
    ref_loss, ref_dh = ref_loss.clone(), ref_dh.clone()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        gdh = eng.capture(h.clone())  # the only reference to the captured input is the engine's
    side.synchronize()
    del h
    # an eager step on other data in between (it overwrites the engine's forward input h_)
    h2 = _h(rows, dim, 6)
    l2, _ = eng.step(h2)
    torch.cuda.synchronize()
    # churn the caching allocator so a freed captured input would be reused and overwritten
    junk = [torch.full((rows, dim), 7.0, dtype=torch.bfloat16, device="cuda") for _ in range(4)]
    with torch.cuda.stream(side):
        gl = eng.replay()
    side.synchronize()
    del junk
    assert gl.item() == ref_loss.item() and gl.item() != l2.item()
    assert torch.equal(gdh, ref_dh)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, W, port, n, dim, T, negatives, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=W)  # carries only the RCCL unique id
    try:
        from ntxent_amd.parallel.commstats import rccl_shared_gpu_env
        from ntxent_amd.parallel.native import NativeNTXent

        rccl_shared_gpu_env(rank)
        eng = NativeNTXent.from_process_group(2 * n, dim, T, negatives=negatives)
        h = _h(2 * n, dim, 100 + rank)
        loss, dh = eng.step(h)
        torch.cuda.synchronize()
        q.put((rank, loss.item(), dh.double().cpu().numpy()))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("W,n,dim,negatives", [(2, 512, 128, "symmetric"), (2, 512, 128, "allgather"),
                                               (3, 256, 64, "symmetric")])
def test_native_engine_rccl_processes_match_oracle(W, n, dim, negatives):
    T = 0.1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, W, port, n, dim, T, negatives, q)) for r in range(W)]
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
    shards = [_h(2 * n, dim, 100 + r).double().cpu() for r in range(W)]
    hg = R.global_pair_order(shards).requires_grad_(True)
    lref = R.ntxent_loss(hg, T)
    (gref,) = torch.autograd.grad(lref, hg)
    scale = gref.abs().max().item()
    N = W * n
    for r in range(W):
        loss, g = res[r]
        g = torch.from_numpy(g)
        assert abs(loss - lref.item()) <= 3e-3 * max(1.0, abs(lref.item())), (r, loss, lref.item())
        err = max((g[:n] - gref[r * n:(r + 1) * n]).abs().max().item(),
                  (g[n:] - gref[N + r * n:N + (r + 1) * n]).abs().max().item())
        assert err <= 2e-2 * scale, (r, err, scale)
