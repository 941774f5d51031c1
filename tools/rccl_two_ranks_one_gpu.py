"""Probe: can two RCCL ranks share one MI355X? If RCCL accepts it, the symmetric data-parallel
mode's real RCCL point-to-point path (``parallel/symmetric.py``) runs at world size 2 on the
1-GPU box and is checked against the single-process fp64 oracle of the global batch.

Launched as ``python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
tools/rccl_two_ranks_one_gpu.py``. Prints one JSON line per rank."""
from __future__ import annotations

import datetime
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main() -> int:
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    # RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"): a per-rank
    # host id makes the ranks look like separate hosts, so RCCL connects them over its socket
    # transport on loopback. Same collectives, kernels and grouped P2P calls as over xGMI.
    os.environ.setdefault("NCCL_HOSTID", f"ntxent-probe-rank{rank}")
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {"rank": rank, "world": world}
    try:
        dist.init_process_group("nccl", timeout=datetime.timedelta(seconds=60))
        t = torch.full((1 << 20,), float(rank + 1), device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        out["all_reduce_ok"] = bool(torch.all(t == sum(range(1, world + 1))).item())
    except Exception as e:  # noqa: BLE001 - the probe reports whatever RCCL says
        out["error"] = f"{type(e).__name__}: {str(e)[:300]}"
        print(json.dumps(out), flush=True)
        return 0
    import ntxent_amd
    from ntxent_amd.ops import reference as R
    from ntxent_amd.parallel import symmetric

    B, d, T = 1024, 256, 0.07
    g = torch.Generator().manual_seed(7)
    shards = [torch.randn(2 * B, d, generator=g) for _ in range(world)]
    mine = shards[rank].to(dev, torch.bfloat16).requires_grad_(True)
    loss = symmetric.sym_ntxent_loss(mine, T)
    loss.backward()
    torch.cuda.synchronize()
    hg = R.global_pair_order([s.to(torch.bfloat16).double() for s in shards]).requires_grad_(True)
    lref = R.ntxent_loss(hg, T)
    (gref,) = torch.autograd.grad(lref, hg)
    N = world * B
    gm = mine.grad.double().cpu()
    err = max((gm[:B] - gref[rank * B:(rank + 1) * B]).abs().max().item(),
              (gm[B:] - gref[N + rank * B:N + (rank + 1) * B]).abs().max().item())
    out.update(loss=loss.item(), ref=lref.item(), grad_err_rel=err / gref.abs().max().item(),
               version=ntxent_amd.__version__)
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
