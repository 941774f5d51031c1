#!/usr/bin/env python3
"""Config-3-size correctness rehearsal of the data-parallel paths on ONE GPU (verdict r4, item 1).

Run under torchrun with W ranks that all share cuda:0 (RCCL over its socket transport, one
``NCCL_HOSTID`` per rank, ``commstats.rccl_shared_gpu_env``):

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29711 tools/w8_full_check.py --batch 4096 --dim 2048

Every rank holds B pairs (2B rows, d) of synthetic two-view data, as ``bench.py`` makes them.
Checks, at the shape the driver's 8-GPU SCALE run uses (B = 4096/rank, d = 2048, W = 8):

* the symmetric (``negatives="symmetric"``) and all-gather losses agree, and each rank's
  gradient from the two modes agrees to fp16-operand tolerance, for each ``--impls`` entry
  (the native engine behind autograd, the default on RCCL, and the torch-driven stages);
* both agree with an fp32 torch computation of the global problem (torch ops only, sharded
  like the all-gather path: each rank's rows against the gathered fp32 rows);
* peak HBM per rank of each mode (``torch.cuda.max_memory_allocated`` around one step).

Writes one JSON line (rank 0) with the per-rank errors and peaks, and exits non-zero when a
tolerance is exceeded. Timings are socket timings (all ranks share one GPU) and are reported
only as a sanity figure. The reference has no multi-GPU code.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--temperature", type=float, default=0.07)
    ap.add_argument("--steps", type=int, default=2, help="steps per mode (the last one is checked)")
    ap.add_argument("--oracle", default="fp32", choices=["fp32", "none"])
    ap.add_argument("--loss-tol", type=float, default=2e-4, help="relative loss tolerance")
    ap.add_argument("--grad-tol", type=float, default=2e-2, help="max|dg| / max|g| tolerance")
    ap.add_argument("--impls", default="engine,torch",
                    help="dist_ntxent_loss implementations to check (engine: the native C++ engine "
                         "behind autograd, the default on RCCL; torch: the Python-driven stages)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo + the torch CPU paths (plumbing test of this script)")
    a = ap.parse_args()

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    from ntxent_amd.parallel.commstats import rccl_shared_gpu_env, use_compute_stream

    on_gpu = a.device == "cuda"
    if on_gpu:
        rccl_shared_gpu_env(rank)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", device_id=dev, timeout=timedelta(seconds=900))
        use_compute_stream(dev)
    else:
        dev = torch.device("cpu")
        dist.init_process_group("gloo", timeout=timedelta(seconds=900))

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    from ntxent_amd.parallel import dist_ntxent_loss

    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    base = torch.randn(a.batch, a.dim, device=dev, generator=g)
    v1 = base + 0.5 * torch.randn(a.batch, a.dim, device=dev, generator=g)
    v2 = base + 0.5 * torch.randn(a.batch, a.dim, device=dev, generator=g)
    # bf16 on the GPU (the bench dtype); fp32 on the CPU plumbing run (CPU bf16 math is bf16)
    h = torch.cat([v1, v2], 0).to(torch.bfloat16 if on_gpu else torch.float32).requires_grad_(True)
    del base, v1, v2
    one = torch.ones((), device=dev)

    from ntxent_amd.parallel.engine_loss import cached_engine_bytes, release_engines

    impls = [i for i in a.impls.split(",") if i] if on_gpu else ["torch"]
    runs = [(m, i) for i in impls for m in ("symmetric", "allgather")]
    res = {}
    for mode, impl in runs:
        sync()
        dist.barrier()
        if on_gpu:
            torch.cuda.reset_peak_memory_stats(dev)
        base_mb = torch.cuda.memory_allocated(dev) / 2**20 if on_gpu else 0.0
        arena0 = cached_engine_bytes()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            loss = dist_ntxent_loss(h, a.temperature, negatives=mode, impl=impl)
            (gh,) = torch.autograd.grad(loss, h, grad_outputs=one)
        sync()
        dt = (time.perf_counter() - t0) / a.steps
        # torch allocator peak of the step + the engine arena this mode created (outside torch)
        peak = (torch.cuda.max_memory_allocated(dev) / 2**20 - base_mb + (cached_engine_bytes() - arena0) / 2**20
                if on_gpu else 0.0)
        res[(mode, impl)] = (float(loss.item()), gh.detach().float(), peak, dt * 1e3)
        del gh, loss
    release_engines()

    # every run against the first all-gather run (loss, gradient), and the first two as before
    ls, gs, peak_s, ms_s = res[runs[0]]
    la, ga, peak_a, ms_a = res[runs[1]]
    gmax = ga.abs().max().item()
    err_sa = max((res[k][1] - ga).abs().max().item() for k in runs) / max(gmax, 1e-30)
    loss_sa = max(abs(res[k][0] - la) for k in runs) / max(abs(la), 1e-30)

    # fp32 torch oracle of the global problem, sharded the all-gather way (each rank: its rows
    # against the gathered fp32 rows; ops/reference.sharded_forward_backward, which the CPU
    # tests pin to the unsharded fp64 oracle), independent of every HIP kernel
    loss_ref = None
    err_ref = [None, None]
    if a.oracle == "fp32":
        from ntxent_amd.ops import reference as R

        with torch.no_grad():
            z, inv = R.normalize(h.detach().float())
            parts = [torch.empty_like(z) for _ in range(world)]
            dist.all_gather(parts, z)
            z_all = torch.cat(parts, 0)
            del parts
            Rl = z.shape[0]
            n = Rl // 2
            ar = torch.arange(Rl, device=dev)
            own = ar + rank * Rl
            pos = (ar + n) % Rl + rank * Rl
            S = z @ z_all.t() / a.temperature
            S[ar, own] = float("-inf")
            lse = torch.logsumexp(S, 1)
            lsum = (lse - S[ar, pos]).sum().double()
            dist.all_reduce(lsum)
            loss_ref = float(lsum.item()) / (world * Rl)
            lparts = [torch.empty_like(lse) for _ in range(world)]
            dist.all_gather(lparts, lse)
            lse_all = torch.cat(lparts)
            S.sub_(lse.unsqueeze(1))
            Cm = torch.exp(S)
            S.add_(lse.unsqueeze(1)).sub_(lse_all.unsqueeze(0))
            Cm.add_(torch.exp(S))
            del S
            Cm[ar, own] = 0.0
            Cm[ar, pos] -= 2.0
            dz = (Cm @ z_all) / (world * Rl * a.temperature)
            del Cm, z_all
            dot = (z * dz).sum(1, keepdim=True)
            mine = inv.unsqueeze(1) * (dz - z * dot)
            del dz, z
        gm = mine.abs().max().item()
        err_runs = [(res[k][1] - mine).abs().max().item() / gm for k in runs]
        err_ref = [max(e for k, e in zip(runs, err_runs) if k[0] == "symmetric"),
                   max(e for k, e in zip(runs, err_runs) if k[0] == "allgather")]
        del mine

    row = torch.tensor([loss_sa, err_sa, max(res[k][2] for k in runs if k[0] == "symmetric"),
                        max(res[k][2] for k in runs if k[0] == "allgather"), ms_s, ms_a,
                        -1.0 if err_ref[0] is None else err_ref[0],
                        -1.0 if err_ref[1] is None else err_ref[1]]
                       + [res[k][2] for k in runs] + [res[k][0] for k in runs], dtype=torch.float64, device=dev)
    allrows = [torch.empty_like(row) for _ in range(world)]
    dist.all_gather(allrows, row)
    ok = True
    if rank == 0:
        per = [r.tolist() for r in allrows]
        # each mode within grad_tol of the fp32 oracle; symmetric vs all-gather (two independent bf16
        # roundings of the gradient) within twice that
        worst_grad = max(max(p[1] / 2, p[6], p[7]) for p in per)
        worst_loss = max(p[0] for p in per)
        nr = len(runs)
        losses = {f"{m}/{i}": per[0][8 + nr + j] for j, (m, i) in enumerate(runs)}
        lref_err = None if loss_ref is None else max(abs(v - loss_ref) for v in losses.values()) / abs(loss_ref)
        ok = worst_grad <= a.grad_tol and worst_loss <= a.loss_tol and (lref_err is None or lref_err <= a.loss_tol)
        out = {
            "check": "w8_full", "ok": ok, "world": world, "batch_per_rank": a.batch, "dim": a.dim,
            "loss_symmetric": ls, "loss_allgather": la, "loss_fp32_torch": loss_ref,
            "loss_rel_err_vs_fp32": lref_err, "runs": [f"{m}/{i}" for m, i in runs], "losses": losses,
            "peak_mib_per_run_max_over_ranks": {f"{m}/{i}": round(max(p[8 + j] for p in per), 1)
                                                for j, (m, i) in enumerate(runs)},
            "per_rank": [{"rank": i, "loss_rel_sym_vs_ag": p[0], "grad_err_sym_vs_ag": p[1],
                          "grad_err_sym_vs_fp32": p[6], "grad_err_ag_vs_fp32": p[7],
                          "peak_mib_symmetric": round(p[2], 1), "peak_mib_allgather": round(p[3], 1),
                          "socket_ms_symmetric": round(p[4], 1), "socket_ms_allgather": round(p[5], 1)}
                         for i, p in enumerate(per)],
            "tolerances": {"loss_rel": a.loss_tol, "grad_max_rel": a.grad_tol},
            "note": ("all ranks share one GPU over RCCL sockets: timings are not xGMI timings" if on_gpu
                     else "CPU / gloo plumbing run"),
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            Path(a.json_out).write_text(line + "\n")
    flag = torch.tensor([0.0 if ok else 1.0], device=dev)
    dist.broadcast(flag, 0)
    dist.barrier()
    dist.destroy_process_group()
    if flag.item() != 0.0:
        raise SystemExit("w8_full_check: tolerance exceeded")


if __name__ == "__main__":
    main()
