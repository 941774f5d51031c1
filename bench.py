#!/usr/bin/env python3
"""Headline benchmark: NT-Xent fwd+bwd samples/s, B=4096 per view per GPU, d=2048, bf16.

BASELINE.json metric: "NT-Xent fwd+bwd samples/sec, B=4096 d=2048, at 1/2/4/8 MI355X".
One rank per GPU (torchrun); for N>1 negatives are gathered over RCCL/xGMI, so each GPU's
similarity work grows with N (global batch = N * 4096 pairs) while its own batch is fixed
(weak scaling). A "sample" is one positive pair. Inputs are synthetic random-normal
embeddings (no dataset); the timed region is the complete loss forward + backward
(gradient w.r.t. the embeddings) of every step.

  python bench.py [--gpus N --steps K --warmup W --batch 4096 --dim 2048 --dtype bf16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BASELINE_VALUE = None  # BASELINE.json "published": {} — the reference publishes no numbers


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096, help="pairs (per view) per GPU")
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--compute", default="auto", choices=["auto", "fp16", "bf16", "fp32"])
    ap.add_argument("--temperature", type=float, default=0.07)
    ap.add_argument("--recompute", action="store_true", help="recompute logits in backward")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--negatives", default="symmetric", choices=["allgather", "symmetric", "ring"],
                    help="N>1: symmetric = each rank pair's similarity block computed once (column partials and "
                         "partner gradient contributions exchanged point to point); allgather = every rank computes "
                         "its whole row block against the gathered rows; ring = O(local) memory")
    ap.add_argument("--data", default="views", choices=["views", "iid"],
                    help="views: two noisy views of a shared random-normal basis (positives correlated, "
                         "as from a SimCLR encoder; what build/bin/ntxent_bench uses); iid: independent "
                         "random-normal rows")
    ap.add_argument("--impl", default="fused", choices=["fused", "torch"],
                    help="torch: unfused PyTorch NT-Xent (hipBLASLt GEMM + eager softmax / cross-entropy, "
                         "the reference's cuBLAS-GEMM + row-kernel design) as an on-device baseline; 1 GPU")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--share-gpu", action="store_true", help="all ranks on cuda:0 (rehearsal with gloo)")
    ap.add_argument("--graph", action="store_true",
                    help="capture one full fwd+bwd step in a hipGraph (torch.cuda.CUDAGraph) and replay it "
                         "every step (1 GPU)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world != 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    dev_index = 0 if a.share_gpu else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    import ntxent_amd
    from ntxent_amd.parallel import dist_ntxent_loss

    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    R = 2 * a.batch
    if a.data == "views":  # positive pairs share a random-normal basis: view = basis + 0.5 noise
        base = torch.randn(a.batch, a.dim, device=dev, generator=g)
        v1 = base + 0.5 * torch.randn(a.batch, a.dim, device=dev, generator=g)
        v2 = base + 0.5 * torch.randn(a.batch, a.dim, device=dev, generator=g)
        h = torch.cat([v1, v2], 0).to(dt).requires_grad_(True)
        del base, v1, v2
    else:
        h = torch.randn(R, a.dim, device=dev, dtype=dt, generator=g).requires_grad_(True)
    if a.impl == "torch" and world > 1:
        raise SystemExit("--impl torch is a single-GPU baseline")

    one = torch.ones((), device=dev)  # d(loss)/d(loss), allocated once outside the timed loop

    def step():
        if a.impl == "torch":
            from ntxent_amd.ops.reference import ntxent_loss as torch_ntxent
            loss = torch_ntxent(h, a.temperature)
        elif world > 1:
            loss = dist_ntxent_loss(h, a.temperature, compute=a.compute, keep_logits=not a.recompute,
                                    overlap=not a.no_overlap, negatives=a.negatives)
        else:
            loss = ntxent_amd.ntxent_loss(h, a.temperature, compute=a.compute, keep_logits=not a.recompute)
        (gh,) = torch.autograd.grad(loss, h, grad_outputs=one)
        return loss, gh

    if a.graph:
        if world > 1:
            raise SystemExit("--graph is a single-GPU mode")
        side = torch.cuda.Stream()  # warm-up (plans, scratch, tile lists) outside the capture
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(2, a.warmup)):
                step()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_loss, g_gh = step()
        eager_step = step

        def step():  # noqa: F811 - every replay runs the complete forward + backward
            graph.replay()
            return g_loss, g_gh

    for _ in range(a.warmup):
        loss, gh = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss, gh = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt_s = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt_s], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_s = float(t.item())
    ms = dt_s / a.steps * 1e3
    samples = world * a.batch
    value = samples / (ms / 1e3)
    lossv = float(loss.item())
    if not (lossv == lossv) or not torch.isfinite(gh).all():
        raise SystemExit("non-finite loss or gradient")
    from ntxent_amd.ops.reference import flops_fwd_bwd

    tflops = flops_fwd_bwd(R, world * R, a.dim,
                           symmetric_global=world > 1 and a.negatives == "symmetric") / (ms / 1e3) / 1e12
    if rank == 0:
        out = {
            "metric": "NT-Xent fwd+bwd samples/sec, B=4096 d=2048, at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else value / BASELINE_VALUE,
            "dtype": a.dtype,
            "data": ("synthetic random-normal two-view embeddings (view = shared N(0,1) basis + 0.5 N(0,1))"
                     if a.data == "views" else "synthetic iid random-normal embeddings"),
            "config": {
                "model": ("NT-Xent loss (SimCLR), fused MFMA fwd+bwd" if a.impl == "fused"
                          else "NT-Xent loss (SimCLR), unfused PyTorch baseline (hipBLASLt + eager)"),
                "global_batch": world * a.batch,
                "seq_len": None,
                "batch_per_gpu": a.batch,
                "dim": a.dim,
                "temperature": a.temperature,
                "compute": a.compute,
                "mfma_dtype": (a.compute if a.compute != "auto" else ("fp32" if a.dtype == "fp32" else "fp16")),
                "keep_logits": not a.recompute,
                "parallelism": f"dp{world}",
                "negatives": a.negatives if world > 1 else None,
                "hip_graph": bool(a.graph),
            },
            "loss": lossv,
            "note": ("global-batch negatives: each rank's rows meet all N*B negatives, so per-GPU similarity "
                     "work grows linearly with N and the ideal whole-job samples/s is flat in N"
                     if world > 1 else None),
            "tflops_per_gpu_useful": round(tflops, 1),
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            Path(a.json_out).write_text(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
