#!/usr/bin/env python3
"""Headline benchmark: NT-Xent fwd+bwd samples/s, B=4096 per view per GPU, d=2048, bf16.

BASELINE.json metric: "NT-Xent fwd+bwd samples/sec, B=4096 d=2048, at 1/2/4/8 MI355X".
One rank per GPU; for N>1 negatives are exchanged over RCCL/xGMI, so each GPU's similarity
work grows with N (global batch = N * 4096 pairs) while its own batch is fixed (weak
scaling). A "sample" is one positive pair. Inputs are synthetic random-normal embeddings (no
dataset); the timed region is the complete loss forward + backward (gradient w.r.t. the
embeddings) of every step.

Launch modes (the reference only links MPI/NCCL in CMake, /root/reference/CMakeLists.txt:13-14,
41-47; here the ranks are real processes over RCCL):
  * ``python bench.py --gpus N``: with no WORLD_SIZE in the environment and N > 1 this process
    is a LAUNCHER. It never touches the GPU; it starts N rank processes of this script
    (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1/MASTER_PORT set), relays rank 0's single
    JSON line, and exits non-zero if any rank fails or the job exceeds ``--timeout``.
  * ``torchrun --nproc-per-node N bench.py --gpus N``: each process is a rank already.
A rank whose WORLD_SIZE disagrees with ``--gpus`` exits with an error (never silently runs
fewer GPUs than asked).

  python bench.py [--gpus N --steps K --warmup W --batch 4096 --dim 2048 --dtype bf16]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import signal
import socket
import subprocess
import sys
import time
from datetime import timedelta
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402

METRIC = "NT-Xent fwd+bwd samples/sec, B=4096 d=2048, at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # BASELINE.json "published": {} — the reference publishes no numbers
CHILD_ENV = "NTXENT_BENCH_RANK_CHILD"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096, help="pairs (per view) per GPU")
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--compute", default="auto", choices=["auto", "fp16", "bf16", "fp32", "fp8"])
    ap.add_argument("--temperature", type=float, default=0.07)
    ap.add_argument("--recompute", action="store_true", help="recompute logits in backward")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--compute-stream", default="high", choices=["default", "new", "high"],
                    help="stream the step runs on: the device's default stream, a new stream, or a new "
                         "high-priority stream (default; RCCL kernels then run beside the GEMMs instead of "
                         "queueing behind them on a shared hardware queue, profiles/r3/overlap)")
    ap.add_argument("--negatives", default="symmetric", choices=["allgather", "symmetric", "ring"],
                    help="N>1: symmetric = each rank pair's similarity block computed once (column partials and "
                         "partner gradient contributions exchanged point to point); allgather = every rank computes "
                         "its whole row block against the gathered rows; ring = O(local) memory")
    ap.add_argument("--dist-impl", default="auto", choices=["auto", "engine", "torch"],
                    help="N>1, --impl fused: auto/engine = the native C++ engine behind autograd "
                         "(parallel/engine_loss.py: one C++ call per forward/backward, its own RCCL "
                         "communicator); torch = the Python-driven stages over torch.distributed")
    ap.add_argument("--host-profile", default=None,
                    help="rank 0: cProfile of 10 extra steps' host enqueue after the timed region, top "
                         "entries written to this path (where the host time of a step goes)")
    ap.add_argument("--data", default="views", choices=["views", "iid"],
                    help="views: two noisy views of a shared random-normal basis (positives correlated, "
                         "as from a SimCLR encoder); iid: independent random-normal rows")
    ap.add_argument("--impl", default="fused", choices=["fused", "native", "torch"],
                    help="torch: unfused PyTorch NT-Xent (hipBLASLt GEMM + eager softmax / cross-entropy, "
                         "the reference's cuBLAS-GEMM + row-kernel design) as an on-device baseline; 1 GPU")
    ap.add_argument("--backend", default=None, choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (GPU default); gloo = CPU transport (--device cpu, or the "
                         "--share-gpu rehearsal of N ranks on one GPU)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: run the same launcher / timing / JSON path on CPU tensors (plumbing tests)")
    ap.add_argument("--share-gpu", action="store_true", help="all ranks on cuda:0 (rehearsal with gloo)")
    ap.add_argument("--graph", action="store_true",
                    help="capture one full fwd+bwd step in a hipGraph (torch.cuda.CUDAGraph) and replay it "
                         "every step (1 GPU)")
    ap.add_argument("--secondary-fp32", default="auto", choices=["auto", "on", "off"],
                    help="also time the exact-fp32 MFMA path (fp32 inputs, fp32 compute) at the same shape "
                         "(auto: on for 1 GPU)")
    ap.add_argument("--prewarm-steps", type=int, default=60,
                    help="untimed steps run BEFORE the --warmup steps so the timed region measures the "
                         "steady state: from a cold start the GPU clock ramps for ~60 steps (0.51 ms/step "
                         "at steps 10-19, 0.44 from step 60 on: profiles/r2/ramp); reported in the JSON")
    ap.add_argument("--timeout", type=float, default=1500.0,
                    help="launcher: seconds before the whole job is killed; ranks: process-group timeout")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------
# launcher (no GPU access in this process)
# ------------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base: dict, r: int, n: int, port: int) -> dict:
    """Environment of rank r of an n-rank single-node job (what torchrun would set): rank r is
    LOCAL_RANK r, so run_rank puts it on cuda:r (rank_device)."""
    env = dict(base)
    env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **{CHILD_ENV: "1"})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return env


def rank_device(local_rank: int, share_gpu: bool) -> int:
    """GPU index of a rank: its LOCAL_RANK (one rank per GPU), or 0 for the one-GPU rehearsal."""
    return 0 if share_gpu else int(local_rank)


def launch(a, argv) -> int:
    """Start a.gpus rank processes of this script and relay rank 0's JSON line."""
    n = a.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = rank_env(os.environ, r, n, port)
        cmd = [sys.executable, "-u", str(Path(__file__).resolve()), *argv]
        # rank 0's stdout carries the JSON line; every rank's stderr passes through
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                                      stderr=None, start_new_session=True, text=True))

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t_end = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass

    deadline = time.time() + a.timeout
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = f"rank {bad[0][0]} exited with code {bad[0][1]}"
            break
        if all(c == 0 for c in codes):
            break
        if time.time() > deadline:
            failed = f"timeout after {a.timeout:.0f} s"
            break
        time.sleep(0.2)
    if failed:
        kill_all()  # before reading: a rank blocked in a collective would never close its pipe
    out = procs[0].stdout.read() if procs[0].stdout else ""
    if failed:
        sys.stderr.write(f"bench launcher: {failed}; rank 0 stdout:\n{out}\n")
        return 1
    lines = [l for l in out.splitlines() if l.startswith("{")]
    if len(lines) != 1:
        sys.stderr.write(f"bench launcher: expected one JSON line from rank 0, got {len(lines)}:\n{out}\n")
        return 1
    rec = json.loads(lines[0])
    if rec.get("n_gpus") != n or rec.get("world_size_seen") != n:
        sys.stderr.write(f"bench launcher: rank 0 reports n_gpus={rec.get('n_gpus')} "
                         f"world_size_seen={rec.get('world_size_seen')}, expected {n}\n")
        return 1
    print(lines[0], flush=True)
    if a.json_out:
        Path(a.json_out).write_text(lines[0] + "\n")
    return 0


# ------------------------------------------------------------------------------------------
# one rank
# ------------------------------------------------------------------------------------------
def _stats(ms):
    m = sum(ms) / len(ms)
    sd = math.sqrt(sum((x - m) ** 2 for x in ms) / len(ms)) if len(ms) > 1 else 0.0
    return {"mean": round(m, 4), "std": round(sd, 4), "min": round(min(ms), 4), "max": round(max(ms), 4)}


def run_rank(a) -> None:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        raise SystemExit(f"bench: --gpus {a.gpus} but this process belongs to a job of WORLD_SIZE={world} "
                         f"(run `python bench.py --gpus {a.gpus}` to launch the ranks, or torchrun with "
                         f"--nproc-per-node {a.gpus})")
    on_gpu = a.device == "cuda"
    backend = a.backend or ("nccl" if on_gpu else "gloo")
    if not on_gpu and backend != "gloo":
        raise SystemExit("--device cpu needs the gloo backend")
    if on_gpu:
        dev_index = rank_device(local_rank, a.share_gpu)
        if not a.share_gpu and dev_index >= torch.cuda.device_count():
            raise SystemExit(f"bench: LOCAL_RANK {local_rank} but only {torch.cuda.device_count()} GPUs visible")
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
    else:
        dev = torch.device("cpu")
        torch.set_num_threads(max(1, min(4, (os.cpu_count() or 1) // max(1, world))))
    world_seen = 1
    if world > 1:
        kw = {"timeout": timedelta(seconds=a.timeout)}
        if backend == "nccl":
            if a.share_gpu:  # RCCL rehearsal on one GPU: per-rank host ids, socket transport
                from ntxent_amd.parallel.commstats import rccl_shared_gpu_env

                rccl_shared_gpu_env(rank)
            dist.init_process_group("nccl", device_id=dev, **kw)
        else:
            dist.init_process_group("gloo", **kw)
        world_seen = dist.get_world_size()
        if world_seen != world:
            raise SystemExit(f"process group has {world_seen} ranks, expected {world}")
    if on_gpu and a.compute_stream != "default":
        # A non-default compute stream: on the default stream the RCCL kernels of the overlapped
        # transfers shared a hardware queue with the GEMMs and ran only between them (1-2 % of a
        # transfer hidden under the forward GEMM vs 13-18 % on a new or high-priority stream,
        # tools/overlap_proxy.py, profiles/r3/overlap).
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1 if a.compute_stream == "high" else 0))
    if os.environ.get("NTXENT_BENCH_FAIL_RANK") == str(rank):  # fault injection (launcher tests)
        raise SystemExit(3)

    import ntxent_amd
    from ntxent_amd.ops.reference import flops_fwd_bwd
    from ntxent_amd.ops.reference import ntxent_loss as torch_ntxent
    from ntxent_amd.parallel import commstats, dist_ntxent_loss

    if a.impl == "torch" and world > 1:
        raise SystemExit("--impl torch is a single-GPU baseline")
    if a.impl == "native":
        if not on_gpu or a.graph or (world > 1 and a.negatives == "ring"):
            raise SystemExit("--impl native: GPU only, no --graph, negatives symmetric|allgather")
        if world > 1 and a.share_gpu:  # the Engine's own RcclComm on one GPU (socket transport)
            from ntxent_amd.parallel.commstats import rccl_shared_gpu_env

            rccl_shared_gpu_env(rank)
    R = 2 * a.batch

    def make_input(dtype):
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + rank)
        if a.data == "views":  # positive pairs share a random-normal basis: view = basis + 0.5 noise
            base = torch.randn(a.batch, a.dim, device=dev, generator=g)
            v1 = base + 0.5 * torch.randn(a.batch, a.dim, device=dev, generator=g)
            v2 = base + 0.5 * torch.randn(a.batch, a.dim, device=dev, generator=g)
            return torch.cat([v1, v2], 0).to(dtype).requires_grad_(True)
        return torch.randn(R, a.dim, device=dev, generator=g).to(dtype).requires_grad_(True)

    def make_step(h, compute):
        one = torch.ones((), device=dev, dtype=torch.float32 if h.dtype != torch.float64 else h.dtype)
        if a.impl == "native":  # the C++ Engine (+ its own RcclComm at N > 1), no autograd graph
            from ntxent_amd.parallel.native import NativeNTXent

            hd = h.detach()
            kw = dict(dtype=hd.dtype, compute=compute, negatives=a.negatives, keep_cos=not a.recompute)
            eng = (NativeNTXent.from_process_group(R, a.dim, a.temperature, **kw) if world > 1
                   else NativeNTXent(R, a.dim, a.temperature, **kw))
            make_step.engine_bytes = eng.device_bytes  # its own hipMalloc arena (not torch's allocator)
            return lambda: eng.step(hd)

        def step():
            if a.impl == "torch":
                loss = torch_ntxent(h, a.temperature)
            elif world > 1:
                loss = dist_ntxent_loss(h, a.temperature, compute=compute, keep_logits=not a.recompute,
                                        overlap=not a.no_overlap, negatives=a.negatives, impl=a.dist_impl)
            else:
                loss = ntxent_amd.ntxent_loss(h, a.temperature, compute=compute, keep_logits=not a.recompute)
            (gh,) = torch.autograd.grad(loss, h, grad_outputs=one.to(loss.dtype))
            return loss, gh
        return step

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    def timed(step, steps, warmup, per_step_events=True, comm=False):
        """warmup untimed steps, then exactly `steps` steps bracketed by barrier + synchronize
        on both sides; returns (total s, per-step ms list or None, comm ms per step or None).
        (Python's cyclic GC stays on: paused inside the bracket, the steps' autograd garbage piled up
        and the allocator's growth made them 0.46-0.47 ms instead of 0.406, profiles/r5/bench_gc.)"""
        for _ in range(warmup):
            loss, gh = step()
        sync()
        barrier()
        sync()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)] if (on_gpu and per_step_events) else None
        if comm:
            commstats.enable(True)
        t0 = time.perf_counter()
        if evs:
            evs[0].record()
        for i in range(steps):
            loss, gh = step()
            if evs:
                evs[i + 1].record()
        t_enq = time.perf_counter()  # host side done: the GPU may still be working
        sync()
        barrier()
        sync()
        dt = time.perf_counter() - t0
        timed.host_ms = (t_enq - t0) / steps * 1e3
        per = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)] if evs else None
        comm_ms = None
        if comm:
            c = commstats.collect()
            commstats.enable(False)
            comm_ms = {k: v / steps for k, v in c.items()}
        return dt, per, comm_ms, loss, gh

    dt_in = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    h = make_input(dt_in)
    step = make_step(h, a.compute)
    if a.graph:
        if world > 1 or not on_gpu:
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

        def step():  # noqa: F811 - every replay runs the complete forward + backward
            graph.replay()
            return g_loss, g_gh

    prewarm = max(0, a.prewarm_steps) if on_gpu else 0
    for _ in range(prewarm):  # same count on every rank (each step runs collectives)
        step()
    if on_gpu:
        torch.cuda.reset_peak_memory_stats(dev)
    # The timed region records no events at all, at every N (a timing event recorded between two
    # steps left a ~5-8 us bubble per step in the kernel trace, and the communication spans would
    # add several per step at N > 1): the per-step distribution and the per-rank communication
    # waits come from a separate pass right after it.
    dt_s, _, _, loss, gh = timed(step, a.steps, a.warmup, per_step_events=False, comm=False)
    host_ms = timed.host_ms  # host CPU time to enqueue one step (autograd + launches) in the timed run
    per_ms = comm_ms = None
    if on_gpu or world > 1:
        _, per_ms, comm_ms, _, _ = timed(step, min(a.steps, 20), 1, per_step_events=on_gpu, comm=world > 1)
    if a.host_profile and rank == 0:
        host_profile(step, a.host_profile, sync)
    elif a.host_profile:
        for _ in range(10):  # the same steps as rank 0 (they run collectives)
            step()
        sync()
    # torch allocator peak, plus the native Engine arenas (allocated once, outside torch)
    from ntxent_amd.parallel.engine_loss import cached_engine_bytes

    dist_impl = None
    if world > 1 and a.impl == "fused":
        dist_impl = "engine" if cached_engine_bytes() > 0 else "torch"
    peak_mb = ((torch.cuda.max_memory_allocated(dev) + getattr(make_step, "engine_bytes", 0)
                + cached_engine_bytes()) / 2**20 if on_gpu else None)
    lossv = float(loss.item())
    finite = bool(lossv == lossv and torch.isfinite(gh).all().item())

    def rank_max(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def rank_all(x: float):
        if world == 1:
            return [x]
        t = torch.zeros(world, dtype=torch.float64, device=dev)
        t[rank] = x
        dist.all_reduce(t)  # SUM of one-hot slots = gather
        return [float(v) for v in t.cpu()]

    dt_s = rank_max(dt_s)
    host_ms = rank_max(host_ms)
    ok = rank_max(0.0 if finite else 1.0) == 0.0
    ms = dt_s / a.steps * 1e3
    value = world * a.batch / (ms / 1e3)
    comm_total = sum(comm_ms.values()) if comm_ms else 0.0
    comm_all = rank_all(comm_total) if world > 1 else None
    peak_all = rank_all(peak_mb) if peak_mb is not None and world > 1 else None

    secondary = None
    want_fp32 = a.secondary_fp32 == "on" or (a.secondary_fp32 == "auto" and world == 1 and on_gpu
                                             and a.impl == "fused" and a.dtype != "fp32" and not a.graph)
    if want_fp32:
        del h, step, gh
        h32 = make_input(torch.float32)
        s32 = make_step(h32, "fp32")
        n32 = max(2, min(5, a.steps // 4))
        dt32, per32, _, _, _ = timed(s32, n32, 1)
        ms32 = rank_max(dt32) / n32 * 1e3
        secondary = {"dtype": "fp32", "mfma_dtype": "fp32 (exact, v_mfma_f32_16x16x4_f32)", "steps": n32,
                     "ms_per_step": round(ms32, 4), "value": round(world * a.batch / (ms32 / 1e3), 1)}
        del h32, s32

    tflops = flops_fwd_bwd(R, world * R, a.dim,
                           symmetric_global=world > 1 and a.negatives == "symmetric") / (ms / 1e3) / 1e12
    if rank == 0:
        if not ok:
            raise SystemExit("non-finite loss or gradient")
        mfma = mfma_dtypes(a, world, rank, dev) if on_gpu else {"forward": None, "backward": None}
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "world_size_seen": world_seen,
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
                "model": ("NT-Xent loss (SimCLR), torch CPU path (plumbing only)" if not on_gpu
                          else "NT-Xent loss (SimCLR), fused MFMA fwd+bwd" if a.impl == "fused"
                          else "NT-Xent loss (SimCLR), fused MFMA fwd+bwd, native C++ Engine" if a.impl == "native"
                          else "NT-Xent loss (SimCLR), unfused PyTorch baseline (hipBLASLt + eager)"),
                "global_batch": world * a.batch,
                "seq_len": None,
                "batch_per_gpu": a.batch,
                "dim": a.dim,
                "temperature": a.temperature,
                "compute": a.compute,
                "mfma_dtype_forward": mfma["forward"],
                "mfma_dtype_backward": mfma["backward"],
                "keep_logits": not a.recompute,
                "parallelism": f"dp{world}",
                "negatives": a.negatives if world > 1 else None,
                "dist_impl": dist_impl,
                "backend": backend if world > 1 else None,
                "hip_graph": bool(a.graph),
                "compute_stream": a.compute_stream if on_gpu else None,
                "device": a.device,
            },
            "prewarm_steps": prewarm,
            "prewarm_note": ("untimed steps before the warmup steps: the GPU clock ramps over the first "
                             "~60 steps after a cold start (profiles/r2/ramp); the timed region is the "
                             "steady state") if prewarm else None,
            "step_ms": _stats(per_ms) if per_ms else None,
            "step_ms_list": [round(x, 4) for x in per_ms] if per_ms else None,
            "step_ms_source": ("HIP events around each of %d steps, a separate pass after the timed region "
                               "(one untimed step first)" % min(a.steps, 20)) if per_ms else None,
            "host_enqueue_ms_per_step": round(host_ms, 4),
            "host_enqueue_note": ("host CPU time to issue one step (autograd graph + kernel launches) in the "
                                  "timed run, max over ranks; the GPU is the bottleneck while it is below "
                                  "ms_per_step"),
            "peak_hbm_mb": round(peak_mb, 1) if peak_mb is not None else None,
            "peak_hbm_mb_per_rank": [round(x, 1) for x in peak_all] if peak_all else None,
            "comm_wait_ms_per_step": {k: round(v, 4) for k, v in comm_ms.items()} if comm_ms else None,
            "comm_wait_ms_per_step_per_rank": [round(x, 4) for x in comm_all] if comm_all else None,
            "comm_wait_fraction_max": (round(max(comm_all) / ms, 4) if comm_all else None),
            "loss": lossv,
            "note": ("global-batch negatives: each rank's rows meet all N*B negatives, so per-GPU similarity "
                     "work grows linearly with N and the ideal whole-job samples/s is flat in N"
                     if world > 1 else None),
            "tflops_per_gpu_useful": round(tflops, 1),
            "secondary": secondary,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            Path(a.json_out).write_text(line + "\n")
    if world > 1:
        dist.barrier()
        from ntxent_amd.parallel.engine_loss import release_engines

        release_engines()
        dist.destroy_process_group()


def mfma_dtypes(a, world: int, rank: int, dev) -> dict:
    """The MFMA operand dtypes the forward and backward GEMMs of this configuration run."""
    from ntxent_amd.ops import _ext
    from ntxent_amd.ops.ntxent import resolve_compute

    dt_in = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    comp = resolve_compute(dt_in, False, a.compute)
    if a.impl == "torch":
        return {"forward": "hipBLASLt " + a.dtype, "backward": "hipBLASLt " + a.dtype}
    C = _ext.load()
    R = 2 * a.batch
    plan = C.get_plan(R, a.dim, world, rank, float(a.temperature), comp, dev.index)
    name = {"fp32": "fp32 (v_mfma_f32_16x16x4_f32)", "fp16": "fp16 (v_mfma_f32_16x16x32_f16)",
            "bf16": "bf16 (v_mfma_f32_16x16x32_bf16)", "fp8": "e4m3 (block-scaled v_mfma_scale_f32_*_f8f6f4)"}
    if plan.small:
        fwd = plan.compute_dtype
    elif comp == "fp8":
        fwd = "fp8"
    elif (world == 1 and not a.recompute and C.raw_forward_enabled() and a.dtype in ("bf16", "fp16")
          and comp in ("fp16", a.dtype) and R % 256 == 0 and a.dim % 64 == 0):
        fwd = a.dtype  # raw-operand forward: the input rows themselves are the MFMA operands
    else:
        fwd = plan.compute_dtype
    bwd = ("fp8" if comp == "fp8" and world == 1 and C.fp8_backward_enabled() and a.dim % 8 == 0 and not plan.small
           else plan.backward_dtype)
    return {"forward": name.get(fwd, fwd), "backward": name.get(bwd, bwd)}


def host_profile(step, path: str, sync) -> None:
    """cProfile of the host side of 10 steps (the GPU runs behind); top entries by own time."""
    import cProfile
    import io
    import pstats

    sync()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(10):
        step()
    pr.disable()
    t_enq = (time.perf_counter() - t0) / 10 * 1e3
    sync()
    buf = io.StringIO()
    st = pstats.Stats(pr, stream=buf)
    st.sort_stats("tottime").print_stats(40)
    buf2 = io.StringIO()
    pstats.Stats(pr, stream=buf2).sort_stats("cumulative").print_stats(40)
    Path(path).write_text(f"host enqueue under cProfile: {t_enq:.3f} ms/step (10 steps; profiling adds overhead)\n\n"
                          f"== by own time ==\n{buf.getvalue()}\n== by cumulative time ==\n{buf2.getvalue()}")


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        raise SystemExit(launch(a, argv))  # launcher: no GPU access in this process
    run_rank(a)


if __name__ == "__main__":
    main()
