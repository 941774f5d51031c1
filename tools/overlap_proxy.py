#!/usr/bin/env python3
"""One-GPU proxy for comm/compute overlap on RCCL (no second GPU needed).

A world-1 RCCL process group runs a self send/recv batch (one grouped P2P, executed by an RCCL
device kernel on the communicator's stream, like a peer transfer over xGMI) while the forward
similarity GEMM runs on the compute stream with ``reserve_cus=n``. The persistent GEMM
holds every CU it is given for its whole duration (128 KiB LDS, the full register file), so
with n = 0 the RCCL kernel can only start when the GEMM ends; with n > 0 it runs on the
reserved CUs underneath the GEMM. For each n this prints the GEMM alone, the transfer alone,
and both launched together (makespan), in microseconds (median of --iters), so the default
reserve can be chosen from data. Run it under ``rocprofv3 --kernel-trace`` to see the RCCL
kernel's start/end inside the GEMM's span.

  python tools/overlap_proxy.py [--mib 256] [--reserves 0,4,8,16,32] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256, help="bytes moved by the self send/recv batch")
    ap.add_argument("--chunks", type=int, default=8, help="tensors in the batch")
    ap.add_argument("--reserves", default="0,4,8,16,32")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--gemm-stream", default="current", choices=["current", "new", "high"],
                    help="stream the GEMM runs on: the current (default) stream, a new pool stream, or a new "
                         "high-priority stream")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()

    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0,
                            device_id=torch.device("cuda", 0))
    from ntxent_amd.ops import _ext
    from ntxent_amd.parallel.symmetric import _p2p

    C = _ext.load()
    g = torch.Generator(device="cuda").manual_seed(0)
    h = torch.randn(a.rows, a.dim, device="cuda", generator=g).bfloat16()
    plan = C.get_plan(a.rows, a.dim, 1, 0, 0.07, "fp16", 0)
    zq, _, _, _ = C.prep(h, plan)
    n = a.mib * 1024 * 1024 // 4 // a.chunks
    src = [torch.ones(n, device="cuda") for _ in range(a.chunks)]
    dst = [torch.empty(n, device="cuda") for _ in range(a.chunks)]
    if a.gemm_stream == "current":
        comp = torch.cuda.current_stream()
    else:
        comp = torch.cuda.Stream(priority=-1 if a.gemm_stream == "high" else 0)
    torch.cuda.set_stream(comp)
    print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')} gemm stream={a.gemm_stream}", flush=True)

    reserve = [0]
    part = torch.empty((plan.col_tiles, plan.rows_pad, 2), dtype=torch.float32, device="cuda")

    def gemm():
        C.fwd_stats_range(zq, zq, plan, part, None, 0, plan.n_fwd_tiles, reserve_cus=reserve[0])

    def xfer():
        return _p2p([(t, 0) for t in src], [(t, 0) for t in dst], dist.group.WORLD)

    def timed(fn_gemm, fn_xfer):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(comp)
        works = fn_xfer() if fn_xfer else []
        if fn_gemm:
            fn_gemm()
        for w in works:
            w.wait()  # the compute stream waits for the transfer: e1 marks both done
        e1.record(comp)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3

    out = {"rows": a.rows, "dim": a.dim, "mib": a.mib, "gemm_stream": a.gemm_stream,
           "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "results": []}
    for _ in range(3):  # warm-up (plans, communicator, clocks)
        timed(gemm, xfer)
    for r in [int(x) for x in a.reserves.split(",")]:
        reserve[0] = r
        g_us = statistics.median(timed(gemm, None) for _ in range(a.iters))
        x_us = statistics.median(timed(None, xfer) for _ in range(a.iters))
        b_us = statistics.median(timed(gemm, xfer) for _ in range(a.iters))
        hidden = (g_us + x_us - b_us) / x_us if x_us > 0 else 0.0
        rec = {"reserve_cus": r, "gemm_us": round(g_us, 1), "xfer_us": round(x_us, 1), "both_us": round(b_us, 1),
               "xfer_hidden_frac": round(hidden, 3)}
        out["results"].append(rec)
        print(f"reserve={r:3d}  gemm={g_us:8.1f} us  xfer({a.mib} MiB)={x_us:8.1f} us  both={b_us:8.1f} us  "
              f"transfer hidden: {100 * hidden:5.1f} %", flush=True)
    assert all(torch.equal(d, s) for d, s in zip(dst, src))
    if a.json:
        Path(a.json).write_text(json.dumps(out, indent=1) + "\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
