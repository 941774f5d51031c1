#!/usr/bin/env python3
"""Kernel-trace overlap of the data-parallel step (verdict r4, item 1c).

Launches a W-rank ``bench.py`` job on ONE GPU (RCCL over its socket transport, every rank on
cuda:0) with each rank under its own ``rocprofv3 --kernel-trace`` (rocprofv3 is the program
each child starts; this launcher never touches the GPU), once per CU reserve
(``NTXENT_COMM_RESERVE_CUS``), then reads every rank's kernel trace and reports how much of
the RCCL kernel time falls inside the similarity-GEMM spans:

* ``own``: inside the same rank's ``sim_gemm`` kernels (what a real 8-GPU node overlaps: each
  GPU runs one rank);
* ``any``: inside any rank's ``sim_gemm`` kernels (on the shared GPU the other ranks' GEMMs also
  hold the CUs).

  python tools/overlap_trace.py run --out gpurun_out/ov --world 2 --reserves 0,8,16
  python tools/overlap_trace.py analyze gpurun_out/ov

The transfers ride loopback sockets here, so the RCCL kernels spend most of their time waiting
for the proxy thread: the numbers say whether the kernels CAN run beside the GEMMs (the CU
reserve and the compute stream's priority), not how long an xGMI transfer takes.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(a) -> int:
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    for res in [int(x) for x in a.reserves.split(",")]:
        port = _port()
        procs = []
        for r in range(a.world):
            env = dict(os.environ)
            env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.world), LOCAL_WORLD_SIZE=str(a.world),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NTXENT_COMM_RESERVE_CUS=str(res),
                       HSA_ENABLE_IPC_MODE_LEGACY="0")
            d = out / f"res{res}" / f"rank{r}"
            cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", str(d), "-o", "run", "--",
                   sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", str(a.world), "--backend", "nccl",
                   "--share-gpu", "--batch", str(a.batch), "--dim", str(a.dim), "--steps", str(a.steps),
                   "--warmup", "1", "--prewarm-steps", "2", "--secondary-fp32", "off",
                   "--negatives", a.negatives, "--timeout", str(a.timeout)]
            log = open(out / f"res{res}_rank{r}.log", "w")
            procs.append((subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT,
                                           start_new_session=True), log))
        deadline = time.time() + a.timeout
        bad = None
        while True:
            codes = [p.poll() for p, _ in procs]
            if any(c not in (None, 0) for c in codes):
                bad = f"reserve {res}: exit codes {codes}"
                break
            if all(c == 0 for c in codes):
                break
            if time.time() > deadline:
                bad = f"reserve {res}: timeout"
                break
            time.sleep(0.5)
        if bad:
            for p, _ in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
            print(bad, flush=True)
            return 1
        for _, log in procs:
            log.close()
        print(f"reserve {res}: done", flush=True)
    return 0


def _spans(path, pred):
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if pred(name):
                out.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    return out


def _union(sp):
    sp = sorted(sp)
    out = []
    for s, e in sp:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _inside(sp, union):
    """ns of the spans ``sp`` covered by the (sorted, disjoint) ``union``."""
    tot = 0
    import bisect

    starts = [u[0] for u in union]
    for s, e in sp:
        i = max(0, bisect.bisect_right(starts, s) - 1)
        while i < len(union) and union[i][0] < e:
            lo, hi = max(s, union[i][0]), min(e, union[i][1])
            if hi > lo:
                tot += hi - lo
            i += 1
    return tot


def analyze(a) -> int:
    root = Path(a.dir)
    is_gemm = lambda n: "sim_gemm" in n  # noqa: E731
    is_rccl = lambda n: "nccl" in n.lower() or "rccl" in n.lower()  # noqa: E731
    rows = []
    for resdir in sorted(root.glob("res*"), key=lambda p: int(p.name[3:]) if p.name[3:].isdigit() else -1):
        if not resdir.is_dir():
            continue
        traces = {}
        for rk in sorted(resdir.glob("rank*")):
            f = glob.glob(str(rk / "**" / "*kernel_trace.csv"), recursive=True)
            if f:
                traces[rk.name] = f[0]
        if not traces:
            continue
        gem = {k: _spans(v, is_gemm) for k, v in traces.items()}
        rcc = {k: _spans(v, is_rccl) for k, v in traces.items()}
        any_union = _union([s for v in gem.values() for s in v])
        for k in traces:
            tot = sum(e - s for s, e in rcc[k])
            gu = _union(gem[k])
            own = _inside(rcc[k], gu)
            anyg = _inside(rcc[k], any_union)
            gt = sum(e - s for s, e in gem[k])
            covered = _inside(gem[k], _union(rcc[k]))  # GEMM time with an own RCCL kernel running
            # RCCL kernels that START inside one of the rank's GEMMs: with the GEMM holding every CU
            # (reserve 0) a kernel queued behind it can only start when it ends
            starts = sum(1 for s, _ in rcc[k] if _inside([(s, s + 1)], gu))
            rows.append({"reserve_cus": int(resdir.name[3:]), "rank": k, "rccl_kernels": len(rcc[k]),
                         "rccl_us": round(tot / 1e3, 1), "gemm_us": round(gt / 1e3, 1),
                         "rccl_in_own_gemm_frac": round(own / tot, 3) if tot else None,
                         "rccl_in_any_gemm_frac": round(anyg / tot, 3) if tot else None,
                         "gemm_with_rccl_frac": round(covered / gt, 3) if gt else None,
                         "rccl_starts_inside_gemm": starts})
    print("| reserve CUs | rank | RCCL kernels | RCCL kernel us | own sim_gemm us | RCCL time in own GEMM spans | "
          "in any rank's GEMM spans | own GEMM time with an RCCL kernel running | RCCL kernels starting inside own GEMMs |")
    print("|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['reserve_cus']} | {r['rank']} | {r['rccl_kernels']} | {r['rccl_us']} | {r['gemm_us']} | "
              f"{r['rccl_in_own_gemm_frac']} | {r['rccl_in_any_gemm_frac']} | {r['gemm_with_rccl_frac']} | "
              f"{r['rccl_starts_inside_gemm']} |")
    if a.json:
        Path(a.json).write_text(json.dumps(rows, indent=1) + "\n")
    return 0


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--out", required=True)
    r.add_argument("--world", type=int, default=2)
    r.add_argument("--reserves", default="0,8,16")
    r.add_argument("--batch", type=int, default=4096)
    r.add_argument("--dim", type=int, default=2048)
    r.add_argument("--steps", type=int, default=3)
    r.add_argument("--negatives", default="symmetric", choices=["symmetric", "allgather"])
    r.add_argument("--timeout", type=float, default=240.0)
    z = sub.add_parser("analyze")
    z.add_argument("dir")
    z.add_argument("--json", default=None)
    a = ap.parse_args()
    sys.exit(run(a) if a.cmd == "run" else analyze(a))


if __name__ == "__main__":
    main()
