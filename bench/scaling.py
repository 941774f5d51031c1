#!/usr/bin/env python3
"""Scaling driver: runs ``bench.py --gpus N`` for N = 1, 2, 4, 8 (one rank per GPU
over RCCL/xGMI, launched by bench.py itself) and writes one JSON document with the curve.

The reference promises MPI/NCCL scaling in its build (/root/reference/CMakeLists.txt:13-14,
41-47, 115-121) and measures nothing; its perf harness is python/test.py:81-130.

Two efficiencies are reported per N, because the headline metric is weak-scaled in the batch
but NOT in the work: with global-batch negatives every rank's rows meet all N*B negatives, so
the similarity work of the whole job grows as N^2 while the GPUs grow as N.

* ``samples_efficiency`` = samples/s(N) / (N * samples/s(1)): what a per-GPU-batch weak-scaling
  reading expects; its ideal for this loss is 1/N (samples/s stays flat).
* ``pair_efficiency`` = similarity-pairs/s(N) / (N * similarity-pairs/s(1)), with
  (2 N B)^2 pairs per step: the work-normalised efficiency, ideal 1.

  python bench/scaling.py                       # N in {1,2,4,8} up to the visible GPU count
  python bench/scaling.py --ns 1,2 --device cpu --batch 32 --dim 16   # plumbing on CPU (gloo)
  python bench/scaling.py --ns 1,2,4 --backend gloo --share-gpu      # multi-rank rehearsal on 1 GPU
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
BENCH = ROOT / "bench.py"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8", help="comma-separated GPU counts")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--negatives", default="symmetric", choices=["allgather", "symmetric", "ring"])
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--backend", default=None, choices=["nccl", "gloo"])
    ap.add_argument("--share-gpu", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--timeout", type=float, default=1500.0, help="per-N job timeout (s)")
    ap.add_argument("--out", default=None, help="write the JSON document here (default: stdout only)")
    return ap.parse_args(argv)


def visible_gpus() -> int:
    """GPU count without initialising the GPU in this process (device_count does not)."""
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:
        return 0


def run_one(a, n: int) -> dict:
    cmd = [sys.executable, str(BENCH), "--gpus", str(n), "--steps", str(a.steps), "--warmup", str(a.warmup),
           "--batch", str(a.batch), "--dim", str(a.dim), "--negatives", a.negatives, "--device", a.device,
           "--dtype", a.dtype, "--timeout", str(a.timeout), "--secondary-fp32", "off"]
    if a.backend:
        cmd += ["--backend", a.backend]
    if a.share_gpu:
        cmd += ["--share-gpu"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout + 60, env=env)
    wall = time.time() - t0
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or len(lines) != 1:
        raise RuntimeError(f"bench.py --gpus {n} failed (rc={r.returncode}):\n{r.stderr[-3000:]}")
    d = json.loads(lines[0])
    d["driver_wall_s"] = round(wall, 2)
    return d


def main(argv=None) -> int:
    a = parse(argv)
    ns = [int(x) for x in a.ns.split(",") if x.strip()]
    if a.device == "cuda" and not a.share_gpu:
        have = visible_gpus()
        skipped = [n for n in ns if n > have]
        ns = [n for n in ns if n <= have]
        if skipped:
            sys.stderr.write(f"scaling: skipping N={skipped} ({have} GPU(s) visible)\n")
    if not ns:
        raise SystemExit("scaling: no runnable GPU count")
    runs = {n: run_one(a, n) for n in ns}
    base = runs.get(1)
    curve = []
    for n in ns:
        d = runs[n]
        pairs = (2.0 * n * a.batch) ** 2 / (d["ms_per_step"] / 1e3)  # similarity pairs per second
        row = {"n_gpus": n, "value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"],
               "similarity_pairs_per_s": pairs, "comm_wait_fraction_max": d.get("comm_wait_fraction_max"),
               "peak_hbm_mb": d.get("peak_hbm_mb")}
        if base is not None:
            pairs1 = (2.0 * a.batch) ** 2 / (base["ms_per_step"] / 1e3)
            row["samples_efficiency"] = d["value"] / (n * base["value"])
            row["pair_efficiency"] = pairs / (n * pairs1)
        curve.append(row)
    doc = {"metric": runs[ns[0]]["metric"], "negatives": a.negatives, "batch_per_gpu": a.batch, "dim": a.dim,
           "dtype": a.dtype, "device": a.device, "backend": a.backend, "share_gpu": a.share_gpu,
           "curve": curve, "runs": {str(n): runs[n] for n in ns}}
    text = json.dumps(doc, indent=1)
    print(text)
    if a.out:
        Path(a.out).write_text(text + "\n")
    for row in curve:
        eff = (f"samples_eff={row['samples_efficiency']:.3f} pair_eff={row['pair_efficiency']:.3f}"
               if "pair_efficiency" in row else "")
        sys.stderr.write(f"N={row['n_gpus']}: {row['value']:.1f} {row['unit']} {row['ms_per_step']:.3f} ms/step {eff}\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
