#!/usr/bin/env python3
"""Python test/benchmark harness — the working counterpart of the reference's python/test.py.

Reference behaviour (python/test.py:57-209) and what changes here:
  * stability sweep, scales {1e-5, 1, 1e5} x T {0.01, 0.07, 1.0} (:57-79): kept, and each
    point is also checked against the fp64 oracle (loss and gradient), not only for NaN/Inf;
  * perf sweep B in {32..512} x D in {64..512}, fp32 and "AMP" (:81-130, :141-158): kept; the
    reference's AMP was a no-op around a custom op, here mixed precision is the real fp16-MFMA
    path (use_mixed_precision=True); forward AND forward+backward are timed with HIP events;
  * GPUMemoryTracker (:25-40) per config, including the peak of each fwd+bwd;
  * result dump (:185-208) crashed on ``Path.ctime`` and tuple JSON keys: here keys are
    strings "B=..,d=..,dtype=..,world=1" and files are timestamped.

  python bench/harness.py                     # stability + reference perf sweep
  python bench/harness.py --quick             # small sweep
  python bench/harness.py --only stability
"""
from __future__ import annotations

import argparse
import json
import logging
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import ntxent_amd  # noqa: E402
from ntxent_amd.ops import reference as R  # noqa: E402
from ntxent_amd.utils import GPUMemoryTracker, device_summary, summarize, time_fn  # noqa: E402

log = logging.getLogger("ntxent.harness")


def stability(device, T_grid=(0.01, 0.07, 1.0), scales=(1e-5, 1.0, 1e5), B=128, D=256):
    out = {}
    for s in scales:
        for T in T_grid:
            g = torch.Generator().manual_seed(0)
            z = torch.nn.functional.normalize(torch.randn(2 * B, D, generator=g), dim=1) * s
            x = z.to(device).requires_grad_(True)
            loss = ntxent_amd.ntxent_loss(x, T)
            (gr,) = torch.autograd.grad(loss, x)
            h = z.double().requires_grad_(True)
            lref = R.ntxent_loss(h, T)
            (gref,) = torch.autograd.grad(lref, h)
            finite = bool(torch.isfinite(loss).item() and torch.isfinite(gr).all().item())
            lerr = abs(loss.item() - lref.item()) / max(1.0, abs(lref.item()))
            gerr = ((gr.double().cpu() - gref).norm() / gref.norm().clamp_min(1e-300)).item()
            ok = finite and lerr < 1e-4 and gerr < 1e-3
            out[f"scale={s:g},T={T:g}"] = {"finite": finite, "loss": loss.item(), "loss_rel_err": lerr,
                                           "grad_rel_err": gerr, "pass": ok}
            log.info("stability scale=%g T=%g loss=%.6f rel_err=%.2e grad_err=%.2e %s", s, T, loss.item(), lerr, gerr,
                     "PASS" if ok else "FAIL")
    return out


def perf(device, batches, dims, modes, warmup, runs, T=0.07, tracker=None):
    out = {}
    for mode in modes:
        for B in batches:
            for D in dims:
                g = torch.Generator().manual_seed(B * 131 + D)
                dtype = torch.bfloat16 if mode == "bf16" else torch.float32
                z = torch.randn(2 * B, D, generator=g).to(device=device, dtype=dtype)
                mp = mode == "amp"
                x = z.clone().requires_grad_(True)

                def fwd():
                    with torch.no_grad():
                        ntxent_amd.ntxent_loss(z, T, use_mixed_precision=mp)

                def fwd_bwd():
                    loss = ntxent_amd.ntxent_loss(x, T, use_mixed_precision=mp)
                    torch.autograd.grad(loss, x)

                f = summarize(time_fn(fwd, runs, warmup))
                fb = summarize(time_fn(fwd_bwd, runs, warmup))
                peak_mb = 0.0
                if tracker is not None:
                    with tracker.region(f"B={B},d={D},{mode}"):
                        fwd_bwd()
                    peak_mb = tracker.records[-1]["region_peak_mb"]
                key = f"B={B},d={D},dtype={mode},world=1"
                out[key] = {"fwd_ms": f, "fwd_bwd_ms": fb, "samples_per_s": B / (fb["mean"] * 1e-3),
                            "peak_mb": peak_mb}
                log.info("%-36s fwd %.4f ms  fwd+bwd %.4f ms (min %.4f)  %.0f samples/s  peak %.1f MB", key, f["mean"],
                         fb["mean"], fb["min"], B / (fb["mean"] * 1e-3), peak_mb)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["stability", "perf"], default=None)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--runs", type=int, default=100)
    ap.add_argument("--out-dir", default=str(ROOT / "benchmark_results"))
    a = ap.parse_args()
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(message)s")
    if not torch.cuda.is_available():
        raise SystemExit("harness needs a GPU (MI355X)")
    device = torch.device("cuda", 0)
    info = device_summary(0)
    log.info("device %s", info)
    res = {"device": info, "timestamp": time.strftime("%Y-%m-%dT%H:%M:%S")}
    tracker = GPUMemoryTracker()
    if a.only in (None, "stability"):
        res["stability"] = stability(device)
    if a.only in (None, "perf"):
        if a.quick:
            batches, dims, warmup, runs = [32, 256], [64, 512], 3, 10
        else:  # python/test.py:141-142
            batches, dims, warmup, runs = [32, 64, 128, 256, 512], [64, 128, 256, 512], a.warmup, a.runs
        res["perf"] = perf(device, batches, dims, ["fp32", "amp", "bf16"], warmup, runs, tracker=tracker)
    out = Path(a.out_dir)
    out.mkdir(parents=True, exist_ok=True)
    stamp = time.strftime("%Y%m%d_%H%M%S")
    (out / f"results_{stamp}.json").write_text(json.dumps(res, indent=2))
    tracker.dump(out / f"memory_profile_{stamp}.json")
    log.info("wrote %s", out / f"results_{stamp}.json")
    bad = [k for k, v in res.get("stability", {}).items() if not v["pass"]]
    if bad:
        log.error("stability failures: %s", bad)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
