#!/usr/bin/env python3
"""Per-item phase times of the persistent GEMM from a timing build (NTXENT_TIMING=1, see
sim_gemm.h): for each work-item index, over all blocks, the time from item start to the main
loop's first K-step (prologue / first operands landed), the main loop, and the epilogue, in
shader-clock cycles (s_memtime) and in us at --ghz.

  tools/build_variant.sh timing -DNTXENT_TIMING=1
  NTXENT_TIMING_OUT=gpurun_out/t build/bin/ntxent_bench_timing --batch 4096 --dim 512 --iters 3
  python tools/gemm_timing.py gpurun_out/t/gemm_m0_e2_g256.bin [--ghz 2.1]
"""
import struct
import sys

import numpy as np


def main():
    path = sys.argv[1]
    ghz = float(sys.argv[sys.argv.index("--ghz") + 1]) if "--ghz" in sys.argv else 2.1
    raw = open(path, "rb").read()
    grid, items, marks = struct.unpack("iii", raw[:12])
    t = np.frombuffer(raw[12:], dtype=np.uint64).reshape(grid, items, marks).astype(np.int64)
    if "diag_up" in path:
        return diag_up(t[:, 0, :], grid, ghz, path)
    print(f"{path}: grid {grid}, {items} item slots; cycles (us at {ghz} GHz): mean / p10 / p90 / max over blocks")
    used = t[:, :, 3] > 0
    for it in range(items):
        m = used[:, it]
        if not m.any():
            break
        x = t[m, it]
        cols = {"to loop": x[:, 1] - x[:, 0], "loop": x[:, 2] - x[:, 1], "epilogue": x[:, 3] - x[:, 2],
                "item": x[:, 3] - x[:, 0]}
        if (x[:, 5] > 0).all():  # forward epilogue phases: pre (dequant / fixup), exp + row sums, barrier, merge
            cols.update({"e.pre": x[:, 4] - x[:, 2], "e.exp": x[:, 5] - x[:, 4], "e.bar": x[:, 6] - x[:, 5],
                         "e.merge": x[:, 3] - x[:, 6]})
        parts = []
        for k, v in cols.items():
            parts.append(f"{k} {v.mean():7.0f} ({v.mean() / ghz / 1e3:5.2f}) / {np.percentile(v, 10):6.0f} / "
                         f"{np.percentile(v, 90):6.0f} / {v.max():6.0f}")
        print(f"item {it} ({m.sum()} blocks): " + " | ".join(parts))
    # a block's whole span (its own clock): first item start to last epilogue end
    last = np.where(used, t[:, :, 3], 0).max(1)
    span = last - t[:, 0, 0]
    print(f"block span: mean {span.mean():.0f} cycles ({span.mean() / ghz / 1e3:.2f} us), max {span.max():.0f} "
          f"({span.max() / ghz / 1e3:.2f} us)")


def diag_up(x, grid, ghz, path):
    """diag_up_kernel marks: 0 start, 1 ring prologue issued, 2 K loop done, 3 K pieces merged
    (last piece only), 4 epilogue stores issued, 5 drained, 6 past the row-group ticket."""
    print(f"{path}: grid {grid}; ticks (us at {ghz} GHz): mean / p50 / p90 / max over the blocks that reach each mark")
    names = ["prologue", "K loop", "piece merge", "epilogue", "drain", "ticket"]
    for k, nm in enumerate(names):
        m = (x[:, k + 1] > 0) & (x[:, k] > 0)
        if not m.any():
            continue
        v = x[m, k + 1] - x[m, k]
        print(f"  {nm:12s} ({m.sum():4d} blocks): {v.mean():8.0f} ({v.mean() / ghz / 1e3:5.2f}) / {np.median(v):7.0f} / "
              f"{np.percentile(v, 90):7.0f} / {v.max():7.0f}")
    last = x.max(1)
    span = last - x[:, 0]
    print(f"  block span: mean {span.mean():.0f} ({span.mean() / ghz / 1e3:.2f} us), max {span.max():.0f}; "
          f"start spread (if clocks agree) {(x[:, 0].max() - x[:, 0].min()) / ghz / 1e3:.2f} us, "
          f"first start to last mark {(last.max() - x[:, 0].min()) / ghz / 1e3:.2f} us")


if __name__ == "__main__":
    main()
