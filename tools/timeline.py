#!/usr/bin/env python3
"""Kernel timeline of one training step from a rocprofv3 --kernel-trace CSV: per dispatch its
start offset from the step's first kernel, duration and the idle gap before it, for the last
complete step (the step = the repeating kernel sequence that starts with FIRST).

  python tools/timeline.py run_kernel_trace.csv [FIRST-kernel-substring] [--steps N]
"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"void |ntxent::dev::|\(.*", "", n)
    return n[:60]


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "prep"
    nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 1
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    if len(starts) < 2:
        sys.exit(f"fewer than 2 dispatches matching {first!r}")
    a, b = starts[-1 - nsteps], starts[-1]
    seg = rows[a:b]
    t0 = int(seg[0]["Start_Timestamp"])
    prev_end = None
    busy = 0
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        busy += e - s
        print(f"{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:7.1f} us  gap {gap:5.1f}  {short(r['Kernel_Name'])}")
        prev_end = e
    span = (int(rows[b]["Start_Timestamp"]) - t0) / 1e3
    print(f"step span {span:.1f} us over {nsteps} step(s), kernels busy {busy / 1e3:.1f} us, idle {span - busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
