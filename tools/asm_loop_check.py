#!/usr/bin/env python3
"""Spill / drain check of the GEMM kernels' main loops from the device assembly.

A scratch reload inside the MFMA main loop comes with an `s_waitcnt vmcnt(0)` (the reload is a
vector-memory load behind the in-flight LDS-DMA), which drains the operand prefetch every K-step:
the round-4 fp8 dZ ran at 2.3x its round-3 time that way (profiles/r5/fp8_dz). For every kernel
whose name matches, prints the span of MFMA instructions, scratch accesses and vmcnt(0) waits in it.

  hipcc --offload-arch=gfx950 -std=c++17 -Iinclude -O3 -S --cuda-device-only \\
      kernels/ntxent_kernels.hip -o /tmp/k.s
  python tools/asm_loop_check.py /tmp/k.s [name-regex]

(The span runs from the first to the last MFMA in the text, so it can include a persistent
kernel's once-per-item code: the per-tile-max forwards (FX = 0, tau < ~0.024) reload two
hand-over pointers there, once per work item.)
"""
import re
import sys


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"sim_gemm_kernel|diag_up_kernel")
    lines = open(path).read().split("\n")
    bad = 0
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if not m or not pat.search(m.group(1)):
            continue
        end = next(k for k in range(i, len(lines)) if lines[k].startswith(".Lfunc_end"))
        body = lines[i:end]
        mf = [n for n, x in enumerate(body) if "v_mfma" in x]
        if not mf:
            continue
        lo, hi = mf[0], mf[-1]
        sc = [n for n in range(lo, hi) if "scratch_" in body[n]]
        vm = [n for n in range(lo, hi) if "vmcnt(0)" in body[n]]
        bad += bool(sc)
        print(f"{m.group(1)[:90]}: mfma span {hi - lo} lines, {len(mf)} mfma, scratch in span {len(sc)}, "
              f"vmcnt(0) in span {len(vm)}")
    print(f"{bad} kernel(s) with scratch accesses between their first and last MFMA")


if __name__ == "__main__":
    main()
