#!/usr/bin/env python3
"""Markdown summary of a tools/gpu_variants.sh run: per shape and variant, the native bench's
fwd+bwd ms (median of the 30 timed iterations' mean per round) and the per-kernel mean
microseconds under rocprofv3 --kernel-trace --stats, both rounds side by side, plus the
gradient-digest check (every variant must match the default build bit for bit).

usage: tools/summarize_variants.py gpurun_out/<tag> > profiles/r4/<tag>.md
"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path

KPAT = re.compile(r"sim_gemm|coef|diag_up|sk_|prep|lse_|dot_reduce")


def short(name):
    m = re.match(r"_ZN6ntxent3dev(\d+)", name)
    if m:  # mangled: length-prefixed base name, template ints as Li<n>E
        L = int(m.group(1))
        base = name[m.end():m.end() + L]
        ints = re.findall(r"Li(\d+)E", name[m.end() + L:])
        if base == "sim_gemm_kernel":
            return "gemm[" + {"0": "fwd", "1": "coef-rc", "2": "dZ"}.get(ints[0] if ints else "", "?") + "]"
        if base == "diag_up_kernel" and len(ints) > 1:
            return f"diag_up[ks{ints[1]}]"
        return base
    n = re.sub(r"^void |ntxent::dev::|\(.*$", "", name)
    m = re.match(r"(\w+)<(.*)>", n)
    if not m:
        return n
    args = [a.strip() for a in m.group(2).split(",")]
    base = m.group(1)
    if base == "sim_gemm_kernel":  # <T, MODE, ...>: MODE 0 forward, 2 dZ
        mode = {"0": "fwd", "1": "coef-rc", "2": "dZ"}.get(args[1], args[1]) if len(args) > 1 else "?"
        return f"gemm[{mode}]"
    return base


def fwdbwd(log):
    txt = log.read_text(errors="replace").splitlines()
    for i, ln in enumerate(txt):
        if "fwd+bwd" in ln and i + 1 < len(txt):
            cols = txt[i + 1].split("|")
            if len(cols) > 3:
                try:
                    return float(cols[3].split()[0])
                except (ValueError, IndexError):
                    pass
    return None


def main(d):
    d = Path(d)
    runs = defaultdict(dict)  # (shape, variant) -> round -> (fb, {kernel: us})
    order_v, order_s = [], []
    for sub in sorted(d.glob("r[0-9]_*")):
        if not sub.is_dir():
            continue
        rnd, shape, var = sub.name.split("_", 2)
        ks = next(iter(sub.rglob("*kernel_stats.csv")), None)
        if ks is None:
            continue
        kern = {}
        for row in csv.DictReader(open(ks)):
            if KPAT.search(row["Name"]):
                k = short(row["Name"])
                kern[k] = kern.get(k, 0.0) + float(row["AverageNs"]) / 1e3
        runs[(shape, var)][rnd] = (fwdbwd(Path(str(sub) + ".log")), kern)
        if var not in order_v:
            order_v.append(var)
        if shape not in order_s:
            order_s.append(shape)
    print(f"# Variant A/B: {d.name}\n")
    digs = {}
    for f in sorted(d.glob("dig_*.log")):
        _, shape, var = f.stem.split("_", 2)
        m = re.search(r"grad digest: (\S+)", f.read_text(errors="replace"))
        digs[(shape, var)] = m.group(1) if m else "?"
    if digs:
        print("Gradient digest (FNV-1a of dh) vs the default build: " + ", ".join(
            f"{s}/{v} {'=' if digs[(s, v)] == digs.get((s, 'base')) else 'DIFFERS'}"
            for (s, v) in sorted(digs) if v != "base") + "\n")
    for shape in order_s:
        kernels = []
        for v in order_v:
            for r in runs.get((shape, v), {}).values():
                for k in r[1]:
                    if k not in kernels:
                        kernels.append(k)
        print(f"## {shape}\n")
        print("| variant | round | fwd+bwd ms | " + " | ".join(kernels) + " |")
        print("|---|---|---|" + "---|" * len(kernels))
        for v in order_v:
            for rnd, (fb, kern) in sorted(runs.get((shape, v), {}).items()):
                cells = [f"{kern[k]:.1f}" if k in kern else "" for k in kernels]
                print(f"| {v} | {rnd} | {fb if fb is not None else ''} | " + " | ".join(cells) + " |")
        print()


if __name__ == "__main__":
    main(sys.argv[1])
