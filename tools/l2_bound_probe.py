#!/usr/bin/env python3
"""Upper bound on what L2-resident operands would buy the GEMM main loop.

Times the forward GEMM (fwd_stats_tiles: 2 persistent rounds of 256 tiles, headline plan,
B = 4096/view, d = 2048) on two 512-tile lists with the same instruction stream:

  plan512  the plan's first 512 tiles (4 x 8 superblocks, ~79 % L2 hits: the misses are the
           first touch of each panel line by an XCD)
  same512  512 copies of tile (0, 1): every CU of an XCD streams the same two panels in near
           lockstep, so all but the first touch of a line is an L2 hit

  zero512  the plan's tiles on all-zero operands: same instructions and addresses, near-zero
           switching energy in the MFMAs, so a clock the chip holds down under load rises
           (MI355X_MICROARCH.md, DVFS give-back)

If same512 is much faster, the loop pays for the L2 misses' latency and a prefetch path that
does not take the CU's L1 request slots (e.g. another kernel's loads on the same XCD) could buy
the difference. If it is not, the L2 miss rate is not what holds the loop.

usage: tools/l2_bound_probe.py [--only plan512|same512|zero512] [--iters N]
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warm", type=int, default=400)
    args = ap.parse_args()
    from ntxent_amd.ops import _ext
    C = _ext.load(build_if_missing=False)
    dev = torch.device("cuda", 0)
    rows, dim = 8192, 2048
    plan = C.get_plan(rows, dim, 1, 0, 0.07, "fp16", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    h = torch.randn(rows, dim, device=dev, generator=g).to(torch.bfloat16)
    zq, inv, ypos, _ = C.prep(h, plan)
    part = torch.empty((plan.col_tiles, plan.rows_pad, 2), dtype=torch.float32, device=dev)
    t = plan.fwd_tiles.cpu()
    lists = {"plan512": t[:512].clone(), "same512": t[:1].repeat(512, 1), "zero512": t[:512].clone()}
    zq0 = torch.zeros_like(zq)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, lst in lists.items():
        if args.only and name != args.only:
            continue
        td = lst.contiguous().to(dev)
        op = zq0 if name == "zero512" else zq  # zero512: the plan's tiles on all-zero operands
        for _ in range(args.warm):  # back to back: the clock settles under sustained load
            C.fwd_stats_tiles(op, op, 0, td, plan, part)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.iters):  # batches of 50 back-to-back launches
            ev[0].record()
            for _ in range(50):
                C.fwd_stats_tiles(op, op, 0, td, plan, part)
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]) * 1e3 / 50)
        ts.sort()
        print(f"{name:8s} first tile {tuple(lst[0].tolist())} per launch: median {ts[len(ts) // 2]:.1f} us  "
              f"min {ts[0]:.1f} us (batches of 50 after {args.warm} warm launches)", flush=True)


if __name__ == "__main__":
    main()
