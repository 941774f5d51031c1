#!/usr/bin/env python3
"""Is a diagonal forward tile (A and B the same 256 Zq rows) cheaper than an off-diagonal one?

Times the forward GEMM (fwd_stats_tiles: 2 persistent rounds, no kept cosines) on 512-tile lists
of the headline plan (B = 4096/view, d = 2048): all off-diagonal tiles, all diagonal tiles (the
32 repeated), and mixes with 32 diagonal tiles placed in one round. If the diagonal tiles' duplicate
line requests are merged in the L1, a diagonal tile costs less than an off-diagonal one, and the
16 remainder tiles could ride as third items on the CUs that hold a diagonal tile.
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402


def main():
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
    diag = t[t[:, 2] == 1]
    off = t[t[:, 2] != 1]
    print(f"tiles: {t.shape[0]} ({diag.shape[0]} diagonal)")
    lists = {
        "off512": torch.cat([off, off[:512 - off.shape[0]]]),
        "diag512": diag.repeat(16, 1),
        "off480+diag32_round2": torch.cat([off[:256], off[256:480], diag]),
        "off496+diag16": torch.cat([off, diag[:16]]),
    }
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, lst in lists.items():
        td = lst.contiguous().to(dev)
        for _ in range(3):
            C.fwd_stats_tiles(zq, zq, 0, td, plan, part)
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            ev[0].record()
            C.fwd_stats_tiles(zq, zq, 0, td, plan, part)
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
        ts.sort()
        print(f"{name:24s} n={lst.shape[0]} median {ts[len(ts) // 2]:.1f} us  min {ts[0]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
