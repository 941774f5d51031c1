#!/usr/bin/env python3
"""Does the coefficient pass read kept cosines from L2 when nothing streams between it and the
forward? Times the coefficient launch after the same forward in two orders (headline plan):

  A (default): prep -> forward -> LSE with the Z^T transpose blocks (64 MiB through the L2s) -> coef
  B:           prep -> transpose -> forward -> LSE alone -> coef

If B's coefficient pass is faster, the forward's last-round cosines survive in L2 across the
kernel boundaries, and a coefficient tile order matched to the forward's XCD assignment is worth
building.
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
    g = torch.Generator(device=dev).manual_seed(3)
    base = torch.randn(rows // 2, dim, device=dev, generator=g)
    h = torch.cat([base + 0.5 * torch.randn(rows // 2, dim, device=dev, generator=g),
                   base + 0.5 * torch.randn(rows // 2, dim, device=dev, generator=g)]).to(torch.bfloat16)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def run(order):
        zq, inv, ypos, _ = C.prep(h, plan)
        zqt = torch.empty((plan.dim_n, plan.ld_t), dtype=zq.dtype, device=dev)
        if order == "B":
            C.transpose(zq, plan, zqt)
        part, sc = C.fwd_stats(zq, zq, plan, True)
        lse2 = torch.empty((plan.rows_pad,), dtype=torch.float32, device=dev)
        cpos = torch.empty((plan.rows_pad,), dtype=torch.float32, device=dev)
        if order == "A":
            C.lse(part, ypos, lse2, cpos, plan, zq, zqt)
        else:
            C.lse(part, ypos, lse2, cpos, plan)
        ev[0].record()
        cb = C.coef(sc, lse2, cpos, plan)
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) * 1e3

    for order in ("A", "B", "A", "B"):
        for _ in range(3):
            run(order)
        ts = sorted(run(order) for _ in range(15))
        print(f"order {order}: coefficient pass median {ts[len(ts) // 2]:.1f} us, min {ts[0]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
