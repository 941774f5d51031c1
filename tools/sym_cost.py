#!/usr/bin/env python3
"""Per-rank GPU work of the data-parallel modes at world size W, measured on ONE GPU.

Runs exactly the stage ops one rank of a W-GPU job enqueues (rank r's plan, global column
indices, gathered buffers filled locally instead of by RCCL) and times them with HIP events:

  allgather  prep + fwd over the whole row block + lse + coef + dZ (K = W*R) + norm_bwd
  symmetric  prep + fwd over the own triangle and the assigned cross tiles + lse + coef_sym
             + partner dZ contributions + own dZ contributions + received adds + norm_bwd

Communication is excluded (it runs on the RCCL stream beside these kernels); the numbers are
the compute floor of one rank's step at that W. Usage:
  python tools/sym_cost.py [--batch 4096 --dim 2048 --worlds 1,2,4,8 --iters 5]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--T", type=float, default=0.07)
    ap.add_argument("--modes", default="allgather,symmetric", help="subset of allgather,symmetric")
    a = ap.parse_args()

    from ntxent_amd.ops import _ext
    from ntxent_amd.parallel.symmetric import (sym_coef, sym_grad_slabs, sym_norm_bwd, sym_own_grad, sym_partner_grads,
                                               sym_tiles)

    C = _ext.load(build_if_missing=False)
    dev = torch.device("cuda", 0)
    R, d = 2 * a.batch, a.dim
    g = torch.Generator(device=dev).manual_seed(0)
    results = []
    for W in [int(x) for x in a.worlds.split(",")]:
        for r in sorted({0, W // 2}) if W > 1 else [0]:
            plan = C.get_plan(R, d, W, r, a.T, "fp16", 0)
            Rpad = plan.rows_pad
            cdt = torch.float16
            zq_all = torch.empty((W * Rpad, plan.ld_k), dtype=cdt, device=dev)
            zqt_all = torch.empty((W, plan.dim_n, plan.ld_t), dtype=cdt, device=dev)
            hs = []
            for q in range(W):
                h = torch.randn(R, d, device=dev, generator=g).to(torch.bfloat16)
                pq = C.get_plan(R, d, W, q, a.T, "fp16", 0)
                C.prep(h, pq, zq_all[q * Rpad:(q + 1) * Rpad])
                C.transpose(zq_all[q * Rpad:(q + 1) * Rpad], pq, zqt_all[q])
                hs.append(h)
            h = hs[r]
            go = torch.ones(1, device=dev)
            zq = zq_all[r * Rpad:(r + 1) * Rpad]

            def allgather_step():
                _, inv, ypos, _ = C.prep(h, plan, zq)
                C.transpose(zq, plan, zqt_all[r])
                part = torch.empty((plan.col_tiles, Rpad, 2), dtype=torch.float32, device=dev)
                sc = torch.empty((plan.n_fwd_tiles * 65536,), dtype=cdt, device=dev)
                C.fwd_stats_range(zq, zq_all, plan, part, sc, 0, plan.n_fwd_tiles)
                lse2 = torch.empty((W * Rpad,), dtype=torch.float32, device=dev)
                cpos = torch.empty((Rpad,), dtype=torch.float32, device=dev)
                C.lse(part, ypos, lse2, cpos, plan)
                cb = C.coef(sc, lse2, cpos, plan)
                del sc
                slabs = C.dz(cb, zqt_all, plan)
                return C.norm_bwd(slabs, h, inv, go, plan)

            tiles, nt = sym_tiles(C, plan, dev)

            def symmetric_step():
                _, inv, ypos, _ = C.prep(h, plan, zq)
                C.transpose(zq, plan, zqt_all[r])
                part = torch.empty((plan.col_tiles, Rpad, 2), dtype=torch.float32, device=dev)
                part_x = torch.empty_like(part)
                sc = torch.empty((nt * 65536,), dtype=cdt, device=dev)
                C.fwd_stats_sym(zq, zq_all, tiles, plan, part, part_x, sc, 0, nt)
                part.fill_(1.0)  # stands in for the received column partials (finite LSE inputs)
                lse2 = torch.zeros((W * Rpad,), dtype=torch.float32, device=dev)
                cpos = torch.empty((Rpad,), dtype=torch.float32, device=dev)
                C.lse(part, ypos, lse2, cpos, plan)
                cbuf, mbuf = sym_coef(C, plan, W, tiles, sc, lse2, cpos)
                del sc
                own, recv, views = sym_grad_slabs(plan, W, r, dev)
                outs = list(sym_partner_grads(C, plan, W, r, mbuf, zqt_all).values())
                sym_own_grad(C, plan, W, r, cbuf, zqt_all, own[0])
                for v, o in zip(views.values(), outs):  # stands in for the received contributions
                    if v.shape == o.shape:
                        v.copy_(o)
                return sym_norm_bwd(C, plan, own, recv, h, inv, go)

            row = {"W": W, "rank": r, "batch": a.batch, "dim": d}
            modes = [("allgather", allgather_step)] + ([("symmetric", symmetric_step)] if W > 1 else [])
            modes = [m for m in modes if m[0] in a.modes.split(",")]
            for name, fn in modes:
                for _ in range(2):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                e1.synchronize()
                row[name + "_ms"] = round(e0.elapsed_time(e1) / a.iters, 4)
            if "allgather_ms" in row and "symmetric_ms" in row:
                row["speedup"] = round(row["allgather_ms"] / row["symmetric_ms"], 3)
            print(json.dumps(row), flush=True)
            results.append(row)
            del zq_all, zqt_all, hs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
