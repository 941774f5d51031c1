#!/usr/bin/env python3
"""Where does the opt-in fp8 backward's error sit? (verdict r4, item 7)

Runs the fp8-forward plan with the e4m3 backward and with the fp16 backward on the same inputs
(the same forward: equal losses), then reports the error of the e4m3 gradient against the fp16 one
per row: the worst rows, their positions (row tile, view, padding), and how the error is
distributed. An ideal e4m3 rounding of C and Z predicts ~1.5e-3 of max|g| at rows = 4096, d = 512,
T = 0.07 (numpy emulation of the kernel's scales, tools/README.md); round 4 measured 5e-2.

  python tools/fp8bwd_diag.py [--rows 4096 --dim 512 --T 0.07]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--T", type=float, default=0.07)
    ap.add_argument("--noise", type=float, default=0.3)
    a = ap.parse_args()
    import ntxent_amd
    from test_gpu_kernels import _inputs

    C = ntxent_amd.ops._ext.load(build_if_missing=False)
    _, h = _inputs(a.rows, a.dim, torch.bfloat16, seed=a.rows + a.dim, noise=a.noise)

    def grad(fp8_bwd):
        C.set_fp8_backward(fp8_bwd)
        try:
            x = h.clone().requires_grad_(True)
            loss = ntxent_amd.ntxent_loss(x, a.T, compute="fp8", keep_logits=True)
            (g,) = torch.autograd.grad(loss, x)
            torch.cuda.synchronize()
            return loss.item(), g.float()
        finally:
            C.set_fp8_backward(False)

    l8, g8 = grad(True)
    l16, g16 = grad(False)
    print(f"loss fp8-bwd {l8:.8f} fp16-bwd {l16:.8f}")
    scale = g16.abs().max().item()
    err = (g8 - g16).abs()
    row_err = err.max(1).values / scale
    print(f"max|g8-g16|/max|g16| = {row_err.max().item():.3e}; rows above 1e-2: {(row_err > 1e-2).sum().item()} "
          f"of {a.rows}; median row {row_err.median().item():.3e}; 99th pct {row_err.quantile(0.99).item():.3e}")
    top = torch.topk(row_err, 12)
    n = a.rows // 2
    for v, i in zip(top.values.tolist(), top.indices.tolist()):
        e_row = err[i]
        j = int(e_row.argmax())
        print(f"  row {i:5d} (tile {i // 256:3d}, view {i // n}, pair {(i + n) % a.rows:5d}) err {v:.3e} at col {j:4d}; "
              f"|g16| row max {g16[i].abs().max().item() / scale:.3e}; g8 {g8[i, j].item():+.4e} g16 {g16[i, j].item():+.4e}")
    col_err = err.max(0).values / scale
    print("worst columns (embedding dims):", torch.topk(col_err, 8).indices.tolist())
    # relative error of the row direction (what the optimiser sees)
    rel = ((g8 - g16).norm(dim=1) / g16.norm(dim=1).clamp_min(1e-30))
    print(f"per-row relative L2 error: median {rel.median().item():.3e}, max {rel.max().item():.3e} (row {int(rel.argmax())})")


if __name__ == "__main__":
    main()
