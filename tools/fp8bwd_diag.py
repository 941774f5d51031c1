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
    emulate(C, h, a, g8, g16)


def emulate(C, h, a, g8, g16):
    """torch emulation from the same plan's stage ops: the fp16 coefficient tiles of the fp8 forward
    (coef), reassembled, against e4m3 copies of C (per-row power-of-two scale from the row's
    actual max) and of 256 z; both through the same normalisation backward. Says what e4m3 operands
    cost by themselves, next to what the kernels' two backwards differ by."""
    plan = C.get_plan(a.rows, a.dim, 1, 0, a.T, "fp8", 0)
    zq, inv, ypos, zq8 = C.prep(h, plan)
    part, sc = C.fwd_stats(zq8, zq8, plan, True)
    lse2 = torch.empty((plan.rows_pad,), dtype=torch.float32, device="cuda")
    cpos = torch.empty_like(lse2)
    C.lse(part, ypos, lse2, cpos, plan)
    cb = C.coef(sc, lse2, cpos, plan)
    torch.cuda.synchronize()
    rt, ct, R, d = plan.row_tiles, plan.col_tiles, a.rows, a.dim
    Cf = cb.view(rt, ct, 256, 256).permute(0, 2, 1, 3).reshape(rt * 256, ct * 256)[:R, :R].float()
    z = zq[:R, :d].float()
    n = R // 2
    pos = (torch.arange(R, device="cuda") + n) % R
    ar = torch.arange(R, device="cuda")
    cp = Cf[ar, pos].clone()
    alpha = 1.0 / (R * a.T)

    def dh(dz):
        dz = dz * alpha
        return inv[:R, None] * (dz - z * (z * dz).sum(1, keepdim=True))

    d16 = dh(Cf @ z)
    Cn = Cf.clone()
    Cn[ar, pos] = 0.0
    rmax = Cn.abs().amax(1, keepdim=True).clamp_min(1e-30)
    e = torch.floor(torch.log2(448.0 / rmax))
    Cq = (Cn * 2.0 ** e).clamp(-448, 448).to(torch.float8_e4m3fn).float() / 2.0 ** e
    Zq = (256 * z).to(torch.float8_e4m3fn).float() / 256
    d8 = dh(Cq @ Zq + cp[:, None] * z[pos])
    s = d16.abs().max().item()
    print(f"emulated: max|dh(e4m3 C, e4m3 z) - dh(fp16 C)| / max = {(d8 - d16).abs().max().item() / s:.3e}; "
          f"e4m3 C only {(dh(Cq @ z + cp[:, None] * z[pos]) - d16).abs().max().item() / s:.3e}; "
          f"e4m3 z only {(dh(Cf @ Zq - cp[:, None] * Zq[pos] + cp[:, None] * z[pos]) - d16).abs().max().item() / s:.3e}")
    sk = g16.abs().max().item()
    print(f"kernel fp16 backward vs emulated fp16: {(g16 - d16).abs().max().item() / sk:.3e}; "
          f"kernel fp8 backward vs emulated fp16: {(g8 - d16).abs().max().item() / sk:.3e}; "
          f"vs emulated e4m3: {(g8 - d8).abs().max().item() / sk:.3e}")
    print(f"C: positive |C_ip| median {cp.abs().median().item():.3e}; negatives row max median {rmax.median().item():.3e}; "
          f"negatives row sum median {Cn.sum(1).median().item():.3e}")


if __name__ == "__main__":
    main()
