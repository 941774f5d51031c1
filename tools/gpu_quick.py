"""Quick GPU sanity: run each kernel path on a few shapes and print errors vs the oracle."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import ntxent_amd
from ntxent_amd.ops import reference as R

def one(rows, dim, dtype, compute, keep=True, T=0.07):
    g = torch.Generator().manual_seed(rows * 7 + dim)
    n = rows // 2
    b = torch.randn(n, dim, generator=g, dtype=torch.float64)
    h64 = torch.cat([b + 0.3 * torch.randn(n, dim, generator=g, dtype=torch.float64),
                     b + 0.3 * torch.randn(n, dim, generator=g, dtype=torch.float64)])
    x = h64.to(dtype).cuda().requires_grad_(True)
    loss = ntxent_amd.ntxent_loss(x, T, compute=compute, keep_logits=keep)
    (gr,) = torch.autograd.grad(loss, x)
    torch.cuda.synchronize()
    hr = x.detach().double().cpu().requires_grad_(True)
    lr = R.ntxent_loss(hr, T)
    (gref,) = torch.autograd.grad(lr, hr)
    err = (gr.double().cpu() - gref).abs().max().item() / gref.abs().max().item()
    print(f"rows={rows:6d} dim={dim:5d} in={str(dtype):15s} comp={compute:5s} keep={keep}: "
          f"loss={loss.item():.6f} ref={lr.item():.6f} dloss={abs(loss.item()-lr.item()):.2e} grad_rel={err:.2e}", flush=True)

print(torch.cuda.get_device_properties(0))
for (rows, dim) in [(64, 128), (34, 100), (600, 200), (1024, 512)]:
    for comp in ["fp32", "fp16", "bf16"]:
        one(rows, dim, torch.float32, comp)
one(1024, 512, torch.float32, "fp16", keep=False)
one(2048, 256, torch.bfloat16, "auto")
