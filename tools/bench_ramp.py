"""Per-step GPU time (HIP events) of the headline step from a cold start: shows the clock ramp
that the driver's short warm-up (W = 5) leaves inside a K = 20 timed region."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import ntxent_amd

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1234)
base = torch.randn(4096, 2048, device=dev, generator=g)
h = torch.cat([base + 0.5 * torch.randn(4096, 2048, device=dev, generator=g),
               base + 0.5 * torch.randn(4096, 2048, device=dev, generator=g)]).to(torch.bfloat16).requires_grad_(True)
one = torch.ones((), device=dev)
N = 200
ev = [torch.cuda.Event(enable_timing=True) for _ in range(N + 1)]
ev[0].record()
for i in range(N):
    loss = ntxent_amd.ntxent_loss(h, 0.07)
    (gh,) = torch.autograd.grad(loss, h, grad_outputs=one)
    ev[i + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(N)]
for a in range(0, N, 10):
    blk = ms[a:a + 10]
    print(f"steps {a:3d}-{a + 9:3d}: mean {sum(blk) / len(blk):.4f} ms  min {min(blk):.4f}  max {max(blk):.4f}")
