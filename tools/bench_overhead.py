"""Where bench.py's timed region spends time beyond the kernels: host enqueue cost per step,
and wall time of K steps (barrier/synchronize bracketed) for several K (fixed vs per-step cost)."""
import sys, time
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

def step():
    loss = ntxent_amd.ntxent_loss(h, 0.07)
    (gh,) = torch.autograd.grad(loss, h, grad_outputs=one)
    return loss, gh

for _ in range(10):
    step()
torch.cuda.synchronize()
# host enqueue cost: steps issued back to back without waiting (GPU runs behind)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue 20 steps: host {1e3*(t1-t0)/20:.4f} ms/step, wall {1e3*(t2-t0)/20:.4f} ms/step", flush=True)
for K in (5, 20, 50, 100, 200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"K={K}: {1e3*dt/K:.4f} ms/step", flush=True)
t0 = time.perf_counter(); torch.cuda.synchronize(); print(f"idle sync {1e6*(time.perf_counter()-t0):.1f} us")
