import torch, time
dev = torch.device("cuda", 0)
def bench(fn, it=30):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it): fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b) / it * 1e3
for dt in (torch.float16, torch.bfloat16):
    C = (torch.randn(8192, 8192, device=dev) * 1e-3).to(dt)
    Z = torch.randn(8192, 2048, device=dev).to(dt)
    ZT = Z.t().contiguous()
    us = bench(lambda: torch.matmul(C, Z))
    print(f"{dt} dZ C[8192x8192] @ Z[8192x2048] -> {dt}: {us:.1f} us, {2*8192*8192*2048/us/1e6:.0f} TF/s")
    us = bench(lambda: torch.matmul(Z, ZT[:, :]))  # 8192x2048 @ 2048x8192 (fwd full square)
    print(f"{dt} fwd Z @ Z^T [8192x8192x2048]: {us:.1f} us, {2*8192*8192*2048/us/1e6:.0f} TF/s")
    try:
        out = torch.empty(8192, 2048, device=dev, dtype=torch.float32)
        us = bench(lambda: torch.mm(C, Z, out_dtype=torch.float32))
        print(f"{dt} dZ with out_dtype=fp32: {us:.1f} us, {2*8192*8192*2048/us/1e6:.0f} TF/s")
    except Exception as e:
        print("out_dtype not supported:", repr(e)[:120])
