"""Practical HBM bandwidth on the box (torch copy_ / fill_ / sum, hipEvent timing): the ceiling
the memory-bound passes (prep, LSE + transpose, coefficient pass) are compared against."""
import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


for mib in (32, 64, 128, 512):
    n = mib * 2 ** 20 // 2
    a = torch.empty(n, dtype=torch.float16, device="cuda").normal_()
    b = torch.empty_like(a)
    big = torch.empty(2 ** 30, dtype=torch.uint8, device="cuda")  # 1 GiB: evict MALL between reps

    def cp():
        b.copy_(a)

    t_cp = timeit(cp)
    t_fill = timeit(lambda: b.fill_(1.0))
    t_sum = timeit(lambda: a.sum())
    print(f"{mib:4d} MiB: copy {t_cp:7.1f} us = {2 * mib * 2**20 / t_cp / 1e6:5.2f} TB/s (r+w) | "
          f"fill {t_fill:7.1f} us = {mib * 2**20 / t_fill / 1e6:5.2f} TB/s | "
          f"sum {t_sum:7.1f} us = {mib * 2**20 / t_sum / 1e6:5.2f} TB/s", flush=True)
    del big
