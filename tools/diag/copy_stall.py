"""Does a small async copy between two kernels stall the GPU queue?  Times 20 iterations
of (matmul, [copy], matmul) with the host far ahead, per copy kind."""
import time

import torch

dev = "cuda"
x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
hp = torch.zeros(512, dtype=torch.float32, pin_memory=True)
hq = torch.zeros(512, dtype=torch.float32)           # pageable
d = torch.zeros(512, device=dev)


def run(kind, n=20):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        y = x @ x
        if kind == "h2d_pinned":
            d.copy_(hp, non_blocking=True)
        elif kind == "d2h_pinned":
            hp.copy_(d, non_blocking=True)
        elif kind == "h2d_pageable":
            d.copy_(hq, non_blocking=True)
        elif kind == "kernel":
            d.add_(1.0)
        y = x @ x
    b.record()
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / n, (time.perf_counter() - t0) * 1e3


for _ in range(2):
    for kind in ("none", "kernel", "h2d_pinned", "d2h_pinned", "h2d_pageable"):
        us, wait_ms = run(kind)
        print("%-13s %8.1f us / iteration   (host waited %.1f ms at the end)" % (kind, us, wait_ms),
              flush=True)
