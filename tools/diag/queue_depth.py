#!/usr/bin/env python3
"""How far can the host run ahead of the GPU?  Launch many GPU-bound kernels
(torch.cuda._sleep) without syncing and record host time per launch: when the
host blocks after N launches, N is the effective queue depth."""
import time

import torch

torch.cuda.init()
torch.cuda._sleep(1000)
torch.cuda.synchronize()
for cycles in (200_000, 50_000):
    ts = []
    t0 = time.perf_counter()
    for i in range(3000):
        torch.cuda._sleep(cycles)
        ts.append(time.perf_counter() - t0)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    per = t_all / 3000 * 1e6
    # first launch index where host time exceeds 2x the pure-launch rate
    block = next((i for i in range(1, 3000) if ts[i] - ts[i - 1] > 0.5 * per * 1e-6), None)
    print("sleep %d cycles: GPU %.1f us/kernel, host loop %.1f ms of %.1f ms total; "
          "host first waited at launch %s" % (cycles, per, t_host * 1e3, t_all * 1e3, block))
