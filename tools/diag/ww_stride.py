#!/usr/bin/env python3
"""wgrad4w per-K-tile time vs the operands' row stride: ONE 256 x 256 output tile (one
workgroup, so no bandwidth limit) over T rows, with rows packed (512 B apart) or strided
(a 256-column slice of a wider tensor), and with 16 / 64 workgroups for reference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    from apex_example_amd import _native
    dn = _native.require().dense
    T = 16384
    for lay in (0, 2):
        os.environ["APEX_AMD_W4W_LAYOUT"] = str(lay)
        for width in (256, 1024, 4096):
            big_a = torch.randn(T, width, device="cuda").to(torch.bfloat16)
            big_b = torch.randn(T, width, device="cuda").to(torch.bfloat16)
            dy, x = big_a[:, :256], big_b[:, :256]
            us = timeit(lambda: dn.wgrad4w(dy, x, 1, torch.float32))
            print("layout %d  row stride %5d B  1 workgroup, %d K-tiles: %8.1f us = %.2f us per K-tile"
                  % (lay, width * 2, T // 64, us, us / (T // 64)), flush=True)
        for (m, n, s) in ((1024, 1024, 1), (1024, 1024, 4), (4096, 1024, 4)):
            dy = torch.randn(T, m, device="cuda").to(torch.bfloat16)
            x = torch.randn(T, n, device="cuda").to(torch.bfloat16)
            us = timeit(lambda: dn.wgrad4w(dy, x, s, torch.float32))
            kt = T // s // 64
            print("layout %d  %d x %d, S=%d: %d workgroups x %d K-tiles: %8.1f us = %.2f us per K-tile"
                  % (lay, m, n, s, (m // 256) * (n // 256) * s, kt, us, us / kt), flush=True)


if __name__ == "__main__":
    main()
