#!/usr/bin/env python3
"""Run ONE implicit-GEMM conv shape many times (for rocprofv3 --pmc passes): 3x3 forward
of `--c` channels at `--hw`, or the 3x3 weight gradient (`--wgrad algo`)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c", type=int, default=128)
    ap.add_argument("--hw", type=int, default=28)
    ap.add_argument("--wgrad", type=int, default=-1)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--halo", type=int, default=1)
    a = ap.parse_args()
    from apex_example_amd import _native

    cv = _native.require().conv
    cv.set_halo(bool(a.halo))
    g = torch.Generator(device="cuda").manual_seed(0)
    cl = torch.channels_last
    x = torch.randn(256, a.c, a.hw, a.hw, device="cuda", generator=g).to(torch.bfloat16).to(
        memory_format=cl)
    w = (torch.randn(a.c, a.c, 3, 3, device="cuda", generator=g) * 0.03).to(torch.bfloat16).to(
        memory_format=cl)
    dy = torch.randn(256, a.c, a.hw, a.hw, device="cuda", generator=g).to(torch.bfloat16).to(
        memory_format=cl)
    for _ in range(a.iters):
        if a.wgrad >= 0:
            cv.conv_wgrad(dy, x, torch.bfloat16, a.wgrad, 1)
        else:
            cv.conv_fwd(x, w, 1)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
