#!/usr/bin/env python3
"""Run ONE stride-1 1x1 conv forward with the BN-statistics epilogue (the ResNet-50 channel-
expanding convs) many times, for rocprofv3 --pmc passes: --ci -> --co channels at --hw."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ci", type=int, default=512)
    ap.add_argument("--co", type=int, default=2048)
    ap.add_argument("--hw", type=int, default=7)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    from apex_example_amd import _native

    cv = _native.require().conv
    cl = torch.channels_last
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(256, a.ci, a.hw, a.hw, device="cuda", generator=g).to(torch.bfloat16).to(
        memory_format=cl)
    w = (torch.randn(a.co, a.ci, 1, 1, device="cuda", generator=g) * 0.03).to(torch.bfloat16).to(
        memory_format=cl)
    sh = torch.zeros(a.co, device="cuda")
    for _ in range(a.iters):
        cv.conv_fwd_stats(x, w, 1, sh)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
