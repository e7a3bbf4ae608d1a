#!/usr/bin/env python3
"""Run ONE GEMM shape many times through gemm4w and torch.mm (hipBLASLt), for
rocprofv3 --pmc passes (tools/diag/run_pmc.sh tools/diag/g8_pmc.py tools/diag/g8_pmc.txt)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--kernels", default="4w,lt", help="gemm4w, hipBLASLt")
    a = ap.parse_args()
    from apex_example_amd import _native

    dn = _native.require().dense
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(a.m, a.k, device="cuda", generator=g).to(torch.bfloat16)
    w = torch.randn(a.n, a.k, device="cuda", generator=g).to(torch.bfloat16)
    ks = a.kernels.split(",")
    for _ in range(a.iters):
        if "4w" in ks:
            dn.gemm4w(x, w)
        if "lt" in ks:
            torch.mm(x, w.t())
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
