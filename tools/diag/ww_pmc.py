#!/usr/bin/env python3
"""Run the BERT FFN weight gradient (dW[4096, 1024] over 16384 tokens) many times through
the own wgrad4w kernel (both LDS layouts) and the hipBLASLt split-K batched GEMM, for
rocprofv3 --pmc passes (tools/diag/run_pmc.sh tools/diag/ww_pmc.py tools/diag/g4w_pmc.txt)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--t", type=int, default=16384)
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--splits", type=int, default=4)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from apex_example_amd import _native

    dn = _native.require().dense
    g = torch.Generator(device="cuda").manual_seed(0)
    dy = torch.randn(a.t, a.m, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(a.t, a.n, device="cuda", generator=g).to(torch.bfloat16)
    s = a.splits
    for _ in range(a.iters):
        dn.wgrad4w(dy, x, s, torch.bfloat16)
        torch.bmm(dy.view(s, a.t // s, a.m).transpose(1, 2), x.view(s, a.t // s, a.n),
                  out_dtype=torch.float32)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
