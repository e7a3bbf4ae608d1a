#!/usr/bin/env python3
"""BN NHWC passes on two ResNet-50 layer shapes, repeated, for rocprofv3 --pmc passes
(tools/diag/run_pmc.sh tools/diag/bn_pmc.py tools/diag/bn_pmc.txt): stats_k
(local_stats), reduce_k (reduce_grad, residual + ReLU), backward_k, apply_k."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from apex_example_amd import _native

    C_ = _native.require().bn
    for (n, c, h, w) in [(256, 256, 56, 56), (256, 64, 56, 56), (256, 1024, 14, 14)]:
        x = torch.randn(n, c, h, w, device="cuda", dtype=torch.bfloat16).to(
            memory_format=torch.channels_last)
        z, dy = torch.randn_like(x), torch.randn_like(x)
        wt, bs = torch.ones(c, device="cuda"), torch.zeros(c, device="cuda")
        mean, var = C_.local_stats(x)
        invstd = (var + 1e-5).rsqrt()
        for _ in range(10):
            C_.local_stats(x)
            s1, s2, _, _ = C_.reduce_grad(dy, x, mean, invstd, wt, bs, z, True, True)
            C_.backward_elemt(dy, x, mean, invstd, wt, bs, s1, s2, float(n * h * w), z, True, True)
            C_.apply(x, mean, invstd, wt, bs, z, True)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
