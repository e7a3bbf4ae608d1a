#!/usr/bin/env python3
"""Stride-2 conv data gradients (parity-class kernels) of ResNet-50, with the classes in
dispatch order (APEX_AMD_DGRAD_LPT=0) vs heaviest first (=1), same process, results
bitwise equal."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
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

    cv = _native.require().conv
    cl = torch.channels_last
    N = 256
    print("| stride-2 dgrad | dispatch order | heaviest first | equal |")
    print("|---|---|---|---|")
    for (c, hw, k) in [(128, 56, 3), (256, 28, 3), (512, 14, 3), (256, 56, 1), (512, 28, 1),
                       (1024, 14, 1)]:
        co = c if k == 3 else 2 * c
        g = torch.Generator(device="cuda").manual_seed(c + hw)
        dy = torch.randn(N, co, hw // 2, hw // 2, device="cuda", generator=g).to(
            torch.bfloat16).to(memory_format=cl)
        w = (torch.randn(c, co, k, k, device="cuda", generator=g) * 0.03).to(
            torch.bfloat16).to(memory_format=cl)
        fn = lambda: cv.conv_dgrad_s2(dy, w, hw, hw)
        res = {}
        outs = {}
        for v in ("0", "1"):
            os.environ["APEX_AMD_DGRAD_LPT"] = v
            outs[v] = fn().clone()
        for _ in range(3):
            for v in ("0", "1"):
                os.environ["APEX_AMD_DGRAD_LPT"] = v
                res.setdefault(v, []).append(timeit(fn))
        print("| %dx%d %d->%d @%d | %.1f us | %.1f us | %s |" % (
            k, k, co, c, hw, min(res["0"]), min(res["1"]), torch.equal(outs["0"], outs["1"])),
            flush=True)


if __name__ == "__main__":
    main()
