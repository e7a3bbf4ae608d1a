#!/usr/bin/env python3
"""Stride-1 1x1 weight gradients of ResNet-50: the model's split-K hipBLASLt path
(ops/conv.py wgrad_1x1: bmm with fp32 partials + the two-stage slab reduction) vs the
own per-tap MFMA wgrad kernel (conv.conv_wgrad, ksize 1, algo 0), same process,
interleaved rounds; results must agree to fp32-accumulation rounding."""
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
    from apex_example_amd.ops import conv as C

    cv = _native.require().conv
    cl = torch.channels_last
    N = 256
    print("| 1x1 wgrad | GFLOP | split-K hipBLASLt (model) | own conv_wgrad | rel diff |")
    print("|---|---|---|---|---|")
    for (ci, co, hw) in [(64, 64, 56), (64, 256, 56), (256, 64, 56), (256, 128, 56),
                         (128, 512, 28), (512, 128, 28), (512, 256, 28), (256, 1024, 14),
                         (1024, 256, 14), (1024, 512, 14), (512, 2048, 7), (2048, 512, 7)]:
        g = torch.Generator(device="cuda").manual_seed(ci + co + hw)
        x = torch.randn(N, ci, hw, hw, device="cuda", generator=g).to(torch.bfloat16).to(
            memory_format=cl)
        dy = torch.randn(N, co, hw, hw, device="cuda", generator=g).to(torch.bfloat16).to(
            memory_format=cl)
        xr, dyr = C._as_rows(x), C._as_rows(dy)
        gf = 2.0 * N * hw * hw * ci * co / 1e9
        lib = lambda: C.wgrad_1x1(dyr, xr, torch.bfloat16)
        own = lambda: cv.conv_wgrad(dy, x, torch.bfloat16, 0, 1, 1)
        a = C.wgrad_1x1(dyr, xr, torch.float32).float()
        b = cv.conv_wgrad(dy, x, torch.float32, 0, 1, 1).float().reshape(a.shape)
        err = float((a - b).abs().max() / (a.abs().max() + 1e-30))
        t = {"lib": [], "own": []}
        for _ in range(3):
            t["lib"].append(timeit(lib))
            t["own"].append(timeit(own))
        tl, to = min(t["lib"]), min(t["own"])
        print("| %d->%d @%d | %.1f | %.1f us (%.0f TF) | %.1f us (%.0f TF) | %.1e |" % (
            ci, co, hw, gf, tl, gf / tl * 1e3, to, gf / to * 1e3, err), flush=True)


if __name__ == "__main__":
    main()
