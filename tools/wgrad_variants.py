#!/usr/bin/env python3
"""3x3 weight-gradient kernel variants (conv_wgrad `algo`: 0 = 64-deep K-tiles on a 2-deep
ring, 2 = 32-deep on a 4-deep ring, 3 = 64-deep on a 3-deep ring) on the ResNet-50 3x3
shapes, same process, interleaved rounds; results must match algo 0 to fp32 rounding.

    python tools/wgrad_variants.py [--algos 0 2 3] [--rounds 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TF = 2500.0


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--algos", nargs="+", type=int, default=[0, 2, 3])
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from apex_example_amd import _native

    cv = _native.require().conv
    cl = torch.channels_last
    N = 256
    cases = []
    for (c, hw, s) in [(128, 28, 1), (256, 14, 1), (512, 7, 1), (128, 56, 2), (256, 28, 2),
                       (512, 14, 2)]:
        g = torch.Generator(device="cuda").manual_seed(c + hw + s)
        x = torch.randn(N, c, hw, hw, device="cuda", generator=g).to(torch.bfloat16).to(
            memory_format=cl)
        ho = (hw - 1) // s + 1
        dy = torch.randn(N, c, ho, ho, device="cuda", generator=g).to(torch.bfloat16).to(
            memory_format=cl)
        gf = 2.0 * N * ho * ho * c * c * 9 / 1e9
        cases.append(("3x3 wgrad %d@%d s%d" % (c, hw, s), gf, dy, x, s))
    res = {}
    bad = []
    for name, gf, dy, x, s in cases:
        ref = cv.conv_wgrad(dy, x, torch.float32, a.algos[0], s).float()
        for al in a.algos[1:]:
            got = cv.conv_wgrad(dy, x, torch.float32, al, s).float()
            err = float((got - ref).abs().max() / (ref.abs().max() + 1e-30))
            if err > 1e-4:
                bad.append((name, al, err))
    for _ in range(a.rounds):
        for name, gf, dy, x, s in cases:
            for al in a.algos:
                t = timeit(lambda: cv.conv_wgrad(dy, x, torch.bfloat16, al, s))
                res.setdefault((name, al), []).append(t)
    print("| wgrad | GFLOP | " + " | ".join("algo %d" % al for al in a.algos) + " |")
    print("|---|---|" + "---|" * len(a.algos))
    for name, gf, *_ in cases:
        cells = []
        for al in a.algos:
            t = min(res[(name, al)])
            cells.append("%.1f us (%.0f TF)" % (t, gf / t * 1e3))
        print("| %s | %.1f | %s |" % (name, gf, " | ".join(cells)), flush=True)
    print("\nmismatches vs algo %d: %s" % (a.algos[0], bad if bad else "none"))


if __name__ == "__main__":
    main()
