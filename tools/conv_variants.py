#!/usr/bin/env python3
"""A/B of the implicit-GEMM conv tilings (csrc/hip/conv_igemm.hip launch_conv_tap,
APEX_AMD_CONV_BM) on every ResNet-50 shape that runs on the 128-multiple path: 3x3
forward (with the BN-statistics epilogue the model uses) and stride-1 data gradient,
stride-2 3x3 forward, own-kernel 1x1 forwards.  Interleaved rounds in one process,
random data; every variant's output must equal the default tiling's bitwise (same
per-element accumulation order).

    python tools/conv_variants.py [--variants default 256w8 ...] [--rounds 3]
"""
from __future__ import annotations

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


def cl(t):
    return t.to(memory_format=torch.channels_last)


def _select(v):
    """variant name -> env: 'default', an APEX_AMD_CONV_BM value, 'burst' / 'ileave' (the
    4-wave K loop with each tile's DMA as one burst / with read-ahead and DMA pieces
    between the MFMA rows, APEX_AMD_CONV_BURST=1 / 0)"""
    for k in ("APEX_AMD_CONV_BM", "APEX_AMD_CONV_BURST", "APEX_AMD_CONV_BK32",
              "APEX_AMD_CONV_BK32_64", "APEX_AMD_CONV_PIPE"):
        os.environ.pop(k, None)
    if v in ("pipe", "pipebk32"):  # the pipelined 4-deep-ring K loop (+ on every grid)
        os.environ["APEX_AMD_CONV_PIPE"] = "1"
        if v == "pipebk32":
            os.environ["APEX_AMD_CONV_BK32"] = "1"
    elif v in ("bk32on", "bk32off"):  # the auto BK = 32 choice forced on / off
        os.environ["APEX_AMD_CONV_BK32"] = "1" if v == "bk32on" else "0"
    elif v == "bk32w64":  # the 64-wide-tile BK = 32 form
        os.environ["APEX_AMD_CONV_BK32_64"] = "1"
    elif v in ("burst", "ileave"):
        os.environ["APEX_AMD_CONV_BURST"] = "1" if v == "burst" else "0"
    elif v != "default":
        os.environ["APEX_AMD_CONV_BM"] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", default=["default", "256w8", "256w8n2", "128w8"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from apex_example_amd import _native
    from apex_example_amd.ops.conv import _rot_weight

    cv = _native.require().conv
    dev = "cuda"
    N = 256
    cases = []
    for (c, hw, s) in [(64, 56, 1), (128, 28, 1), (256, 14, 1), (512, 7, 1), (128, 56, 2),
                       (256, 28, 2), (512, 14, 2)]:
        g = torch.Generator(device=dev).manual_seed(c + hw)
        x = cl(torch.randn(N, c, hw, hw, device=dev, generator=g).to(torch.bfloat16))
        w = cl((torch.randn(c, c, 3, 3, device=dev, generator=g) * 0.03).to(torch.bfloat16))
        ho = hw // s
        gf = 2.0 * N * ho * ho * c * c * 9 / 1e9
        shift = torch.zeros(c, device=dev)
        cases.append(("3x3 fwd+stats %d@%d s%d" % (c, hw, s), gf,
                      lambda x=x, w=w, s=s, sh=shift: cv.conv_fwd_stats(x, w, s, sh)[0]))
        if s == 1:
            dy = cl(torch.randn(N, c, hw, hw, device=dev, generator=g).to(torch.bfloat16))
            wr = _rot_weight(w)
            cases.append(("3x3 dgrad %d@%d" % (c, hw), gf,
                          lambda dy=dy, wr=wr: cv.conv_fwd(dy, wr, 1)))
    for (ci, co, hw) in [(256, 64, 56), (64, 256, 56), (256, 128, 56), (512, 128, 28), (512, 256, 28), (1024, 256, 14),
                         (1024, 512, 14), (512, 2048, 7), (2048, 512, 7), (128, 512, 28),
                         (256, 1024, 14)]:
        g = torch.Generator(device=dev).manual_seed(ci + co + hw)
        x = cl(torch.randn(N, ci, hw, hw, device=dev, generator=g).to(torch.bfloat16))
        w = cl((torch.randn(co, ci, 1, 1, device=dev, generator=g) * 0.03).to(torch.bfloat16))
        gf = 2.0 * N * hw * hw * ci * co / 1e9
        cases.append(("1x1 fwd %d->%d@%d" % (ci, co, hw), gf,
                      lambda x=x, w=w: cv.conv_fwd(x, w, 1)))
    res = {(n, v): [] for n, _, _ in cases for v in a.variants}
    bad = []
    for name, gf, fn in cases:
        _select("default")
        ref = fn().clone()
        for v in a.variants:
            _select(v)
            if not torch.equal(fn(), ref):
                bad.append((name, v))
    for _ in range(a.rounds):
        for name, gf, fn in cases:
            for v in a.variants:
                _select(v)
                res[(name, v)].append(timeit(fn, a.iters))
    _select("default")
    print("| conv | GFLOP | " + " | ".join(a.variants) + " |")
    print("|---|---|" + "---|" * len(a.variants))
    for name, gf, _ in cases:
        cells = []
        for v in a.variants:
            t = min(res[(name, v)])
            cells.append("%.1f us (%.0f TF, %.0f%%)" % (t, gf / t * 1e3, gf / t * 1e3 / PEAK_TF * 100))
        print("| %s | %.1f | %s |" % (name, gf, " | ".join(cells)), flush=True)
    print("\nmismatches vs default:", bad if bad else "none")


if __name__ == "__main__":
    main()
