#!/usr/bin/env python3
"""The one-wave-per-SIMD GEMM (csrc/hip/gemm4w.hip, 128 x 128 per wave) against
hipBLASLt (torch.mm, TunableOp off) on the transformer dense shapes and square GEMMs: a
correctness check against fp32 first, then interleaved timing rounds in one process on
random data."""
import argparse
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


SHAPES = [("bert ffn-in", 16384, 4096, 1024), ("bert ffn-out", 16384, 1024, 4096),
          ("bert qkv", 16384, 3072, 1024), ("bert attn-out", 16384, 1024, 1024),
          ("gpt2 ffn-in", 8192, 4096, 1024), ("gpt2 ffn-out", 8192, 1024, 4096),
          ("square 4096", 4096, 4096, 4096), ("square 8192", 8192, 8192, 8192)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    from apex_example_amd import _native

    dn = _native.require().dense
    dev = "cuda"

    # correctness vs fp32 (ragged M, odd K-tile counts, fp16), every variant
    for (m, n, k, dt) in [(256, 256, 64, torch.bfloat16), (1000, 512, 192, torch.bfloat16),
                          (333, 1024, 1088, torch.bfloat16), (4096, 768, 1024, torch.float16),
                          (16384, 256, 128, torch.bfloat16)]:
        g = torch.Generator(device=dev).manual_seed(m + n + k)
        a = torch.randn(m, k, device=dev, generator=g).to(dt)
        b = torch.randn(n, k, device=dev, generator=g).to(dt)
        ref = a.float() @ b.float().t()
        c = dn.gemm4w(a, b)[0]
        err = float((c.float() - ref).abs().max() / ref.abs().max())
        print("check %d x %d x %d %s: max rel err %.2e" % (m, n, k, dt, err), flush=True)
        assert err < 1e-2, err
    shapes = SHAPES[:3] + SHAPES[-1:] if args.quick else SHAPES
    cols = ["gemm4w", "hipBLASLt"]
    print("\n| GEMM | M, N, K | " + " | ".join(cols) + " |")
    print("|---|---|" + "---|" * len(cols))
    for name, m, n, k in shapes:
        g = torch.Generator(device=dev).manual_seed(m + n + k)
        a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        b = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
        gf = 2.0 * m * n * k / 1e9
        fns = [lambda: dn.gemm4w(a, b), lambda: torch.mm(a, b.t())]
        ts = [[] for _ in fns]
        for _ in range(args.rounds):
            for i, fn in enumerate(fns):
                ts[i].append(timeit(fn))
        cells = ["%.1f us (%.0f TF)" % (min(t), gf / min(t) * 1e3) for t in ts]
        print("| %s | %d, %d, %d | %s |" % (name, m, n, k, " | ".join(cells)), flush=True)
    ffn_rows(dn, dev, args.rounds)


def ffn_rows(dn, dev, rounds):
    """The fused FFN epilogues against the unfused sequence they replace (BERT-large
    shapes: x [16384, 1024], W1 [4096, 1024], W2 [1024, 4096], tanh GELU)."""
    m, n, k = 16384, 4096, 1024
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(n, k, device=dev, generator=g) / 32).to(torch.bfloat16)
    b1 = (torch.randn(n, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    dy = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    w2t = (torch.randn(n, k, device=dev, generator=g) / 64).to(torch.bfloat16)  # W2^T
    w2 = w2t.t().contiguous()

    def unfused_fwd():
        pre = torch.addmm(b1, x, w1.t())
        return dn.gelu(pre, True), pre

    pre = unfused_fwd()[1]

    def unfused_bwd():
        dh = dy @ w2
        return dn.gelu_bwd_bias_grad(dh, pre, True, torch.bfloat16)

    rows = [("fwd: hipBLASLt addmm + GELU pass", unfused_fwd),
            ("fwd: gemm4w bias+GELU epilogue",
             lambda: dn.gemm4w(x, w1, 1, bias=b1, want_pre=True, tanh=True)),
            ("bwd: hipBLASLt mm + dGELU/bias-grad pass", unfused_bwd),
            ("bwd: gemm4w dGELU+colsum epilogue",
             lambda: dn.gemm4w(dy, w2t, 2, aux=pre, tanh=True, bias_grad_dtype=torch.bfloat16))]
    ts = [[] for _ in rows]
    for _ in range(rounds):
        for i, (_, fn) in enumerate(rows):
            ts[i].append(timeit(fn))
    print("\n| FFN part (BERT-large, tanh GELU) | us |")
    print("|---|---|")
    for (name, _), t in zip(rows, ts):
        print("| %s | %.1f |" % (name, min(t)), flush=True)


if __name__ == "__main__":
    main()
