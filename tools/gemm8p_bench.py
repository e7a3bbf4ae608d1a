#!/usr/bin/env python3
"""The own 8-phase MFMA GEMM (csrc/hip/gemm8p.hip) vs hipBLASLt (torch.mm on the same
operands, TunableOp tables off) on the transformer FFN shapes and square GEMMs, random
data, interleaved rounds in one process; plus the fused FFN epilogues vs GEMM + the
separate GELU / bias-gradient kernels they replace."""
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

    dn = _native.require().dense
    dev = "cuda"
    shapes = [("bert ffn-in", 16384, 4096, 1024), ("bert ffn-out", 16384, 1024, 4096),
              ("bert ffn dgrad (dh)", 16384, 4096, 1024), ("bert qkv", 16384, 3072, 1024),
              ("gpt2 ffn-in", 8192, 4096, 1024), ("square 4096", 4096, 4096, 4096),
              ("square 8192", 8192, 8192, 8192)]
    print("| GEMM | M, N, K | GFLOP | gemm8p | hipBLASLt (torch.mm) | max rel diff |")
    print("|---|---|---|---|---|---|")
    for name, m, n, k in shapes:
        g = torch.Generator(device=dev).manual_seed(m + n + k)
        a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        b = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
        gf = 2.0 * m * n * k / 1e9
        t8, tl = [], []
        for _ in range(3):
            t8.append(timeit(lambda: dn.gemm8p(a, b)))
            tl.append(timeit(lambda: torch.mm(a, b.t())))
        c8 = dn.gemm8p(a, b)[0].float()
        cl = torch.mm(a, b.t()).float()
        d = float((c8 - cl).abs().max() / cl.abs().max())
        t8, tl = min(t8), min(tl)
        print("| %s | %d, %d, %d | %.1f | %.1f us (%.0f TF) | %.1f us (%.0f TF) | %.1e |" % (
            name, m, n, k, gf, t8, gf / t8 * 1e3, tl, gf / tl * 1e3, d), flush=True)
    # fused FFN epilogues vs the unfused sequence
    m, n, k = 16384, 4096, 1024
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(n, k, device=dev) / 32).to(torch.bfloat16)
    b1 = torch.zeros(n, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w2t = (torch.randn(n, k, device=dev) / 64).to(torch.bfloat16)   # W2^T [4096, 1024]
    w2 = w2t.t().contiguous()

    def unfused_fwd():
        pre = torch.addmm(b1, x, w1.t())
        return dn.gelu(pre, True), pre

    pre = unfused_fwd()[1]

    def unfused_bwd():
        dh = dy @ w2
        return dn.gelu_bwd_bias_grad(dh, pre, True, torch.bfloat16)

    rows = [("FFN fwd: addmm + gelu", unfused_fwd),
            ("FFN fwd: gemm8p bias+gelu epilogue",
             lambda: dn.gemm8p(x, w1, 1, bias=b1, want_pre=True, tanh=True)),
            ("FFN bwd: mm + dgelu/bias-grad", unfused_bwd),
            ("FFN bwd: gemm8p dgelu+colsum epilogue",
             lambda: dn.gemm8p(dy, w2t, 2, aux=pre, tanh=True, bias_grad_dtype=torch.bfloat16))]
    print("\n| FFN step part (BERT-large shapes) | us |")
    print("|---|---|")
    for name, fn in rows:
        print("| %s | %.1f |" % (name, min(timeit(fn) for _ in range(3))), flush=True)


if __name__ == "__main__":
    main()
