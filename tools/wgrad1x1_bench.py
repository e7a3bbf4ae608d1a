#!/usr/bin/env python3
"""1x1 weight gradients of ResNet-50 (batch 256): the default split-K hipBLASLt path
(`ops.conv.wgrad_1x1`, fp32 partials + one native slab reduction) at its own split count
and at forced larger splits, against the own MFMA tap kernel (`conv.conv_wgrad`,
ksize 1).  Correctness against an fp32 reference first, then interleaved timing rounds
in one process (so every row compares on the same box and clocks)."""
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


# (cin, cout, hw, stride, calls per ResNet-50 step)
SHAPES = [(64, 64, 56, 1, 1), (64, 256, 56, 1, 4), (256, 64, 56, 1, 2), (256, 128, 56, 1, 1),
          (128, 512, 28, 1, 4), (512, 128, 28, 1, 3), (512, 256, 28, 1, 1),
          (256, 1024, 14, 1, 6), (1024, 256, 14, 1, 5), (1024, 512, 14, 1, 1),
          (512, 2048, 7, 1, 3), (2048, 512, 7, 1, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--splits", default="256,512")
    ap.add_argument("--dense", action="store_true",
                    help="the transformer dense-layer weight gradients instead (T tokens)")
    ap.add_argument("--w4w", action="store_true",
                    help="1x1 shapes: add the wgrad4w kernel where both channel counts are "
                         "multiples of 256")
    ap.add_argument("--shapes", default="",
                    help="comma-separated indices into SHAPES (default: all)")
    ap.add_argument("--own-only", action="store_true",
                    help="--dense: only the default split and the own kernel")
    ap.add_argument("--tuned", default="",
                    help="read-only TunableOp table tuning/<name>.csv (as bench.py uses)")
    ap.add_argument("--tune-file", default="",
                    help="TunableOp ONLINE tuning into this file (every GEMM shape searched)")
    args = ap.parse_args()
    from apex_example_amd import _native
    from apex_example_amd.ops import conv as C

    cv = _native.require().conv
    dev = "cuda"
    if args.tuned:
        from apex_example_amd.utils.gemm_tuning import use_tuned_gemms
        print("tuned table:", use_tuned_gemms(args.tuned))
    if args.tune_file:
        t = torch.cuda.tunable
        t.enable(True)
        t.tuning_enable(True)
        t.set_filename(args.tune_file, insert_device_ordinal=False)
    splits = [int(s) for s in args.splits.split(",") if s]

    def forced(dyr, xr, s):
        m, co = dyr.shape
        ci = xr.shape[1]
        a = dyr.view(s, m // s, co).transpose(1, 2)
        b = xr.view(s, m // s, ci)
        part = torch.bmm(a, b, out_dtype=torch.float32)
        return cv.splitk_reduce(part, torch.bfloat16, None, True)

    if args.dense:
        return dense(args, cv, forced)
    rows = []
    pick = [int(i) for i in args.shapes.split(",") if i] or range(len(SHAPES))
    for (ci, co, hw, st, calls) in [SHAPES[i] for i in pick]:
        n = args.batch
        g = torch.Generator(device=dev).manual_seed(ci * 7 + co)
        x = torch.randn(n, ci, hw, hw, device=dev, generator=g).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, co, hw, hw, device=dev, generator=g).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        xr, dyr = C._as_rows(x), C._as_rows(dy)
        m = xr.shape[0]
        ref = (dyr.float().t() @ xr.float())
        scale = float(ref.abs().max())
        cands = {"splitk(S=%d)" % C._split_k(m): lambda: C.wgrad_1x1(dyr, xr, torch.bfloat16)}
        for s in splits:
            if m % s == 0 and s != C._split_k(m):
                cands["splitk(S=%d)" % s] = (lambda s=s: forced(dyr, xr, s))
        cands["own tap"] = lambda: cv.conv_wgrad(dy, x, torch.bfloat16, 0, 1, 1)
        if args.w4w:
            # the dense weight-gradient GEMM (csrc/hip/wgrad4w.hip) at split counts that
            # put 64-512 workgroups on the 256 x 256 output tiles
            dn = _native_dense()
            tiles = (co // 256) * (ci // 256) if co % 256 == 0 and ci % 256 == 0 else 0
            ok = [s for s in range(1, 1025) if tiles and 64 <= tiles * s <= 640 and
                  m % (64 * s) == 0 and dn.wgrad4w_ok(dyr, xr, s)]
            for target in (128, 256, 384, 512):
                if ok:
                    s = min(ok, key=lambda s: abs(tiles * s - target))
                    cands["w4w(S=%d)" % s] = (lambda s=s: dn.wgrad4w(
                        dyr, xr, s, torch.bfloat16))
        for name, fn in cands.items():
            out = fn().float().reshape(co, ci)
            err = float((out - ref).abs().max()) / scale
            print("check %d->%d @%d %s: rel err %.2e" % (ci, co, hw, name, err), flush=True)
            assert err < 2e-2, (name, err)
        times = {k: [] for k in cands}
        for _ in range(args.rounds):
            for k, fn in cands.items():
                times[k].append(timeit(fn))
        best = {k: min(v) for k, v in times.items()}
        gf = 2.0 * m * ci * co / 1e9
        rows.append((ci, co, hw, calls, gf, best))
        print("| 1x1 %d->%d @%d | %d | %.1f | %s |" % (
            ci, co, hw, calls, gf, " | ".join("%s %.1f us (%.0f TF)" % (k, t, gf / t * 1e3)
                                              for k, t in best.items())), flush=True)
    tot_def = sum(r[3] * list(r[5].values())[0] for r in rows)
    tot_best = sum(r[3] * min(r[5].values()) for r in rows)
    print("weighted per step: default %.0f us, best-of %.0f us" % (tot_def, tot_best))


DENSE = [("bert ffn-in", 16384, 4096, 1024), ("bert ffn-out", 16384, 1024, 4096),
         ("bert qkv", 16384, 3072, 1024), ("bert attn-out", 16384, 1024, 1024),
         ("gpt2 ffn-in", 8192, 4096, 1024), ("gpt2 ffn-out", 8192, 1024, 4096),
         ("gpt2 qkv", 8192, 3072, 1024), ("gpt2 attn-out", 8192, 1024, 1024)]


def _native_dense():
    from apex_example_amd import _native
    return _native.require().dense


def dense(args, cv, forced):
    """dW[o, i] = dY^T X over T tokens: the default split (fused_dense._splitk_chunks)
    against other split counts and the unsplit GEMM (bf16 out)."""
    from apex_example_amd import fused_dense as FD
    dev = "cuda"
    for (name, T, o, i) in DENSE:
        g = torch.Generator(device=dev).manual_seed(T + o + i)
        dy = torch.randn(T, o, device=dev, generator=g).to(torch.bfloat16)
        x = torch.randn(T, i, device=dev, generator=g).to(torch.bfloat16)
        ref = dy.float().t() @ x.float()
        scale = float(ref.abs().max())
        s0 = FD._splitk_chunks(T, o, i, torch.bfloat16, torch.bfloat16)
        cands = {"default(S=%d)" % s0: lambda: FD._wgrad(dy, x, torch.bfloat16)}
        for s in (1, 2, 4, 8, 16):
            if s != s0 and T % s == 0 and not args.own_only:
                cands["S=%d" % s] = ((lambda s=s: forced(dy, x, s)) if s > 1
                                     else (lambda: dy.t() @ x))
        dn = _native_dense()
        for s in (2, 4, 8):
            if dn.wgrad4w_ok(dy, x, s):
                cands["wgrad4w S=%d" % s] = (lambda s=s: dn.wgrad4w(dy, x, s, torch.bfloat16))
        for k, fn in cands.items():
            err = float((fn().float().reshape(o, i) - ref).abs().max()) / scale
            assert err < 2e-2, (name, k, err)
        times = {k: [] for k in cands}
        for _ in range(args.rounds):
            for k, fn in cands.items():
                times[k].append(timeit(fn))
        gf = 2.0 * T * o * i / 1e9
        print("| %s | %d x %d x %d | %s |" % (name, o, i, T, " | ".join(
            "%s %.1f us (%.0f TF)" % (k, min(v), gf / min(v) * 1e3) for k, v in times.items())),
            flush=True)


if __name__ == "__main__":
    main()
