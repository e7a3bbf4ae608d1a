#!/usr/bin/env python3
"""Every ResNet-50 convolution (bs 256, 224x224, channels-last bf16) in every direction:
the path the model runs (own MFMA kernels / hipBLASLt, exactly the ops/conv.py dispatch)
against the library alternatives (MIOpen through F.conv2d / convolution_backward, and
hipBLASLt through torch.mm for the 1x1 shapes), on random data, one process.

    python tools/conv_table.py [--iters 20] [--json out.json] [--only 3x3]

Per row: GFLOP, microseconds, TFLOP/s, % of the 2.5 PF dense bf16 peak, the library
times, the winner, and a numerics check of our output against the fp32 reference of the
same op.  The footer weights every row by its calls per training step (the model's
layer counts), so the table doubles as the standalone conv budget of one step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TF = 2500.0
N = 256


def timeit(fn, iters=20, warmup=5):
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


# (kind, cin, cout, H_in, stride, calls per step): ResNet-50 v1.5 (stride on the 3x3)
LAYERS = [
    ("3x3", 64, 64, 56, 1, 3), ("3x3", 128, 128, 28, 1, 3), ("3x3", 256, 256, 14, 1, 5),
    ("3x3", 512, 512, 7, 1, 2),
    ("3x3", 128, 128, 56, 2, 1), ("3x3", 256, 256, 28, 2, 1), ("3x3", 512, 512, 14, 2, 1),
    ("1x1", 64, 64, 56, 1, 1), ("1x1", 64, 256, 56, 1, 4), ("1x1", 256, 64, 56, 1, 2),
    ("1x1", 256, 128, 56, 1, 1), ("1x1", 128, 512, 28, 1, 4), ("1x1", 512, 128, 28, 1, 3),
    ("1x1", 512, 256, 28, 1, 1), ("1x1", 256, 1024, 14, 1, 6), ("1x1", 1024, 256, 14, 1, 5),
    ("1x1", 1024, 512, 14, 1, 1), ("1x1", 512, 2048, 7, 1, 3), ("1x1", 2048, 512, 7, 1, 2),
    ("1x1", 256, 512, 56, 2, 1), ("1x1", 512, 1024, 28, 2, 1), ("1x1", 1024, 2048, 14, 2, 1),
    ("stem", 3, 64, 224, 2, 1),
]


def rows_for(kind, ci, co, H, stride, iters, check):
    from apex_example_amd import _native
    from apex_example_amd.ops import conv as C

    cv = _native.require().conv
    dev = "cuda"
    k = {"3x3": 3, "1x1": 1, "stem": 7}[kind]
    pad = k // 2
    Ho = (H + 2 * pad - k) // stride + 1
    g = torch.Generator(device=dev).manual_seed(ci * 7 + co + H)
    x = cl(torch.randn(N, ci, H, H, device=dev, generator=g).to(torch.bfloat16))
    w = cl((torch.randn(co, ci, k, k, device=dev, generator=g) * (1.0 / (ci * k * k)) ** 0.5)
           .to(torch.bfloat16))
    dy = cl(torch.randn(N, co, Ho, Ho, device=dev, generator=g).to(torch.bfloat16))
    gf = 2.0 * N * Ho * Ho * ci * co * k * k / 1e9
    out = []

    def lib_conv():
        return F.conv2d(x, w, stride=stride, padding=pad)

    def lib_dgrad():
        return torch.ops.aten.convolution_backward(
            dy, x, w, None, (stride, stride), (pad, pad), (1, 1), False, (0, 0), 1,
            (True, False, False))[0]

    def lib_wgrad():
        return torch.ops.aten.convolution_backward(
            dy, x, w, None, (stride, stride), (pad, pad), (1, 1), False, (0, 0), 1,
            (False, True, False))[1]

    if kind == "stem":
        xp = cv.stem_pad(x)
        wp = C._pack_stem_weight(w)
        ours = {"fwd": lambda: cv.stem_fwd(xp, wp), "wgrad": lambda: cv.stem_wgrad(xp, dy)}
        libs = {"fwd": {"miopen": lib_conv}, "wgrad": {"miopen": lib_wgrad}}
        refs = {"fwd": lambda: F.conv2d(x.float(), w.float(), stride=2, padding=3),
                "wgrad": None}
        outs = {"fwd": lambda: ours["fwd"](), "wgrad": None}
    elif kind == "3x3":
        wr = C._rot_weight(w)
        ours = {"fwd": lambda: cv.conv_fwd(x, w, stride),
                "dgrad": (lambda: cv.conv_fwd(dy, wr, 1)) if stride == 1 else
                         (lambda: cv.conv_dgrad_s2(dy, wr, H, H)),
                "wgrad": lambda: cv.conv_wgrad(dy, x, torch.bfloat16,
                                               C._wgrad3_algo(x, w, stride), stride)}
        libs = {"fwd": {"miopen": lib_conv}, "dgrad": {"miopen": lib_dgrad},
                "wgrad": {"miopen": lib_wgrad}}
        if C._wgrad3_algo(x, w, stride) != 0:  # the per-tap kernel it replaced
            libs["wgrad"]["per-tap"] = lambda: cv.conv_wgrad(dy, x, torch.bfloat16, 0, stride)
        refs = {"fwd": lambda: F.conv2d(x.float(), w.float(), stride=stride, padding=1),
                "dgrad": None, "wgrad": None}
        outs = {"fwd": lambda: ours["fwd"]()}
    else:  # 1x1
        M = N * Ho * Ho
        xr = C._as_rows(x[:, :, ::stride, ::stride].contiguous(memory_format=torch.channels_last)) \
            if stride == 2 else C._as_rows(x)
        dyr = C._as_rows(dy)
        w2 = w.reshape(co, ci)
        if stride == 1:
            ours = {"fwd": lambda: C._conv1x1_fwd(x, w),
                    "dgrad": lambda: C._conv1x1_dgrad(dy, w, x.shape),
                    "wgrad": lambda: C.wgrad_1x1(dyr, xr, torch.bfloat16)}
        else:
            wt = C._transpose_1x1(w)
            ours = {"fwd": lambda: cv.conv_fwd(x, w, 2),
                    "dgrad": lambda: cv.conv_dgrad_s2(dy, wt, H, H),
                    "wgrad": lambda: cv.conv_wgrad(dy, x, torch.bfloat16, 0, 2, 1)}
        libs = {"fwd": {"miopen": lib_conv, "hipblaslt": lambda: torch.mm(xr, w2.t())},
                "dgrad": {"miopen": lib_dgrad, "hipblaslt": lambda: torch.mm(dyr, w2)},
                "wgrad": {"miopen": lib_wgrad, "hipblaslt": lambda: torch.mm(dyr.t(), xr)}}
        refs = {"fwd": lambda: F.conv2d(x.float(), w.float(), stride=stride)}
        outs = {"fwd": lambda: ours["fwd"]()}
    for d, fn in ours.items():
        t = timeit(fn, iters)
        lt = {name: timeit(f, iters) for name, f in libs[d].items()}
        best_lib = min(lt.values())
        err = None
        if check and refs.get(d) is not None and outs.get(d) is not None:
            r = refs[d]()
            o = outs[d]().float()
            err = float((o - r).abs().max() / r.abs().max())
        out.append({
            "layer": "%s %d->%d @%d s%d" % (kind, ci, co, H, stride), "dir": d,
            "gflop": round(gf, 2), "us": round(t, 1), "tflops": round(gf / t * 1e3, 1),
            "pct_peak": round(gf / t * 1e3 / PEAK_TF * 100, 1),
            "lib_us": {k2: round(v, 1) for k2, v in lt.items()},
            "winner": "ours" if t <= best_lib else min(lt, key=lt.get),
            "rel_err": err,
        })
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="3x3 | 1x1 | stem")
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = False
    rows = []
    print("| layer | calls/step | dir | GFLOP | ours us | TF/s | % peak | MIOpen us | "
          "hipBLASLt us | other | winner | rel err |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    tot = {"ours": 0.0, "best": 0.0}
    for (kind, ci, co, H, s, calls) in LAYERS:
        if a.only and kind != a.only:
            continue
        for r in rows_for(kind, ci, co, H, s, a.iters, not a.no_check):
            r["calls"] = calls
            rows.append(r)
            lib = r["lib_us"]
            tot["ours"] += calls * r["us"]
            tot["best"] += calls * min([r["us"]] + list(lib.values()))
            other = ", ".join("%s %s" % (k2, v) for k2, v in lib.items()
                              if k2 not in ("miopen", "hipblaslt")) or "-"
            print("| %s | %d | %s | %.1f | %.1f | %.0f | %.1f | %s | %s | %s | %s | %s |" % (
                r["layer"], calls, r["dir"], r["gflop"], r["us"], r["tflops"], r["pct_peak"],
                lib.get("miopen", "-"), lib.get("hipblaslt", "-"), other, r["winner"],
                "%.1e" % r["rel_err"] if r["rel_err"] is not None else "-"), flush=True)
    print("\nweighted per step (calls x us): ours %.0f us, best-of(ours, libraries) %.0f us" % (
        tot["ours"], tot["best"]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"rows": rows, "total_us": tot}, f, indent=1)


if __name__ == "__main__":
    main()
