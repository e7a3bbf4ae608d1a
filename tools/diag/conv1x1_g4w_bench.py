"""Stride-1 1x1 conv forwards of ResNet-50 (bs 256) with Cout % 256 == 0: the own implicit
GEMM (conv_tap_k) vs gemm4w vs hipBLASLt (torch.mm), plain and with the BN-statistics
epilogue; us per call (median of 20)."""
import sys

import torch

sys.path.insert(0, ".")
from apex_example_amd import _native  # noqa: E402

C = _native.require()
dev = "cuda"
cl = torch.channels_last


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000)
    ts.sort()
    return ts[len(ts) // 2]


print("| Cin -> Cout @ hw | own fwd | gemm4w fwd | hipBLASLt mm | own +stats | gemm4w +stats |")
print("|---|---|---|---|---|---|")
for ci, co, hw in [(64, 256, 56), (128, 512, 28), (256, 1024, 14), (512, 2048, 7),
                   (1024, 256, 14), (2048, 512, 7), (512, 256, 28), (256, 256, 56)]:
    n = 256
    x = torch.randn(n, ci, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(co, ci, 1, 1, device=dev) / ci ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=cl)
    sh = torch.zeros(co, device=dev)
    x2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
    w2 = w.reshape(co, ci).t()
    r = []
    for mode in (0, 1):
        C.conv.set_1x1_gemm4w(mode)
        r.append(timeit(lambda: C.conv.conv_fwd(x, w, 1)))
    r.append(timeit(lambda: torch.mm(x2, w2)))
    for mode in (0, 1):
        C.conv.set_1x1_gemm4w(mode)
        r.append(timeit(lambda: C.conv.conv_fwd_stats(x, w, 1, sh)))
    print("| %d -> %d @ %d | %s |" % (ci, co, hw, " | ".join("%.1f" % t for t in r)), flush=True)
C.conv.set_1x1_gemm4w(1)
