"""Time the 3x3 stride-1 forward on the ResNet-50 shapes (batch 256) with the halo kernel
(conv3h_k) on and off: plain forward, forward + BN statistics, forward + BN-backward
epilogue.  Prints a markdown table (us per call, median of 20 after warmup)."""
import sys

import torch

sys.path.insert(0, ".")
from apex_example_amd import _native  # noqa: E402

C = _native.require()
dev = torch.device("cuda", 0)
CL = torch.channels_last
SHAPES = [(256, 128, 28, 28, 128), (256, 256, 14, 14, 256), (256, 512, 7, 7, 512),
          (256, 64, 56, 56, 64)]


def bf(t):
    return t.to(torch.bfloat16).contiguous(memory_format=CL)


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


print("| shape (N,Cin,H,W,Cout) | op | per-tap us | halo auto us | halo auto, N tiles fastest us | halo 256-px tiles us | halo 64-wide us | TFLOP/s auto |")
print("|---|---|---|---|---|---|---|---|")
for (N, Ci, H, W, Co) in SHAPES:
    x = bf(torch.randn(N, Ci, H, W, device=dev))
    w = bf(torch.randn(Co, Ci, 3, 3, device=dev) / (Ci * 9) ** 0.5)
    xb = bf(torch.randn(N, Co, H, W, device=dev))
    mean = torch.zeros(Co, device=dev)
    inv = torch.ones(Co, device=dev)
    sh = torch.zeros(Co, device=dev)
    ops = {
        "fwd": lambda: C.conv.conv_fwd(x, w, 1),
        "fwd+stats": lambda: C.conv.conv_fwd_stats(x, w, 1, sh),
        "fwd+bnbwd": lambda: C.conv.conv_fwd_bnbwd(x, w, None, xb, None, mean, inv, None, None, 2),
    }
    flop = 2.0 * N * H * W * Co * Ci * 9
    for name, fn in ops.items():
        C.conv.set_halo(0)
        t0 = timeit(fn)
        C.conv.set_halo(1)
        t1 = timeit(fn)
        C.conv.set_halo_nfast(1)
        t4 = timeit(fn)
        C.conv.set_halo_nfast(0)
        C.conv.set_halo_mtile(256)
        t3 = timeit(fn)
        C.conv.set_halo_mtile(0)
        C.conv.set_halo(64)
        t2 = timeit(fn)
        print("| %s | %s | %.1f | %.1f | %.1f | %.1f | %.1f | %.0f |" % (
            (N, Ci, H, W, Co), name, t0, t1, t4, t3, t2, flop / t1 / 1e6), flush=True)
C.conv.set_halo(1)
