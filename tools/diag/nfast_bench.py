"""conv_tap_k tile order A/B (conv.set_nfast): us per call (median of 20) of the ResNet-50
1x1 forwards with the BN-statistics epilogue and the stride-2 3x3 forward, per mode
(0 = M tiles fastest, 1 = N fastest on the 1x1 launches, 2 = N fastest everywhere)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402

from apex_example_amd import _native  # noqa: E402

C = _native.require()
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


print("| conv | mode 0 us | mode 1 us | mode 2 us |")
print("|---|---|---|---|")
for ci, co, hw, k, s in [(64, 256, 56, 1, 1), (128, 512, 28, 1, 1), (256, 1024, 14, 1, 1),
                         (512, 2048, 7, 1, 1), (1024, 256, 14, 1, 1), (2048, 512, 7, 1, 1),
                         (512, 128, 28, 1, 1), (256, 64, 56, 1, 1), (256, 512, 56, 1, 2),
                         (128, 128, 56, 3, 2), (256, 256, 28, 3, 2)]:
    x = torch.randn(256, ci, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(co, ci, k, k, device="cuda") / ci ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=cl)
    sh = torch.zeros(co, device="cuda")
    r = []
    for mode in (0, 1, 2):
        C.conv.set_nfast(mode)
        r.append(timeit(lambda: C.conv.conv_fwd_stats(x, w, s, sh)))
    print("| %dx%d %d -> %d @ %d s%d | %s |" % (k, k, ci, co, hw, s, " | ".join("%.1f" % t for t in r)),
          flush=True)
# 1x1 data gradients with the BN-backward epilogue (dgrad of a Co -> K conv: K -> Co)
for co, k, hw in [(256, 64, 56), (512, 128, 28), (1024, 256, 14), (2048, 512, 7), (256, 1024, 14),
                  (512, 2048, 7), (128, 512, 28), (64, 256, 56)]:
    dy = torch.randn(256, k, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    wt = (torch.randn(co, k, 1, 1, device="cuda") / k ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=cl)
    xb = torch.randn(256, co, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    mean, invstd = torch.zeros(co, device="cuda"), torch.ones(co, device="cuda")
    bw, bb = torch.ones(co, device="cuda"), torch.zeros(co, device="cuda")
    r = []
    for mode in (0, 1, 2):
        C.conv.set_nfast(mode)
        r.append(timeit(lambda: C.conv.conv_fwd_bnbwd(dy, wt, None, xb, None, mean, invstd, bw, bb, 2)))
    print("| 1x1 dgrad+BN-bwd %d -> %d @ %d | %s |" % (k, co, hw, " | ".join("%.1f" % t for t in r)),
          flush=True)
C.conv.set_nfast(1)
