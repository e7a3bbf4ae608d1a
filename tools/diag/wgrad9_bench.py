"""3x3 stride-1 weight gradients of ResNet-50 (bs 256): per-tap kernel (algo 0) vs the
strip-ring all-taps kernel on 64 x 64 channel tiles (algo 4), us per call incl. the split
reduction (median of 20), bf16 output."""
import sys

import torch

sys.path.insert(0, ".")
from apex_example_amd import _native  # noqa: E402

cv = _native.require().conv
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


print("| C @ hw | per-tap us | strip-ring us | TFLOP/s strip |")
print("|---|---|---|---|")
for c, hw in [(64, 56), (128, 28), (256, 14), (512, 7)]:
    x = torch.randn(256, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    dy = torch.randn(256, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    t0 = timeit(lambda: cv.conv_wgrad(dy, x, torch.bfloat16, 0))
    t4 = timeit(lambda: cv.conv_wgrad(dy, x, torch.bfloat16, 4))
    fl = 2.0 * 256 * hw * hw * c * c * 9
    print("| %d @ %d | %.1f | %.1f | %.0f |" % (c, hw, t0, t4, fl / t4 / 1e6), flush=True)
