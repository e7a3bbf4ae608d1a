"""Run the 3x3 MFMA wgrad kernel on ResNet-50 shapes a few times (a short
program for rocprofv3 --pmc passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from apex_example_amd import _native  # noqa: E402

cv = _native.require().conv
shapes = [(256, 64, 56), (256, 128, 28), (256, 256, 14), (256, 512, 7)]
which = [int(a) for a in sys.argv[1:]] or range(len(shapes))
for i in which:
    n, c, hw = shapes[i]
    x = torch.randn(n, c, hw, hw, device="cuda", dtype=torch.bfloat16).to(
        memory_format=torch.channels_last)
    dy = torch.randn_like(x)
    for _ in range(3):
        cv.conv_wgrad(dy, x, torch.bfloat16, int(os.environ.get("ALGO", "0")))
torch.cuda.synchronize()
print("ok")
