"""Run the MFMA conv kernels on two ResNet-50 shapes (for rocprofv3 --pmc)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from apex_example_amd import _native  # noqa: E402

cv = _native.require().conv
for (n, c, hw) in [(256, 64, 56), (256, 256, 14)]:
    x = torch.randn(n, c, hw, hw, device="cuda", dtype=torch.bfloat16).to(
        memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device="cuda", dtype=torch.bfloat16) * 0.05).to(
        memory_format=torch.channels_last)
    for _ in range(3):
        cv.conv_fwd(x, w)
        cv.conv_wgrad(x, x, torch.bfloat16)
torch.cuda.synchronize()
print("done")
