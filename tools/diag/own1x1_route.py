"""1x1 forwards consumed by a BatchNorm: own conv_tap_k with the statistics epilogue vs
hipBLASLt (torch.mm) + the BN statistics pass, at the ResNet-50 shapes (bs 256).  us per
call (median of 20); the routing table _OWN1X1 in ops/conv.py follows the winners."""
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


print("| Cin -> Cout @ hw | own + stats epilogue us | hipBLASLt + stats pass us | hipBLASLt alone us |")
print("|---|---|---|---|")
for ci, co, hw in [(256, 128, 56), (512, 256, 28), (1024, 512, 14), (1024, 256, 14),
                   (2048, 512, 7), (512, 128, 28), (256, 64, 56), (64, 64, 56), (128, 128, 28),
                   (256, 256, 14), (512, 512, 7), (64, 256, 56), (128, 512, 28),
                   (256, 1024, 14), (512, 2048, 7)]:
    x = torch.randn(256, ci, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(co, ci, 1, 1, device="cuda") / ci ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=cl)
    sh = torch.zeros(co, device="cuda")
    rm, rv = torch.zeros(co, device="cuda"), torch.ones(co, device="cuda")
    x2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
    w2 = w.reshape(co, ci).t()

    def lib():
        y = torch.mm(x2, w2).view(256, hw, hw, co).permute(0, 3, 1, 2)
        C.bn.train_stats(y, rm, rv, None, 1e-5, 0.1)

    t_own = timeit(lambda: C.conv.conv_fwd_stats(x, w, 1, sh))
    t_lib = timeit(lib)
    t_mm = timeit(lambda: torch.mm(x2, w2))
    print("| %d -> %d @ %d | %.1f | %.1f | %.1f |" % (ci, co, hw, t_own, t_lib, t_mm), flush=True)
