"""A/B for BERT-large's FC1: addmm + separate GELU vs hipBLASLt's GELU-bias epilogue
(torch._addmm_activation, tanh-approximate GELU) at [16384 x 1024] @ [1024 x 4096]."""
import torch
import torch.nn.functional as F


def t(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


x = torch.randn(16384, 1024, device="cuda", dtype=torch.bfloat16)
w = torch.randn(4096, 1024, device="cuda", dtype=torch.bfloat16) * 0.03
b = torch.randn(4096, device="cuda", dtype=torch.bfloat16)
print("addmm only             %.1f us" % t(lambda: torch.addmm(b, x, w.t())))
print("addmm + gelu(erf)      %.1f us" % t(lambda: F.gelu(torch.addmm(b, x, w.t()))))
print("addmm + gelu(tanh)     %.1f us" % t(lambda: F.gelu(torch.addmm(b, x, w.t()), approximate="tanh")))
print("_addmm_activation gelu %.1f us" % t(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True)))
ref = F.gelu(torch.addmm(b, x, w.t()).float(), approximate="tanh")
got = torch._addmm_activation(b, x, w.t(), use_gelu=True).float()
print("epilogue vs tanh-gelu max err %.3e (max |ref| %.2f)" % ((got - ref).abs().max(), ref.abs().max()))
ref2 = F.gelu(torch.addmm(b, x, w.t()).float())
print("epilogue vs erf-gelu max err %.3e" % (got - ref2).abs().max())
from apex_example_amd import _native  # noqa: E402

pre = torch.addmm(b, x, w.t())
print("ATen gelu(erf)         %.1f us" % t(lambda: F.gelu(pre)))
print("dense.gelu(erf)        %.1f us" % t(lambda: _native.require().dense.gelu(pre, False)))
print("ATen gelu(tanh)        %.1f us" % t(lambda: F.gelu(pre, approximate="tanh")))
print("dense.gelu(tanh)       %.1f us" % t(lambda: _native.require().dense.gelu(pre, True)))
