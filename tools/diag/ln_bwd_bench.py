"""Time the fused residual-join LayerNorm backward (csrc/hip/layer_norm.hip ln_bwd_fast +
the column-sum kernel) at the GPT-2-medium (fp32 residual, fp16 sublayer output, dropout
0.1) and BERT-large (bf16) shapes.  Prints one markdown row per case."""
import os
import sys

# the package under test: this tree, or another build (AB_ROOT=ab_old) for a same-box A/B
sys.path.insert(0, os.environ.get("AB_ROOT") or os.path.join(os.path.dirname(__file__), "..", ".."))

import torch  # noqa: E402

from apex_example_amd.normalization import FusedLayerNorm  # noqa: E402
from apex_example_amd.normalization.fused_layer_norm import AddDropoutLayerNormFunction  # noqa: E402


def case(name, rows, n2, xdt, hdt, y16):
    torch.manual_seed(0)
    x = torch.randn(rows, n2, device="cuda", dtype=xdt, requires_grad=True)
    h = torch.randn(rows, n2, device="cuda", dtype=hdt, requires_grad=True)
    ln = FusedLayerNorm(n2).to("cuda").to(xdt)
    y, s = AddDropoutLayerNormFunction.apply(x, h, ln.weight, ln.bias, ln.normalized_shape,
                                             ln.eps, 0.1, y16)
    dy = torch.randn_like(y)
    ds = torch.randn_like(s)
    ins = [x, h, ln.weight, ln.bias]
    for _ in range(5):
        torch.autograd.grad([y, s], ins, [dy, ds], retain_graph=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    a.record()
    for _ in range(n):
        torch.autograd.grad([y, s], ins, [dy, ds], retain_graph=True)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / n
    print("| %s | %d x %d | %.1f |" % (name, rows, n2, us), flush=True)


if os.environ.get("LN_ONE_ROW"):
    from apex_example_amd import _native  # noqa: E402
    _native.require().layer_norm.set_bwd_one_row(int(os.environ["LN_ONE_ROW"]))
print("| join | shape | backward us (LN kernel + column sums + autograd) |")
print("|---|---|---|")
case("GPT-2-medium O1 (fp32 x, fp16 h, y fp16)", 8192, 1024, torch.float32, torch.float16, True)
case("BERT-large (bf16)", 16384, 1024, torch.bfloat16, torch.bfloat16, False)
