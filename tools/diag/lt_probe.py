"""Which hipBLASLt epilogues / layouts have algorithms on this GPU (heuristic count),
and how accurate fp32 GEMMs are (vs fp64) - diagnostics for lt_ops.cpp."""
import itertools

import torch

from apex_example_amd import _native

D = _native.require().dense
EPI = {"DEFAULT": 1, "BIAS": 4, "GELU": 32, "GELU_BIAS": 36, "GELU_AUX": 160,
       "GELU_AUX_BIAS": 164, "DGELU": 192, "DGELU_BGRAD": 208, "BGRADA": 256, "BGRADB": 512}
HIP_R_16BF, HIP_R_32F = 14, 0
for (name, e), (ta, tb), aux, bt in itertools.product(
        EPI.items(), [(0, 0), (1, 0), (0, 1), (1, 1)], [-1, HIP_R_16BF], [-1, HIP_R_16BF, HIP_R_32F]):
    n = D.lt_probe(4096, 16384, 1024, e, ta, tb, torch.bfloat16, aux, bt)
    if n != 0:
        print("%-14s ta=%d tb=%d aux=%3d bias=%3d -> %d" % (name, ta, tb, aux, bt, n), flush=True)
print("probe done", flush=True)
a = torch.randn(2048, 2048, device="cuda", dtype=torch.float64)
b = torch.randn(2048, 2048, device="cuda", dtype=torch.float64)
ref = a @ b
for tf in (False, True):
    torch.backends.cuda.matmul.allow_tf32 = tf
    got = (a.float() @ b.float()).double()
    print("fp32 mm allow_tf32=%s: max rel err %.2e" % (tf, float((got - ref).abs().max() / ref.abs().max())))
