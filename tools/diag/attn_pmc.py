"""Run the fused attention kernels (BERT-large and GPT-2-medium shapes, dropout 0.1)
a few times - the workload for rocprofv3 --pmc passes (tools/diag/attn_pmc.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from apex_example_amd.ops import fused_attention  # noqa: E402

for (b, h, s, causal) in [(32, 16, 512, False), (8, 16, 1024, True)]:
    q, k, v = (torch.randn(b, s, h, 64, device="cuda", dtype=torch.bfloat16, requires_grad=True)
               for _ in range(3))
    do = torch.randn(b, s, h, 64, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        o = fused_attention(q, k, v, causal=causal, dropout_p=0.1)
        torch.autograd.grad(o, (q, k, v), do)
torch.cuda.synchronize()
print("done")
