"""Attention kernels alone, for rocprofv3 counter passes: BERT-large shape (32 x 16
heads x 512, d 64, dropout 0.1) forward + backward a few times, per variant
(APEX_AMD_ATTN_FWD / APEX_AMD_ATTN_BASE read per launch).
    rocprofv3 --pmc SQ_WAVE_CYCLES ... --kernel-trace --stats -d out -- python3 tools/diag/attn_pmc.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from apex_example_amd.ops import fused_attention  # noqa: E402


def main():
    dev = "cuda"
    b, h, s, d = 32, 16, 512, 64
    causal = "--causal" in sys.argv
    if causal:
        b, s = 8, 1024
    p = 0.0 if "--p0" in sys.argv else 0.1
    q, k, v = (torch.randn(b, s, h, d, device=dev, dtype=torch.bfloat16, requires_grad=True)
               for _ in range(3))
    do = torch.randn(b, s, h, d, device=dev, dtype=torch.bfloat16)
    for var in ("1", "2"):
        os.environ["APEX_AMD_ATTN_FWD"] = var
        for _ in range(3):
            o = fused_attention(q, k, v, causal=causal, dropout_p=p)
            torch.autograd.grad(o, (q, k, v), do)
    torch.cuda.synchronize()
    print("attn_pmc done", flush=True)


if __name__ == "__main__":
    main()
