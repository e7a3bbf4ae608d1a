#!/usr/bin/env python3
"""wgrad4w tile order at full load: the XCD-grouped walk (APEX_AMD_W4W_GROUPM m-tiles per
group, read per launch; or another per-launch knob given as the 2nd argument, e.g.
APEX_AMD_W4W_LAYOUT) swept over the BERT / GPT-2 weight-gradient shapes at the split
counts the model uses, interleaved rounds in one process (same clocks for every row)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


SHAPES = [("bert ffn-in", 16384, 4096, 1024, 4), ("bert ffn-out", 16384, 1024, 4096, 4),
          ("bert qkv", 16384, 3072, 1024, 4), ("gpt2 ffn-in", 8192, 4096, 1024, 2),
          ("gpt2 ffn-out", 8192, 1024, 4096, 2), ("gpt2 qkv", 8192, 3072, 1024, 2)]


def main():
    from apex_example_amd import _native
    dn = _native.require().dense
    groups = [int(g) for g in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8,16").split(",")]
    var = sys.argv[2] if len(sys.argv) > 2 else "APEX_AMD_W4W_GROUPM"  # or ..._LAYOUT
    for (name, T, m, n, s) in SHAPES:
        dy = torch.randn(T, m, device="cuda").to(torch.bfloat16)
        x = torch.randn(T, n, device="cuda").to(torch.bfloat16)
        best = {g: 1e9 for g in groups}
        for _ in range(3):
            for g in groups:
                os.environ[var] = str(g)
                best[g] = min(best[g], timeit(lambda: dn.wgrad4w(dy, x, s, torch.bfloat16)))
        gf = 2.0 * T * m * n / 1e9
        print("| %s | S=%d | %s |" % (name, s, " | ".join(
            "g%d %.1f us (%.0f TF)" % (g, t, gf / t * 1e3) for g, t in best.items())), flush=True)


if __name__ == "__main__":
    main()
