#!/usr/bin/env python3
"""Does bench.py's ResNet-50 step take the BN-backward conv epilogue?  Counts the
epilogue dgrad calls and the BN outputs tagged for it over one training step.

    python tools/diag/bnbwd_count.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from apex_example_amd.ops import batch_norm as bnmod  # noqa: E402
from apex_example_amd.ops import conv as convmod  # noqa: E402


def main():
    sys.argv = [sys.argv[0], "--batch-size", "32"]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = bench.build_resnet(args, dev, 1)
    stats = {"dgrad_bn": 0, "src": 0, "src_none": 0, "bwd_fused": 0}
    orig_d, orig_s = convmod._dgrad_bn, bnmod._bwd_src

    def d(*a, **k):
        stats["dgrad_bn"] += 1
        return orig_d(*a, **k)

    def s(*a, **k):
        r = orig_s(*a, **k)
        stats["src" if r is not None else "src_none"] += 1
        if r is None:
            x = a[0]
            print("no src: dtype %s shape %s cl %s xl-is-x %s relu %s z %s mask %s" % (
                x.dtype, tuple(x.shape), x.is_contiguous(memory_format=torch.channels_last),
                a[1] is x, a[7], a[8], a[6] is not None))
        return r
    convmod._dgrad_bn, bnmod._bwd_src = d, s
    for _ in range(2):
        w.step(w.batch)
    torch.cuda.synchronize()
    stats["bwd_fused"] = bnmod.FUSED_BWD_CALLS[0]
    print(stats)


if __name__ == "__main__":
    main()
