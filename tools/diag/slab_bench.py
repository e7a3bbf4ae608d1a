#!/usr/bin/env python3
"""The one-launch BatchNorm finalize over a conv epilogue's channel-major slab [2][C][S]
(bn.slab_train_stats / bn.slab_reduce_grad) at the ResNet-50 shapes: us per call."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timeit(fn, iters=50, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    from apex_example_amd import _native

    bn = _native.require().bn
    dev = "cuda"
    print("| S (tiles) | C | MB | slab_train_stats us | slab_reduce_grad us |")
    print("|---|---|---|---|---|")
    for S, C in [(6272, 64), (6272, 256), (12544, 256), (1568, 128), (1568, 512),
                 (392, 256), (392, 1024), (98, 512), (98, 2048)]:
        slab = torch.randn(2, C, S, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.long, device=dev)
        invstd = torch.rand(C, device=dev) + 0.5
        w = torch.ones(C, device=dev)
        t1 = timeit(lambda: bn.slab_train_stats(slab, S * 128, None, rm, rv, nbt, 1e-5, 0.1))
        t2 = timeit(lambda: bn.slab_reduce_grad(slab, invstd, w, True))
        print("| %d | %d | %.1f | %.1f | %.1f |" % (S, C, slab.numel() * 4 / 1e6, t1, t2),
              flush=True)


if __name__ == "__main__":
    main()
