#!/usr/bin/env python3
"""Does the multi-tensor launch-plan cache hit in steady state?  Prints the cache
size after successive bench.py steps (a growing size = a new plan per step).

    python tools/diag/plan_cache.py --model bert_large
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from apex_example_amd import _native  # noqa: E402


def main():
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    build = {"resnet50": bench.build_resnet, "bert_large": bench.build_bert,
             "gpt2_medium": bench.build_gpt2}[args.model]
    w = build(args, dev, 1)
    mt = _native.require().mt
    for i in range(12):
        t0 = time.perf_counter()
        w.step(w.batch)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print("step %2d: plan cache %4d entries, host %.1f ms, wall %.1f ms" % (
            i, mt.plan_cache_size(), (t1 - t0) * 1e3, (time.perf_counter() - t0) * 1e3), flush=True)


if __name__ == "__main__":
    main()
