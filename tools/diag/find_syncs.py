#!/usr/bin/env python3
"""List every host<->device synchronisation inside one training step of a bench.py
workload (torch.cuda.set_sync_debug_mode), with the Python stack that caused it.
A sync inside the step drains the GPU queue; the host's launch work after it then
shows up as idle gaps in the kernel trace (tools/rocprof_summary.py --gaps).

    python tools/diag/find_syncs.py --model bert_large
"""
import os
import sys
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    build = {"resnet50": bench.build_resnet, "resnet18": bench.build_resnet,
             "bert_large": bench.build_bert, "gpt2_medium": bench.build_gpt2}[args.model]
    w = build(args, dev, 1)
    for _ in range(3):
        w.step(w.batch)
    torch.cuda.synchronize()
    seen = []

    def show(message, category, filename, lineno, file=None, line=None):
        stack = [f for f in traceback.format_stack()[:-2]
                 if "apex_example_amd" in f or "bench.py" in f or "torch/nn" in f]
        seen.append((str(message), stack[-6:]))

    warnings.showwarning = show
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    w.step(w.batch)
    torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    print("%d synchronising calls in one %s step" % (len(seen), args.model))
    for msg, stack in seen:
        print("-", msg.splitlines()[0][:150])
        for f in stack:
            print("   ", f.strip().replace("\n", " | ")[:220])


if __name__ == "__main__":
    main()
