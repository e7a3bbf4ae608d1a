#!/usr/bin/env python3
"""Find the call sites of the ATen copy kernels in one ResNet-50 training step
(bench.py's amd path): torch.profiler with stacks, copy-like ops sorted by GPU time.

    python tools/diag/find_copies.py [--batch-size 256]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    bs = sys.argv[sys.argv.index("--batch-size") + 1] if "--batch-size" in sys.argv else "256"
    sys.argv = ["bench.py", "--batch-size", bs]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = bench.build_resnet(args, dev, 1)
    for _ in range(3):
        w.step(w.batch)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
        w.step(w.batch)
        torch.cuda.synchronize()
    names = ("aten::copy_", "aten::contiguous", "aten::clone", "aten::_to_copy", "aten::to",
             "aten::add", "aten::add_", "aten::mul", "aten::fill_", "aten::zero_", "aten::cat")
    seen = 0
    for ev in sorted(prof.events(), key=lambda e: -e.device_time_total):
        if ev.name not in names or ev.device_time_total <= 0:
            continue
        stack = [s for s in (ev.stack or []) if "apex_example_amd" in s or "bench.py" in s]
        print("%8.1f us  %-18s %s" % (ev.device_time_total, ev.name, ev.input_shapes[:2]))
        for s in stack[:5]:
            print("            ", s)
        seen += 1
        if seen >= 40:
            break


if __name__ == "__main__":
    main()
