#!/usr/bin/env python3
"""cProfile of the host side of bench.py training steps (where the Python launch
work goes), e.g. to explain idle GPU gaps around the optimizer step.

    python tools/diag/host_profile.py --model bert_large [--steps 5]
"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    build = {"resnet50": bench.build_resnet, "bert_large": bench.build_bert,
             "gpt2_medium": bench.build_gpt2}[args.model]
    w = build(args, dev, 1)
    for _ in range(3):
        w.step(w.batch)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        w.step(w.batch)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(45)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
