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
    if args.force_collectives:  # a 1-rank RCCL group, as bench.py makes for this mode
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    build = {"resnet50": bench.build_resnet, "bert_large": bench.build_bert,
             "gpt2_medium": bench.build_gpt2, "convnet": bench.build_convnet}[args.model]
    opt_only = os.environ.get("HOST_PROFILE_OPT_ONLY") == "1"
    w = build(args, dev, 1)
    for _ in range(3):
        w.step(w.batch)
    torch.cuda.synchronize()
    import time
    fn = (lambda: w.opt_only()) if opt_only else (lambda: w.step(w.batch))
    # per-call host time of the first calls after a training step (bench.py's
    # optimizer-step metric is taken right after its timed loop)
    per = []
    for _ in range(6):
        h0 = time.perf_counter()
        fn()
        per.append((time.perf_counter() - h0) * 1e6)
    torch.cuda.synchronize()
    print("first calls after a train step, host us: " + " ".join("%.0f" % t for t in per))
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print("host ms per call (no profiler): %.4f  (until sync %.4f)" % (
        (t1 - t0) * 1e3 / args.steps, (time.perf_counter() - t0) * 1e3 / args.steps))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        fn()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(45)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
