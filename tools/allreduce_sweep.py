#!/usr/bin/env python3
"""All-reduce bandwidth sweep for choosing DDP bucket sizes.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/allreduce_sweep.py \
        [--dtype bf16] [--min-mb 0.25] [--max-mb 256] [--iters 20] [--json out.json]

Per message size: mean latency of ``dist.all_reduce`` on the RCCL (nccl)
backend - or gloo on CPU - and the ring "bus bandwidth" 2(n-1)/n * bytes / t,
the number to compare with the per-link xGMI figure (~153 GB/s; 7 links per
MI355X).  A bucket is "big enough" once busbw is within ~80 % of its plateau;
the DDP default ``message_size`` and docs/DDP_TUNING.md come from this table.
Also times the same bytes split over 1, 2 and 4 concurrent process groups
(apex DDP ``num_allreduce_streams``) to show whether extra communicators help.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--min-mb", type=float, default=0.25)
    ap.add_argument("--max-mb", type=float, default=256.0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, nargs="*", default=[1, 2, 4])
    ap.add_argument("--json", default=None)
    a = ap.parse_args()

    from apex_example_amd.utils.dist import init_distributed

    rank, world, device = init_distributed()
    if world < 2:
        print("run under torchrun with >= 2 processes", file=sys.stderr)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    esz = torch.tensor([], dtype=dt).element_size()
    gpu = device.type == "cuda"

    def sync():
        if gpu:
            torch.cuda.synchronize()

    groups = {1: [dist.group.WORLD]}
    for s in a.streams:
        if s > 1:
            groups[s] = [dist.new_group(list(range(world))) for _ in range(s)]

    results = []
    mb = a.min_mb
    while mb <= a.max_mb + 1e-9:
        n = max(1, int(mb * 2**20 / esz))
        buf = torch.ones(n, dtype=dt, device=device)
        row = {"mbytes": round(n * esz / 2**20, 3), "elements": n}
        for s, pgs in groups.items():
            parts = buf.chunk(s)
            for _ in range(a.warmup):
                for p, g in zip(parts, pgs):
                    dist.all_reduce(p, group=g, async_op=True).wait()
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                works = [dist.all_reduce(p, group=g, async_op=True) for p, g in zip(parts, pgs)]
                for w in works:
                    w.wait()
            sync()
            t = (time.perf_counter() - t0) / a.iters
            tt = torch.tensor([t], dtype=torch.float64, device=device)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
            busbw = 2 * (world - 1) / world * n * esz / t / 1e9 if world > 1 else 0.0
            row["us_%dpg" % s] = round(t * 1e6, 1)
            row["busbw_GBs_%dpg" % s] = round(busbw, 1)
        results.append(row)
        if rank == 0:
            print(json.dumps(row), flush=True)
        mb *= 2
    if rank == 0 and a.json:
        with open(a.json, "w") as f:
            json.dump({"world": world, "dtype": a.dtype, "backend": dist.get_backend(),
                       "rows": results}, f, indent=1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
