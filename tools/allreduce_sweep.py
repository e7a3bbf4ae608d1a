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
(apex DDP ``num_allreduce_streams``) to show whether extra communicators help, and
(``--wire``) the three ways DDP can reduce a bf16 bucket in fp32 or bf16: an fp32
all-reduce of an up-cast copy, fp32 reduce-scatter + bf16 all-gather (the default,
parallel/distributed.py ``bf16_wire``), and a native bf16 all-reduce.

RCCL channels (one workgroup each: the CUs a collective takes from the backward
kernels it overlaps) are fixed when a communicator is created, so a channel sweep is
one process set per setting:

    python tools/allreduce_sweep.py --nproc 8 --channels-sweep 4 8 16 32 --json sweep.json

runs this tool under torch.distributed.run once per channel count (NCCL_MIN/MAX_NCHANNELS)
and merges the rows (channels x message size).
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
    ap.add_argument("--wire", action="store_true",
                    help="also time the bf16-bucket wire formats (bf16 dtype only)")
    ap.add_argument("--channels", type=int, default=0,
                    help="NCCL_MIN/MAX_NCHANNELS for this run (0 = RCCL default)")
    ap.add_argument("--channels-sweep", type=int, nargs="*", default=None,
                    help="launcher mode: one torch.distributed.run per channel count")
    ap.add_argument("--nproc", type=int, default=8, help="launcher mode: ranks per run")
    a = ap.parse_args()
    if a.channels_sweep:
        return sweep_channels(a)
    if a.channels > 0:
        os.environ["NCCL_MIN_NCHANNELS"] = str(a.channels)
        os.environ["NCCL_MAX_NCHANNELS"] = str(a.channels)

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
        if a.wire and dt == torch.bfloat16:
            for name, fn in wire_formats(buf, world, rank).items():
                for _ in range(a.warmup):
                    fn()
                sync()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    fn()
                sync()
                tt = torch.tensor([(time.perf_counter() - t0) / a.iters], dtype=torch.float64,
                                  device=device)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                row["us_" + name] = round(float(tt.item()) * 1e6, 1)
        row["channels"] = a.channels or "default"
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
    return 0


def wire_formats(buf, world, rank):
    """The bf16-bucket reductions DDP can run (csrc/torch/reducer.cpp fp32 modes 2, 3, 0)."""
    n = buf.numel() // world * world
    b = buf[:n]

    def fp32_allreduce():
        c = b.float()
        dist.all_reduce(c)
        b.copy_(c)

    def rs_fp32_ag_bf16():
        c = b.float()
        shard = torch.empty(n // world, dtype=torch.float32, device=b.device)
        dist.reduce_scatter_tensor(shard, c)
        mine = b.view(world, -1)[rank]
        mine.copy_(shard)
        dist.all_gather_into_tensor(b, mine)

    def bf16_allreduce():
        dist.all_reduce(b)

    return {"fp32_allreduce": fp32_allreduce, "rs_fp32_ag_bf16": rs_fp32_ag_bf16,
            "bf16_allreduce": bf16_allreduce}


def sweep_channels(a):
    """Run this tool once per channel count under torch.distributed.run; merge rows."""
    import subprocess
    import tempfile

    merged = []
    for ch in a.channels_sweep:
        with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as f:
            out = f.name
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               "--nproc-per-node", str(a.nproc), "--master-addr", "127.0.0.1",
               "--master-port", str(29700 + ch), os.path.abspath(__file__),
               "--dtype", a.dtype, "--min-mb", str(a.min_mb), "--max-mb", str(a.max_mb),
               "--iters", str(a.iters), "--warmup", str(a.warmup), "--channels", str(ch),
               "--json", out, "--streams"] + [str(x) for x in a.streams] + (
                   ["--wire"] if a.wire else [])
        rc = subprocess.call(cmd)
        if rc != 0:
            print("channels %d: run failed (%d)" % (ch, rc), file=sys.stderr)
            return rc
        with open(out) as f:
            merged.extend(json.load(f)["rows"])
        os.unlink(out)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"world": a.nproc, "dtype": a.dtype, "rows": merged}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
