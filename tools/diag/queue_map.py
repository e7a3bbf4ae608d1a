#!/usr/bin/env python3
"""Which HIP streams share which hardware queue: reads a rocprofv3 kernel trace
(``--kernel-trace --output-format csv``) and prints, per (Queue_Id, Stream_Id), the
dispatch count, busy time and the kernel roles seen on it, so the stream -> queue map of a
step (compute, weight-gradient side stream, DDP bucket launch stream, RCCL streams,
SyncBN) can be read off.  Kernels that share a queue run in FIFO order, whatever CUs
are free (GPU_MAX_HW_QUEUES = 4 per process on the box).

    python tools/diag/queue_map.py TRACE_DIR [--range timed_steps] [--md out.md]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rocprof_summary import load_ranges  # noqa: E402

ROLES = [  # (role, substrings of the kernel name), first match wins
    ("rccl", ("nccl", "rccl", "Reduce", "AllGather", "ReduceScatter", "AllReduce")),
    ("wgrad", ("wgrad", "splitk_reduce", "colsum", "bias_grad", "Cijk_Alik_Bljk")),
    ("bn", ("bn_", "batch_norm", "stats_k", "reduce_k", "apply_k", "backward_k", "finalize")),
    ("conv", ("conv_tap", "conv3x3", "stem_conv", "dgrad")),
    ("gemm", ("Cijk", "gemm", "mfma")),
    ("attn", ("attn", "attention")),
    ("ln", ("ln_", "layer_norm")),
    ("optim", ("sgd", "adam", "lamb", "multi_tensor", "l2norm", "scale_k")),
    ("copy", ("copyBuffer", "fillBuffer", "elementwise", "copy")),
]


def role_of(name):
    for role, keys in ROLES:
        if any(k in name for k in keys):
            return role
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--range", default=None)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True))
    if not files:
        sys.exit("no kernel_trace.csv under %s" % a.root)
    ranges = load_ranges(a.root, a.range) if a.range else None
    per = collections.defaultdict(lambda: {"n": 0, "ns": 0, "roles": collections.Counter()})
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                if ranges is not None and not any(s <= t0 < e for s, e in ranges):
                    continue
                key = (r.get("Queue_Id", "?"), r.get("Stream_Id", "?"))
                e = per[key]
                e["n"] += 1
                e["ns"] += t1 - t0
                e["roles"][role_of(r["Kernel_Name"])] += 1
    lines = ["| Queue_Id | Stream_Id | dispatches | busy ms | roles (dispatches) |",
             "|---|---|---|---|---|"]
    for (q, st), e in sorted(per.items(), key=lambda kv: (str(kv[0][0]), str(kv[0][1]))):
        roles = ", ".join("%s %d" % rc for rc in e["roles"].most_common())
        lines.append("| %s | %s | %d | %.2f | %s |" % (q, st, e["n"], e["ns"] / 1e6, roles))
    queues = collections.defaultdict(list)
    for (q, st) in per:
        queues[q].append(st)
    lines.append("")
    lines.append("streams per hardware queue: " + "; ".join(
        "queue %s: streams %s" % (q, ", ".join(sorted(map(str, s)))) for q, s in sorted(queues.items())))
    out = "\n".join(lines)
    print(out)
    if a.md:
        with open(a.md, "w") as fh:
            fh.write(out + "\n")


if __name__ == "__main__":
    main()
