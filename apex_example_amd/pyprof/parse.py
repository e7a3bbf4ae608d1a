"""Attribute rocprofv3 kernels to pyprof op ranges (apex.pyprof.parse + prof).

    python -m apex_example_amd.pyprof.parse OUT_DIR [--top 30] [--csv ops.csv]

Reads ``*kernel_trace.csv`` and ``*marker_api_trace.csv`` from a
``rocprofv3 --kernel-trace --marker-trace --output-format csv`` run.  Kernels
are matched to the innermost op range that was open on the launching thread
when the kernel was dispatched (correlation by thread id + dispatch time
window).  With ``--hip-runtime-trace`` in the same run the kernel's host
enqueue time (by Correlation_Id) is matched against the ranges - exact; without
it the GPU start time is used, which is only right when the host is not
running ahead of the GPU (e.g. under AMD_SERIALIZE_KERNEL=3).  Output: per op signature,
calls, GPU time, estimated TFLOP/s and GB/s.
"""
from __future__ import annotations

import argparse
import bisect
import csv
import glob
import os
import sys
from collections import defaultdict

from .flops import op_flops


def _rows(root, pattern):
    for f in sorted(glob.glob(os.path.join(root, "**", pattern), recursive=True)):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def _ts(row, *keys):
    for k in keys:
        v = row.get(k)
        if v not in (None, ""):
            return int(v)
    return 0


def load_ranges(root):
    """[(start, end, depth, label)] of pyprof op ranges, innermost-resolvable."""
    out = []
    for row in _rows(root, "*marker_api_trace.csv"):
        label = None
        for k in ("Message", "Function", "Marker_Message", "Name"):
            v = row.get(k)
            if v and "(" in v and v.endswith(")"):
                label = v
                break
        if label is None:
            continue
        s = _ts(row, "Start_Timestamp", "Start")
        e = _ts(row, "End_Timestamp", "End")
        if e > s:
            out.append((s, e, label))
    out.sort()
    return out


def load_launch_times(root):
    """Correlation_Id -> host launch timestamp, from a --hip-runtime-trace run."""
    out = {}
    for row in _rows(root, "*hip_api_trace.csv"):
        fn = row.get("Function", "")
        if "Launch" not in fn and "launch" not in fn:
            continue
        cid = row.get("Correlation_Id")
        if cid:
            out[cid] = _ts(row, "Start_Timestamp")
    return out


def attribute(root):
    ranges = load_ranges(root)
    launches = load_launch_times(root)
    starts = [r[0] for r in ranges]
    per_op = defaultdict(lambda: [0, 0.0])  # label -> [calls, us]
    per_kernel = defaultdict(lambda: [0, 0.0])
    for row in _rows(root, "*kernel_trace.csv"):
        s = _ts(row, "Start_Timestamp")
        e = _ts(row, "End_Timestamp")
        name = row.get("Kernel_Name", "?")
        per_kernel[name][0] += 1
        per_kernel[name][1] += (e - s) / 1e3
        t = launches.get(row.get("Correlation_Id"), s)  # host enqueue time when known
        # innermost enclosing range: scan back from the last range starting <= t
        hi = bisect.bisect_right(starts, t) - 1
        i = hi
        best = None
        while i >= 0 and i > hi - 64:
            r0, r1, lab = ranges[i]
            if r0 <= t <= r1 and (best is None or r0 >= best[0]):
                best = (r0, lab)
            i -= 1
        lab = best[1] if best else "<unattributed>"
        per_op[lab][0] += 1
        per_op[lab][1] += (e - s) / 1e3
    return per_op, per_kernel


def report(per_op, top=30):
    lines = ["| op (signature) | kernels | GPU us | est TFLOP/s | est GB/s |", "|---|---|---|---|---|"]
    for lab, (n, us) in sorted(per_op.items(), key=lambda kv: -kv[1][1])[:top]:
        fl, nb = op_flops(lab) if lab != "<unattributed>" else (None, 0)
        tf = "%.1f" % (fl / (us * 1e-6) / 1e12) if fl and us > 0 else "-"
        gb = "%.0f" % (nb / (us * 1e-6) / 1e9) if nb and us > 0 else "-"
        lines.append("| `%s` | %d | %.1f | %s | %s |" % (lab[:120], n, us, tf, gb))
    return "\n".join(lines)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--csv", default=None)
    a = ap.parse_args(argv)
    per_op, _ = attribute(a.root)
    print(report(per_op, a.top))
    if a.csv:
        with open(a.csv, "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["op", "kernels", "gpu_us"])
            for lab, (n, us) in sorted(per_op.items(), key=lambda kv: -kv[1][1]):
                w.writerow([lab, n, "%.3f" % us])
    return 0


if __name__ == "__main__":
    sys.exit(main())
