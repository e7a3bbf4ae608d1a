#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (CSV) into a per-kernel table.

    rocprofv3 --kernel-trace --marker-trace --output-format csv -d OUT -o run -- python bench.py ...
    python tools/rocprof_summary.py OUT [--range timed_steps] [--top 40] [--md out.md]

With ``--range NAME`` only kernels that START inside the roctx range(s) called
NAME (bench.py marks its timed steps with "timed_steps") are counted, so the
MIOpen solver search of the warmup does not pollute the table.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def _find(root, pattern):
    hits = glob.glob(os.path.join(root, "**", pattern), recursive=True)
    return sorted(hits)


def _short(name, n=110):
    name = re.sub(r"\s+", " ", name)
    return name if len(name) <= n else name[: n - 3] + "..."


def load_ranges(root, range_name):
    files = _find(root, "*marker_api_trace.csv")
    ranges = []
    for f in files:
        with open(f) as fh:
            rd = csv.DictReader(fh)
            for row in rd:
                # the range name sits in "Function"/"Message" depending on the
                # rocprofv3 version: accept it in any text column
                if not any(range_name in (v or "") for k, v in row.items()
                           if "Timestamp" not in (k or "")):
                    continue
                s = int(row.get("Start_Timestamp") or row.get("Start") or 0)
                e = int(row.get("End_Timestamp") or row.get("End") or 0)
                if e > s:
                    ranges.append((s, e))
            if not ranges:
                print("marker columns: %s" % (rd.fieldnames,), file=sys.stderr)
    return ranges


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--range", default=None)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--md", default=None)
    ap.add_argument("--steps", type=int, default=None, help="divide totals per step")
    ap.add_argument("--dispatch-filter", default=None,
                    help="regex: also list every matching dispatch in order (grid, duration)")
    ap.add_argument("--dispatch-out", default=None)
    ap.add_argument("--names-out", default=None,
                    help="write every kernel's FULL name with calls / total us (untruncated)")
    ap.add_argument("--gaps", type=int, default=0,
                    help="also list the N largest idle gaps (no kernel running) with the "
                         "kernels on both sides, and the idle total per step")
    a = ap.parse_args(argv)
    disp = []
    spans = []

    files = _find(a.root, "*kernel_trace.csv")
    if not files:
        print("no kernel_trace.csv under", a.root)
        return 1
    ranges = load_ranges(a.root, a.range) if a.range else []
    if a.range and not ranges:
        print("warning: range %r not found; using the whole trace" % a.range, file=sys.stderr)

    tot = defaultdict(float)
    cnt = defaultdict(int)
    t_min, t_max = None, None
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                s = int(row["Start_Timestamp"])
                e = int(row["End_Timestamp"])
                if ranges and not any(r0 <= s <= r1 for r0, r1 in ranges):
                    continue
                name = row.get("Kernel_Name", "?")
                if a.dispatch_filter and re.search(a.dispatch_filter, name):
                    disp.append((s, _short(name, 140), row.get("Grid_Size_X", ""),
                                 row.get("Grid_Size_Y", ""), row.get("Grid_Size_Z", ""),
                                 row.get("Workgroup_Size_X", ""), (e - s) / 1e3))
                tot[name] += (e - s) / 1e3  # us
                cnt[name] += 1
                if a.gaps:
                    spans.append((s, e, name))
                t_min = s if t_min is None else min(t_min, s)
                t_max = e if t_max is None else max(t_max, e)
    total = sum(tot.values())
    span = (t_max - t_min) / 1e3 if t_min is not None else 0.0
    rows = sorted(tot.items(), key=lambda kv: -kv[1])
    div = a.steps or 1
    lines = []
    lines.append("| # | kernel | calls | total us%s | %% of kernel time |" % (
        "/step" if a.steps else ""))
    lines.append("|---|---|---|---|---|")
    for i, (k, v) in enumerate(rows[: a.top]):
        lines.append("| %d | `%s` | %d | %.1f | %.1f |" % (i + 1, _short(k), cnt[k] // div,
                                                         v / div, 100.0 * v / total))
    head = ("kernels: %d distinct, %d dispatches; summed kernel time %.1f us; window %.1f us "
            "(busy %.1f%%)" % (len(tot), sum(cnt.values()), total, span,
                               100.0 * total / span if span else 0.0))
    out = head + "\n\n" + "\n".join(lines) + "\n"
    if a.gaps and spans:
        spans.sort()
        gaps = []
        end, prev = spans[0][1], spans[0][2]
        for s0, e0, n0 in spans[1:]:
            if s0 > end:
                gaps.append(((s0 - end) / 1e3, prev, n0))
            if e0 > end:
                end, prev = e0, n0
        idle = sum(g[0] for g in gaps)
        out += "\nidle (no kernel running): %.1f us total%s, %d gaps; largest:\n\n" % (
            idle / div if a.steps else idle, " per step" if a.steps else "", len(gaps))
        out += "| gap us | after | before |\n|---|---|---|\n"
        for g, p0, n0 in sorted(gaps, key=lambda t: -t[0])[: a.gaps]:
            out += "| %.1f | `%s` | `%s` |\n" % (g, _short(p0, 70), _short(n0, 70))
    print(out)
    if a.md:
        with open(a.md, "w") as fh:
            fh.write(out)
    if a.names_out:
        with open(a.names_out, "w") as fh:
            for k, v in rows:
                fh.write("%d\t%.1f\t%s\n" % (cnt[k] // div, v / div, re.sub(r"\s+", " ", k)))
    if a.dispatch_out:
        with open(a.dispatch_out, "w") as fh:
            for s0, n, gx, gy, gz, wg, us in sorted(disp):
                fh.write("%d\t%s\t%s\t%s\t%s\t%s\t%.2f\n" % (s0, n, gx, gy, gz, wg, us))
    return 0


if __name__ == "__main__":
    sys.exit(main())
