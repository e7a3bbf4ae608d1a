#!/usr/bin/env python3
"""Summarise a rocprofv3 --hip-runtime-trace CSV: per HIP API function, calls /
total / max host time inside a roctx range (default timed_steps), to find the
call that blocks the host (a device sync) when the kernel trace shows idle gaps.

    rocprofv3 --hip-runtime-trace --kernel-trace --marker-trace --output-format csv -d OUT -o run -- python3 bench.py ...
    python tools/diag/hip_api_summary.py OUT
"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rocprof_summary import load_ranges  # noqa: E402


def main():
    root = sys.argv[1]
    rng = sys.argv[2] if len(sys.argv) > 2 else "timed_steps"
    ranges = load_ranges(root, rng)
    files = glob.glob(os.path.join(root, "**", "*hip_api_trace.csv"), recursive=True)
    tot, cnt, mx = defaultdict(float), defaultdict(int), defaultdict(float)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                if ranges and not any(r0 <= s <= r1 for r0, r1 in ranges):
                    continue
                n = row.get("Function") or row.get("Operation") or "?"
                d = (e - s) / 1e3
                tot[n] += d
                cnt[n] += 1
                mx[n] = max(mx[n], d)
    # idle gaps on the GPU: was the next kernel's launch call issued before the gap
    # began (device-side wait) or during it (host lag)?
    launches = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                cid = row.get("Correlation_Id")
                if cid:
                    launches[cid] = (int(row["Start_Timestamp"]), row.get("Function", "?"))
    kern = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                s0 = int(row["Start_Timestamp"])
                if ranges and not any(r0 <= s0 <= r1 for r0, r1 in ranges):
                    continue
                kern.append((s0, int(row["End_Timestamp"]), row.get("Kernel_Name", "?")[:60],
                             row.get("Correlation_Id")))
    kern.sort()
    gaps = []
    end = kern[0][1] if kern else 0
    for i in range(1, len(kern)):
        s0, e0, n0, cid = kern[i]
        if s0 - end > 50_000:
            call = launches.get(cid)
            lag = (call[0] - end) / 1e3 if call else float("nan")
            gaps.append(((s0 - end) / 1e3, lag, kern[i - 1][2], n0))
        end = max(end, e0)
    print("| gap us | launch call after gap start (us; >0 = host lag) | after | before |")
    print("|---|---|---|---|")
    for g in sorted(gaps, key=lambda t: -t[0])[:20]:
        print("| %.1f | %.1f | `%s` | `%s` |" % g)
    print()
    print("| HIP API | calls | total us | max us |")
    print("|---|---|---|---|")
    for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
        print("| %s | %d | %.1f | %.1f |" % (n, cnt[n], t, mx[n]))


if __name__ == "__main__":
    main()
