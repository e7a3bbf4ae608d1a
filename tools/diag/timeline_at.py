"""Kernel timeline (all queues) around the N-th-from-last dispatch of a kernel matching a
pattern, from a rocprofv3 kernel-trace CSV run.
    python tools/diag/timeline_at.py OUT_DIR PATTERN [--nth 2] [--before-ms 1.5] [--after-ms 0.8]"""
import argparse
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("pattern")
    ap.add_argument("--nth", type=int, default=2)
    ap.add_argument("--before-ms", type=float, default=1.5)
    ap.add_argument("--after-ms", type=float, default=0.8)
    a = ap.parse_args()
    ks = []
    for f in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                       r.get("Queue_Id", "?"), r.get("Stream_Id", r.get("Correlation_Id", "?"))))
    ks.sort()
    hits = [k for k in ks if re.search(a.pattern, k[2])]
    s0 = hits[-a.nth][0]
    lo, hi = s0 - int(a.before_ms * 1e6), s0 + int(a.after_ms * 1e6)
    for s, e, n, q, st in ks:
        if lo <= s <= hi:
            print("%9.1f us  %7.1f us  q%-3s s%-4s %s" % ((s - s0) / 1e3, (e - s) / 1e3, q, st,
                                                        n[:100]))


if __name__ == "__main__":
    main()
