"""Long HIP API calls (host-blocking candidates) from a rocprofv3 --hip-trace CSV run:
per API name, calls and total time above a threshold, plus the longest individual calls.
    python tools/diag/hip_api_long.py OUT_DIR [--min-us 50]"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--min-us", type=float, default=50.0)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.root, "**", "*hip_api_trace.csv"), recursive=True)
    agg = defaultdict(lambda: [0, 0.0])
    longest = []
    for f in files:
        for r in csv.DictReader(open(f)):
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
            if d >= a.min_us:
                agg[r["Function"]][0] += 1
                agg[r["Function"]][1] += d
                longest.append((d, r["Function"], int(r["Start_Timestamp"])))
    print("| HIP API | calls >= %.0f us | total us |" % a.min_us)
    print("|---|---|---|")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("| %s | %d | %.0f |" % (k, n, t))
    longest.sort(reverse=True)
    print("\nlongest:")
    for d, fn, ts in longest[:25]:
        print("%10.1f us  %s  @%d" % (d, fn, ts))




def sync_calls(root, names=("hipMemcpyWithStream", "hipMemcpy", "hipDeviceSynchronize",
                            "hipStreamSynchronize", "hipEventSynchronize", "hipMemcpyDtoH",
                            "hipStreamWaitEvent", "hipMemcpyAsync", "hipMalloc", "hipFree")):
    """Every call of the blocking-candidate APIs, in time order (ms from the first)."""
    files = glob.glob(os.path.join(root, "**", "*hip_api_trace.csv"), recursive=True)
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Function"] in names:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
    rows.sort()
    t0 = rows[-1][0] if rows else 0
    for s, e, fn in rows[-120:]:
        print("%10.3f ms  %8.1f us  %s" % ((s - t0) / 1e6, (e - s) / 1e3, fn))


if __name__ == "__main__":
    import sys
    if "--sync" in sys.argv:
        sync_calls(sys.argv[1])
    else:
        main()
