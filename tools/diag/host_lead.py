"""Host lead per training step: roctx step markers (host time) vs the GPU start of the
step's first kernel (`--first` pattern) and the GPU end of its last SGD kernel, from a
rocprofv3 --kernel-trace --marker-trace CSV run of bench.py with APEX_AMD_BENCH_STEP_MARKS=1."""
import argparse
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--first", default="bfloat16_copy_kernel")
    a = ap.parse_args()
    ks = []
    for f in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    marks = []
    for f in glob.glob(os.path.join(a.root, "**", "*marker_api_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            # the range name sits in "Function" / "Message" depending on the rocprofv3
            # version: take it from any text column
            msg = next((v for k, v in r.items() if "Timestamp" not in (k or "")
                        and re.fullmatch(r"step\d+", v or "")), None)
            if msg and int(r["End_Timestamp"]) > int(r["Start_Timestamp"]):
                marks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), msg))
    marks.sort()
    print("| step | host start -> GPU first kernel (us) | host end -> GPU last sgd end (us) | host step (ms) |")
    print("|---|---|---|---|")
    for s, e, m in marks:
        first = next((k for k in ks if k[0] >= s and re.search(a.first, k[2])), None)
        sg = [k for k in ks if "sgd_pair_kernel" in k[2] and k[0] >= s]
        lst = sg[0] if sg else None
        print("| %s | %s | %s | %.2f |" % (
            m, "%.0f" % ((first[0] - s) / 1e3) if first else "-",
            "%.0f" % ((lst[1] - e) / 1e3) if lst else "-", (e - s) / 1e6))


if __name__ == "__main__":
    main()
