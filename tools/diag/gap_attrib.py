"""GPU idle gaps of a rocprofv3 --kernel-trace --hip-trace run, attributed: for the last
N ms of kernels, every gap > --min-us with the kernel (and queue) before / after and the
non-launch HIP API calls issued on the host during [gap - 1 ms, gap end].
    python tools/diag/gap_attrib.py OUT_DIR [--last-ms 60] [--min-us 30]"""
import argparse
import csv
import glob
import os


def rows(root, pat):
    out = []
    for f in glob.glob(os.path.join(root, "**", pat), recursive=True):
        out.extend(csv.DictReader(open(f)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--last-ms", type=float, default=60.0)
    ap.add_argument("--min-us", type=float, default=30.0)
    a = ap.parse_args()
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70],
           r.get("Queue_Id", "?"), r.get("Correlation_Id", "?"))
          for r in rows(a.root, "*kernel_trace.csv")]
    ks.sort()
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"],
            r.get("Correlation_Id", "?"))
           for r in rows(a.root, "*hip_api_trace.csv")
           if r["Function"] not in ("hipLaunchKernel", "hipStreamWaitEvent", "hipEventRecord",
                                    "hipGetDevice", "hipSetDevice", "hipGetLastError",
                                    "hipStreamGetCaptureInfo", "hipDeviceGetAttribute",
                                    "hipExtModuleLaunchKernel", "hipPeekAtLastError",
                                    "hipEventQuery", "hipStreamIsCapturing",
                                    "hipGetDeviceProperties", "hipModuleLaunchKernel")]
    api.sort()
    t_end = max(e for _, e, _, _, _ in ks)
    t0 = t_end - int(a.last_ms * 1e6)
    busy_until = None
    prev = None
    tot = 0.0
    for s, e, n, q, c in ks:
        if e < t0:
            busy_until = max(busy_until or e, e)
            prev = (s, e, n, q, c)
            continue
        if busy_until is not None and s > busy_until:
            gap = (s - busy_until) / 1e3
            if gap >= a.min_us and s >= t0:
                tot += gap
                print("gap %8.1f us at %9.3f ms | before [q%s] %s | after [q%s c%s] %s" % (
                    gap, (busy_until - t_end) / 1e6, prev[3], prev[2], q, c, n))
                for (as_, ae, fn, ac) in api:
                    if busy_until - 1_000_000 <= as_ <= s:
                        print("      api %9.3f ms  %7.1f us  %s  c%s" % (
                            (as_ - t_end) / 1e6, (ae - as_) / 1e3, fn, ac))
        if busy_until is None or e > busy_until:
            busy_until = e
            prev = (s, e, n, q, c)
    print("total gaps >= %.0f us in the last %.0f ms: %.1f us" % (a.min_us, a.last_ms, tot))


if __name__ == "__main__":
    main()
