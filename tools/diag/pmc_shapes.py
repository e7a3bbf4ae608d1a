#!/usr/bin/env python3
"""Per (kernel, grid) PMC summary of rocprofv3 counter CSVs: duration, FETCH_SIZE-derived
HBM rate (x2, the gfx950 FETCH_SIZE halving), wave-cycle shares, mean VMEM latency, TA busy,
L2 hit rate.  Usage: pmc_shapes.py pmc_*.csv [--match amd::]"""
import collections
import csv
import re
import statistics
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    base = n.split("(")[0]
    return base[:70]


def main():
    files = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = "amd::"
    for a in sys.argv[1:]:
        if a.startswith("--match="):
            match = a.split("=", 1)[1]
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if match not in n:
                continue
            key = (short(n), r["Grid_Size"])
            rows[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for key, cs in sorted(rows.items()):
        m = {c: statistics.median(v) for c, v in cs.items()}
        us = statistics.median(dur[key]) / 1e3
        wc = m.get("SQ_WAVE_CYCLES", 0)
        out = ["%s grid %s" % key, "%.1f us" % us]
        if "FETCH_SIZE" in m:
            out.append("fetch %.0f MB (x2: %.2f TB/s)" % (
                2 * m["FETCH_SIZE"] / 1e3, 2 * m["FETCH_SIZE"] * 1e3 / (us * 1e-6) / 1e12))
        if wc:
            out.append("wait %.0f%% issue %.0f%% active %.0f%%" % (
                100 * m["SQ_WAIT_ANY"] / wc, 100 * m["SQ_WAIT_INST_ANY"] / wc,
                100 * m["SQ_ACTIVE_INST_ANY"] / wc))
        if m.get("SQ_INSTS_VMEM_RD"):
            out.append("vmem level/inst %.0f" % (m["SQ_INST_LEVEL_VMEM"] / m["SQ_INSTS_VMEM_RD"]))
        if "TA_BUSY_sum" in m and m.get("GRBM_GUI_ACTIVE"):
            out.append("TA busy %.0f%%" % (100 * m["TA_BUSY_sum"] / (m["GRBM_GUI_ACTIVE"] / 8 * 256)))
            out.append("TA stalled by TC %.0f%%" % (
                100 * m["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / max(1.0, m["TA_BUSY_sum"])))
        if "TCC_HIT_sum" in m:
            out.append("L2 hit %.0f%%" % (100 * m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])))
        if "SQ_LEVEL_WAVES" in m and m.get("GRBM_GUI_ACTIVE"):
            out.append("waves/CU %.1f" % (m["SQ_LEVEL_WAVES"] / (m["GRBM_GUI_ACTIVE"] / 8) / 256 * 4))
        print(" | ".join(out))


if __name__ == "__main__":
    main()
