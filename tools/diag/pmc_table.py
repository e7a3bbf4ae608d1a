#!/usr/bin/env python3
"""Per-kernel PMC summary of rocprofv3 counter-collection CSVs (one or more passes):
median per dispatch of each counter, plus derived ratios (wave-cycle shares, MFMA busy)."""
import collections
import csv
import statistics
import sys


def load(paths):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"]
                short = name.split("(")[0][:60]
                per[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    per = load(sys.argv[1:])
    for k, cs in per.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        print("==", k)
        for c in sorted(med):
            print("   %-28s %14.0f" % (c, med[c]))
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in med:
                    print("   %-28s %6.1f %% of wave cycles" % (c, 100 * med[c] / wc))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in med and "SQ_BUSY_CYCLES" in med:
            # busy cycles are per SE (32) x 4 SIMD...; report raw ratio and GRBM-normalised
            g = med.get("GRBM_GUI_ACTIVE")
            if g:
                print("   MFMA busy / (GRBM x 1024 SIMDs) %6.1f %%" % (
                    100 * med["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024)))
        if "SQ_LDS_BANK_CONFLICT" in med and "SQ_LDS_IDX_ACTIVE" in med and med["SQ_LDS_IDX_ACTIVE"]:
            print("   LDS bank conflict share %6.1f %%" % (
                100 * med["SQ_LDS_BANK_CONFLICT"] / med["SQ_LDS_IDX_ACTIVE"]))


if __name__ == "__main__":
    main()
