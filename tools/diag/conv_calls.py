#!/usr/bin/env python3
"""Per-call table of one ResNet-50 step's convolution dispatches from a serialized
rocprofv3 dispatch list (tools/gpu_runs/r5/conv_dispatch.sh -> dispatch.tsv: start, name,
grid x/y/z, workgroup, us).  Groups the own implicit-GEMM conv dispatches by (phase,
mode, output pixels M, output channels, epilogue) and the other conv-side kernels by
name, for one step (the first timed step: dispatches between two stem forwards)."""
import collections
import re
import sys

MODES = {0: "3x3 s1/s2 fwd (or s1 dgrad)", 1: "1x1 fwd (or s1 dgrad)", 2: "3x3 s2 dgrad", 3: "1x1 s2 dgrad"}
HW = {802816: 56, 200704: 28, 50176: 14, 12544: 7, 3211264: 112}


def main():
    rows = [l.rstrip("\n").split("\t") for l in open(sys.argv[1])]
    rows = [(int(r[0]), r[1], int(r[2]), int(r[3]), int(r[4]), int(r[5]), float(r[6])) for r in rows]
    rows.sort()
    stems = [i for i, r in enumerate(rows) if "stem_fwd_k" in r[1]]
    if len(stems) >= 2:
        rows = rows[stems[0]:stems[1]]
    # backward starts at the first weight-gradient kernel
    bwd0 = next((i for i, r in enumerate(rows) if "wgrad" in r[1] or "Cijk_Ailk_Bjlk_BSS" in r[1]), len(rows))
    groups = collections.OrderedDict()
    other = collections.OrderedDict()
    for i, (s, name, gx, gy, gz, wg, us) in enumerate(rows):
        phase = "fwd" if i < bwd0 else "bwd"
        m = re.search(r"conv_tap_kILi(\d)ELi(\d+)ELi(\d+)ELi(\d)ELi(\d)ELi(\d)ELi(\d)ELi(\d+)ELi(\d+)E", name)
        if m:
            mode, bm, bn, wm, wn, nb, epi, ct, bk = map(int, m.groups())
            mt = gx // ct
            M = mt * bm
            key = (phase, mode, M, gy * bn, epi, "%dx%d nb%d bk%d" % (bm, bn, nb, bk))
            g = groups.setdefault(key, [0, 0.0])
            g[0] += 1
            g[1] += us
        else:
            k = (phase, re.sub(r"^_Z.*?(\w+_k)I.*$", r"\1", name)[:70], gx, gy, gz)
            g = other.setdefault(k, [0, 0.0])
            g[0] += 1
            g[1] += us
    print("| phase | kernel (mode) | M (tiles x BM) | out ch | BN-bwd epilogue | tile | calls | us total | us/call |")
    print("|---|---|---|---|---|---|---|---|---|")
    tot = 0.0
    for (phase, mode, M, nc, epi, tile), (n, us) in groups.items():
        hw = min(HW, key=lambda v: abs(v - M))
        print("| %s | %s | %d (@%d) | %d | %s | %s | %d | %.1f | %.1f |" % (
            phase, MODES[mode], M, HW[hw], nc, "yes" if epi else "", tile, n, us, us / n))
        tot += us
    print("\nown implicit-GEMM conv kernels: %.1f us per step\n" % tot)
    print("| phase | other conv-side kernel | grid | calls | us total |")
    print("|---|---|---|---|---|")
    tot2 = 0.0
    for (phase, name, gx, gy, gz), (n, us) in other.items():
        print("| %s | %s | %d x %d x %d | %d | %.1f |" % (phase, name, gx, gy, gz, n, us))
        tot2 += us
    print("\nother conv-side kernels: %.1f us per step; all: %.1f us" % (tot2, tot + tot2))


if __name__ == "__main__":
    main()
