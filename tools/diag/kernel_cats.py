#!/usr/bin/env python3
"""Per-step kernel time by category from rocprof_summary.py --names-out TSVs
(calls, us/step, name): conv (own convs, their weight gradients, library GEMMs), BN
passes, the rest.  Usage: kernel_cats.py a_names.tsv [b_names.tsv ...]"""
import sys

CATS = [
    ("conv fwd/dgrad (own)", ("conv_tap_k", "stem_fwd_k")),
    ("conv wgrad (own)", ("conv3x3_wgrad", "stem_wgrad", "wgrad_reduce", "splitk")),
    ("library GEMM (1x1)", ("Cijk",)),
    ("BN", ("apply_k", "backward_k", "reduce_k", "stats_k", "slab_fold", "reduce_finalize",
            "stats_from_rows", "stats_finalize", "bn_")),
    ("pool/stem BN", ("maxpool", "stem_pad", "stem_bn")),
    ("optimizer", ("sgd", "adam", "lamb", "l2norm", "multi_tensor")),
]


def cat_of(name):
    for c, keys in CATS:
        if any(k in name for k in keys):
            return c
    return "other"


def main():
    for p in sys.argv[1:]:
        tot = {}
        for line in open(p):
            calls, us, name = line.rstrip("\n").split("\t", 2)
            c = cat_of(name)
            tot[c] = tot.get(c, 0.0) + float(us)
        print("%s: %s; sum %.1f us/step" % (p, ", ".join("%s %.1f" % kv for kv in sorted(tot.items())),
                                             sum(tot.values())))


if __name__ == "__main__":
    main()
