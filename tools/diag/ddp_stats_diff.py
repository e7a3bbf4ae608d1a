#!/usr/bin/env python3
"""Which side moves when the conv-epilogue BN statistics are on: the 2-rank DDP + SyncBN
run (tests/dist_workers.gpu_ddp_resnet) or the one-process reference on the concatenated
batch (gpu_resnet_reference)?  Runs each with APEX_AMD_CONV_BN_STATS=1 / 0 in child
processes and prints the worst per-parameter update difference after step 1 between
every pair (tests/test_ddp_gpu.py::test_two_ranks_match_concatenated_batch[O2]).

    python tools/diag/ddp_stats_diff.py          # DDP_DIFF_HW=64: 64x64 images
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


HW = int(os.environ.get("DDP_DIFF_HW", "32"))


def child(kind, out):
    import torch

    import dist_workers as W

    if kind == "ddp":
        res = W.run("gpu_ddp_resnet", 2, tempfile.mkdtemp(), syncbn=True, lr=0.01,
                    opt_level="O2", steps=2, hw=HW)
        r = {"masters1": res[0]["masters1"], "losses": [(a + b) / 2 for a, b in
                                                       zip(res[0]["losses"], res[1]["losses"])]}
    else:
        ref = W.gpu_resnet_reference(world=2, lr=0.01, opt_level="O2", steps=2, hw=HW)
        r = {"masters1": ref["masters1"], "losses": ref["losses"], "p0": ref["params0"]}
    torch.save(r, out)


def main():
    if len(sys.argv) > 2:
        child(sys.argv[1], sys.argv[2])
        return
    import torch

    runs = {}
    d = tempfile.mkdtemp()
    for kind in ("ddp", "ref"):
        for stats in ("1", "0"):
            out = os.path.join(d, "%s_%s.pt" % (kind, stats))
            env = dict(os.environ, APEX_AMD_CONV_BN_STATS=stats)
            p = subprocess.run([sys.executable, os.path.abspath(__file__), kind, out], env=env,
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stdout[-2000:], p.stderr[-3000:])
                sys.exit(p.returncode)
            runs["%s_stats%s" % (kind, stats)] = torch.load(out, weights_only=False)
            print("%s stats=%s losses %s" % (kind, stats, runs["%s_stats%s" % (kind, stats)]["losses"]),
                  flush=True)
    p0 = runs["ref_stats0"]["p0"]
    names = list(runs)
    for i in range(len(names)):
        for j in range(i + 1, len(names)):
            a, b = runs[names[i]]["masters1"], runs[names[j]]["masters1"]
            worst, wi = 0.0, -1
            for k, (u, v, q) in enumerate(zip(a, b, p0)):
                du, dv = u - q, v - q
                rel = float((du - dv).abs().max() / (dv.abs().max() + 1e-12))
                if rel > worst:
                    worst, wi = rel, k
            da = torch.cat([(u - q).flatten() for u, q in zip(a, p0)])
            db = torch.cat([(v - q).flatten() for v, q in zip(b, p0)])
            l2 = float((da - db).norm() / db.norm())
            print("%-12s vs %-12s worst per-tensor update rel diff %.3e at param %d %s; "
                  "whole-update rel L2 %.3e" % (names[i], names[j], worst, wi,
                                                tuple(p0[wi].shape), l2))


if __name__ == "__main__":
    main()
