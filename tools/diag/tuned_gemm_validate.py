#!/usr/bin/env python3
"""Numerical check of EVERY entry of the committed TunableOp tables.

For each row of tuning/<name>.csv the exact GEMM the row keys on is rebuilt
(apex_example_amd.utils.gemm_tuning.key_operands: same transposes, M/N/K and leading
dimensions), run once with TunableOp off (library default) and once with the table
loaded (the tuned solution), and both are compared with an fp64 reference of the
same operands:

    err = max |C - C_ref| / max |C_ref|

Results go to a JSON list (one record per row).  Whether the tuned run really used the
table is shown by TunableOp's own log: run with PYTORCH_TUNABLEOP_VERBOSE=3 and
PYTORCH_TUNABLEOP_VERBOSE_FILENAME=<file>; every hit logs "ResultEntry found for
<op>,<params>" (tests/test_gemm_tuning_gpu.py does this and checks every key).

    python tools/diag/tuned_gemm_validate.py --out gpurun_out/tuned.json resnet50 bert_large
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from apex_example_amd.utils import gemm_tuning as gt  # noqa: E402


def _err(c, ref):
    c = c.double()
    finite = bool(torch.isfinite(c).all())
    scale = ref.abs().max().item()
    err = (c - ref).abs().max().item() / max(scale, 1e-30) if finite else float("inf")
    return err, finite


def validate(names, device):
    out = []
    for name in names:
        path = gt.tuning_path(name)
        rows = gt.table_rows(path)
        for i, (op, sig, sol) in enumerate(rows):
            key = gt.parse_key(op, sig)
            P, Q, bias = gt.key_operands(key, device, seed=1000 + i)
            ref = gt.reference_fp64(P, Q, bias)
            torch.cuda.tunable.enable(False)
            c0 = gt.run_key(P, Q, bias)
            torch.cuda.synchronize()
            loaded = gt.use_tuned_gemms(name)
            c1 = gt.run_key(P, Q, bias)
            torch.cuda.synchronize()
            torch.cuda.tunable.enable(False)
            e0, f0 = _err(c0, ref)
            e1, f1 = _err(c1, ref)
            rec = {"table": name, "op": op, "params": sig, "solution": sol,
                   "loaded": loaded is not None, "untuned_err": e0, "tuned_err": e1,
                   "untuned_finite": f0, "tuned_finite": f1,
                   "bitwise_equal": bool(torch.equal(c0, c1))}
            out.append(rec)
            print("%-12s %-34s %-34s %-22s untuned %.2e tuned %.2e%s" % (
                name, op, sig, sol, e0, e1, "" if f1 else "  NON-FINITE"), flush=True)
            del P, Q, bias, ref, c0, c1
            torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="*", default=["resnet50", "bert_large", "gpt2_medium"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # the reference is fp64; keep fp32 GEMMs exact-ish too
    torch.backends.cuda.matmul.allow_tf32 = False
    res = validate(a.names, dev)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
