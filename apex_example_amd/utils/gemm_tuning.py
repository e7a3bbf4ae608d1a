"""Offline-tuned library GEMM selections (PyTorch TunableOp over rocBLAS/hipBLASLt).

The plain library GEMMs of the training step (ResNet's stride-1 1x1 convs on
channels-last tensors, the transformer dense layers, the LM / MLM heads) go
through ``at::cuda::blas::gemm``.  With TunableOp enabled, each (op, transpose,
M, N, K, ld) key is looked up in a results table; a hit runs the rocBLAS or
hipBLASLt solution that measured fastest for exactly that shape on gfx950, a
miss runs the untuned default.  The tables live in ``tuning/<name>.csv`` and
are produced by ``tools/tune_gemms.sh`` on an MI355X (tuning in situ, inside
the real training step, so cache and clock state match the workload).

Tuning is never switched on here: ``use_tuned_gemms`` enables TunableOp
read-only.  The CSV's validator lines (PyTorch, HIP, rocBLAS, hipBLASLt and
gfx arch) are compared with the running stack first; on any mismatch the file
is not loaded and every GEMM keeps the default heuristic (no silent use of
selections tuned for another library build).
"""
from __future__ import annotations

import csv
import os
from typing import Dict, Optional

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TUNING_DIR = os.path.join(ROOT, "tuning")


def tuning_path(name: str) -> str:
    return os.path.join(TUNING_DIR, name + ".csv")


def file_validators(path: str) -> Dict[str, str]:
    out = {}
    with open(path, newline="") as f:
        for row in csv.reader(f):
            if len(row) >= 3 and row[0] == "Validator":
                out[row[1]] = row[2]
    return out


def _running_validators() -> Dict[str, str]:
    try:
        return {k: v for k, v in torch.cuda.tunable.get_validators()}
    except Exception:  # older torch: tuple-of-tuples or unavailable
        return {}


def validators_match(path: str) -> Optional[str]:
    """None if the file's validators agree with the running stack, else a reason."""
    want = file_validators(path)
    have = _running_validators()
    if not have:
        return "TunableOp validators unavailable on this build"
    for k, v in want.items():
        if k in have and have[k] != v:
            return "%s: file %s, running %s" % (k, v, have[k])
    return None


def use_tuned_gemms(name: str) -> Optional[str]:
    """Enable TunableOp read-only with ``tuning/<name>.csv``.

    Returns the path loaded, or None (file absent, no GPU, not a ROCm build, or
    validator mismatch).  Safe to call on every rank: nothing is ever written.
    """
    path = tuning_path(name)
    if not (os.path.exists(path) and torch.cuda.is_available() and torch.version.hip):
        return None
    t = torch.cuda.tunable
    t.tuning_enable(False)
    t.enable(True)
    why = validators_match(path)
    if why is not None:
        t.enable(False)
        if os.environ.get("APEX_AMD_VERBOSE"):
            print("[gemm_tuning] not using %s (%s)" % (path, why))
        return None
    t.set_filename(path, insert_device_ordinal=False)
    if not t.read_file(path):
        t.enable(False)
        return None
    return path


def tuned_entries(path: str) -> int:
    with open(path, newline="") as f:
        return sum(1 for row in csv.reader(f) if row and row[0] != "Validator")


# ---------------------------------------------------------------- per-entry validation
# TunableOp picks the fastest solution of each key WITHOUT a numerical check (round 2
# shipped one selection that returned non-finite values).  The helpers below rebuild the
# exact GEMM a table row keys on, so every committed entry can be run against an fp64
# reference (tools/diag/tuned_gemm_validate.py, tests/test_gemm_tuning_gpu.py).

_DTYPES = {"BFloat16": torch.bfloat16, "Half": torch.float16, "Float": torch.float32}


def table_rows(path: str):
    """[(op_signature, params_signature, solution)] of the non-validator rows."""
    with open(path, newline="") as f:
        return [(r[0], r[1], r[2]) for r in csv.reader(f) if len(r) >= 3 and r[0] != "Validator"]


def parse_key(op_sig: str, params_sig: str) -> dict:
    """'GemmTunableOp_BFloat16_TN', 'tn_M_N_K_ld_lda_ldb_ldc' -> fields (BLAS column-major
    convention: C[m x n] = op(A) op(B), op(A) m x k)."""
    kind, dt, _ = op_sig.split("_", 2)
    f = params_sig.split("_")
    if len(f) != 8 or f[4] != "ld":
        raise ValueError("unsupported TunableOp key %r" % params_sig)
    return {"bias": kind == "GemmAndBiasTunableOp", "dtype": _DTYPES[dt],
            "transa": f[0][0], "transb": f[0][1], "m": int(f[1]), "n": int(f[2]),
            "k": int(f[3]), "lda": int(f[5]), "ldb": int(f[6]), "ldc": int(f[7])}


def key_operands(key: dict, device, seed: int = 0):
    """Row-major operands (P [n x k], Q [k x m], bias [m] or None) whose
    ``torch.mm(P, Q)`` / ``torch.addmm(bias, P, Q)`` (result [n x m]) is exactly the
    key's column-major GEMM: Q plays BLAS A (transa 'n': Q has row stride lda; 't':
    Q = W.t() with W [m x k] of row stride lda), P plays BLAS B (transb 'n': row
    stride ldb; 't': P = V.t() with V [k x n] of row stride ldb)."""
    g = torch.Generator(device=device).manual_seed(seed)
    dt = key["dtype"]
    m, n, k = key["m"], key["n"], key["k"]

    def rnd(rows, cols):
        return torch.randn(rows, cols, generator=g, device=device, dtype=torch.float32).to(dt)

    Q = rnd(k, key["lda"])[:, :m] if key["transa"] == "n" else rnd(m, key["lda"])[:, :k].t()
    P = rnd(n, key["ldb"])[:, :k] if key["transb"] == "n" else rnd(k, key["ldb"])[:, :n].t()
    bias = rnd(1, m)[0].contiguous() if key["bias"] else None
    return P, Q, bias


def run_key(P, Q, bias):
    return torch.addmm(bias, P, Q) if bias is not None else torch.mm(P, Q)


def reference_fp64(P, Q, bias):
    out = P.double() @ Q.double()
    return out + bias.double() if bias is not None else out
