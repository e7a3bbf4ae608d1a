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
