"""Every committed TunableOp entry, run as the exact GEMM it keys on, against an fp64
reference (TunableOp picks the fastest solution with no numerical
check, and round 2 shipped one that returned non-finite values).

The check runs tools/diag/tuned_gemm_validate.py in a child process with TunableOp's
verbose log on, so the test also proves that each tuned run HIT its table entry
("ResultEntry found for <op>,<params>") instead of silently running the default."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# max |C - C_ref| / max |C_ref| for fp32-accumulated GEMMs: one rounding of the output
# (unit roundoff bf16 2^-8, fp16 2^-11) with a 2x / 4x margin.  Measured on MI355X
# (ResNet-50 table): 1.8e-3 .. 3.5e-3 for bf16, tuned == untuned bitwise on every row.
BOUND = {"BFloat16": 2 ** -7, "Half": 2 ** -9}


@pytest.mark.parametrize("name", ["resnet50", "bert_large", "gpt2_medium"])
def test_every_tuned_entry_is_numerically_sound(tmp_path, name):
    from apex_example_amd.utils import gemm_tuning as gt

    path = gt.tuning_path(name)
    if gt.validators_match(path) is not None:
        pytest.skip("table validators do not match this stack: %s" % gt.validators_match(path))
    out, log = tmp_path / "res.json", tmp_path / "tunableop.log"
    env = dict(os.environ, PYTORCH_TUNABLEOP_VERBOSE="3",
               PYTORCH_TUNABLEOP_VERBOSE_FILENAME=str(log))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "diag",
                                                     "tuned_gemm_validate.py"),
                        name, "--out", str(out)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    recs = json.loads(out.read_text())
    rows = gt.table_rows(path)
    assert len(recs) == len(rows) > 0
    text = log.read_text() if log.exists() else ""
    bad = []
    for r in recs:
        bound = BOUND[r["op"].split("_")[1]]
        if not (r["loaded"] and r["tuned_finite"] and r["tuned_err"] <= bound
                and r["untuned_finite"] and r["untuned_err"] <= bound):
            bad.append(r)
        # the tuned call looked the key up in the loaded table
        assert "ResultEntry found for %s,%s" % (r["op"], r["params"]) in text, (
            r["op"], r["params"], text[-2000:])
    assert not bad, json.dumps(bad, indent=1)
    print(p.stdout)
