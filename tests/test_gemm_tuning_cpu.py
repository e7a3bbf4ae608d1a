"""GEMM tuning tables (apex_example_amd.utils.gemm_tuning): CSV parsing, the
committed tables' shape, and the no-GPU behaviour (nothing enabled)."""
import glob
import os

import torch

from apex_example_amd.utils import gemm_tuning as gt


def _write(tmp_path, rows):
    p = tmp_path / "t.csv"
    p.write_text("\n".join(",".join(r) for r in rows) + "\n")
    return str(p)


def test_parse_validators_and_entries(tmp_path):
    p = _write(tmp_path, [
        ("Validator", "PT_VERSION", "2.10.0"),
        ("Validator", "GCN_ARCH_NAME", "gfx950:sramecc+:xnack-"),
        ("GemmTunableOp_BFloat16_TN", "tn_64_802816_64_ld_64_64_64", "Gemm_Hipblaslt_1", "0.06"),
        ("GemmTunableOp_BFloat16_NN", "nn_64_802816_64_ld_64_64_64", "Default", "0.07"),
    ])
    assert gt.file_validators(p) == {"PT_VERSION": "2.10.0",
                                     "GCN_ARCH_NAME": "gfx950:sramecc+:xnack-"}
    assert gt.tuned_entries(p) == 2


def test_no_gpu_keeps_tunableop_off():
    if torch.cuda.is_available():
        return
    assert gt.use_tuned_gemms("resnet50") is None
    assert gt.use_tuned_gemms("no_such_table") is None


def test_committed_tables_are_gfx950():
    for p in glob.glob(os.path.join(gt.TUNING_DIR, "*.csv")):
        v = gt.file_validators(p)
        assert v.get("GCN_ARCH_NAME", "").startswith("gfx950"), p
        assert "HIPBLASLT_VERSION" in v and "PT_VERSION" in v, p
        assert gt.tuned_entries(p) > 0, p
