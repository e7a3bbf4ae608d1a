"""Loader for the in-tree native extension ``apex_example_amd._C``.

The extension is built in-tree by ``tools/build_ext.py`` (hipcc for the gfx950
kernels, g++ for the torch bindings).  It contains both the HIP kernels and the
C++ CPU paths, so it imports on CPU-only hosts as well.

On a machine with a GPU a missing extension is an error (``require()`` raises):
GPU code paths never silently fall back to eager PyTorch.  Set
``APEX_AMD_ALLOW_PYTHON_FALLBACK=1`` to permit the pure-Python reference paths
(used by tests that compare the two, mirroring apex's "Python fallback"
installs without --cpp_ext/--cuda_ext).
"""
from __future__ import annotations

import importlib
import os

_C = None
_err: Exception | None = None


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return _C
    try:
        _C = importlib.import_module("apex_example_amd._C")
    except Exception as e:  # pragma: no cover - exercised only without a build
        _err = e
    else:
        # 3x3 stride-1 convs on the halo-resident kernel (csrc/hip/conv_igemm.hip conv3h_k):
        # APEX_AMD_CONV_HALO = 0 off, 1 automatic (default), 64 / 128 force that tile width
        # (A/B switch, docs/KNOBS.md)
        _C.conv.set_halo(int(os.environ.get("APEX_AMD_CONV_HALO", "1")))
        # its pixel-tile height: 0 = per-shape cost model (default), 224 / 256 force one
        _C.conv.set_halo_mtile(int(os.environ.get("APEX_AMD_CONV_HALO_BM", "0")))
        # conv_tap_k tile order (N tiles fastest): 0 off, 1 by shape (default), 2 all
        _C.conv.set_nfast(int(os.environ.get("APEX_AMD_CONV_NFAST", "1")))
        _C.conv.set_halo_nfast(int(os.environ.get("APEX_AMD_CONV_HALO_NFAST", "0")))
        # stride-1 1x1 forwards with Cout % 256 on gemm4w (statistics epilogue):
        # APEX_AMD_CONV_1X1_G4W = 0 off (default: slower in the model, see conv_igemm.hip),
        # 1 the per-shape winners, 2 every eligible shape
        _C.conv.set_1x1_gemm4w(int(os.environ.get("APEX_AMD_CONV_1X1_G4W", "0")))
    return _C


def available() -> bool:
    return _load() is not None


def python_fallback_allowed() -> bool:
    return os.environ.get("APEX_AMD_ALLOW_PYTHON_FALLBACK", "0") == "1"


def require():
    """Return the native module or raise a loud error."""
    C = _load()
    if C is None:
        raise RuntimeError(
            "apex_example_amd native extension is not built (%r). Run "
            "`python tools/build_ext.py` (hipcc --offload-arch=gfx950)." % (_err,))
    return C


def get():
    """Return the native module or None (only when Python fallback is allowed)."""
    C = _load()
    if C is None and not python_fallback_allowed():
        require()
    return C
