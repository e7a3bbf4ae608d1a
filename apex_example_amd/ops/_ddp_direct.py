"""Gradients written straight into DDP bucket views.

Under ``parallel.DistributedDataParallel`` every parameter's ``.grad`` is a view into a
persistent flat bucket (csrc/torch/reducer.cpp).  Returning a fresh gradient from an
autograd Function makes AccumulateGrad launch an add kernel per parameter into that view
(ResNet-50: 55 bf16 conv weights + 106 fp32 BatchNorm affine tensors, ~0.8 ms per step on
MI355X, `profiles/resnet50_forced_collectives_r3.md`).  The own kernels instead
accumulate their final reduction into the view (one rounding) and announce the
parameter to the reducer on the current stream; autograd gets None for it (the
reducer's AccumulateGrad hook still fires and consumes the announcement).
``APEX_AMD_DDP_DIRECT_GRAD=0`` keeps the autograd path.
"""
from __future__ import annotations

import os

import torch

_ON = os.environ.get("APEX_AMD_DDP_DIRECT_GRAD", "1") == "1"


def slots(*params):
    """[(reducer, index)] when every param's .grad is a bucket view its reducer will take
    an early ready mark for this iteration, else None."""
    if not _ON:
        return None
    out = []
    for p in params:
        if p is None:
            return None
        slot = getattr(p, "_amd_ddp_slot", None)
        if slot is None or p.grad is None:
            return None
        red = slot[0]()
        if red is None or not red.async_ready_ok():
            return None
        out.append((red, slot[1]))
    if torch.cuda.is_current_stream_capturing():
        return None
    return out


def mark_ready(sl):
    """Announce the parameters of ``slots()`` as ready (accumulated on the compute
    stream, which every bucket launch waits for anyway: no per-parameter event)."""
    for red, i in sl:
        red.mark_ready_direct(i)
