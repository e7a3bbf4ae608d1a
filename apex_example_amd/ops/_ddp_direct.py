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

An announcement is only sound when that ONE use of the parameter produces its whole
gradient for the iteration.  So (a) the DDP wrapper excludes parameters listed more than
once in the module tree (tied weights, ``Reducer.set_no_direct``); (b) the own ops count
their forward uses of each parameter (``note_use``) and go direct only for a parameter
used exactly once in the current forward (a module called twice takes the autograd path,
which sums both uses before one AccumulateGrad); a count starts at the first DDP forward
after a completed backward (``forward_epoch``; the reducer counts backwards under
``no_sync`` too), so several DDP forwards feeding ONE backward (siamese / contrastive
losses) share one count and take the autograd path, while gradient-accumulation
micro-steps and grad-free eval forwards in between do not disturb it; (c) the reducer refuses a second announcement, and the ready
mark itself comes from the AccumulateGrad hook after every use has been summed, so an
autograd gradient of some other use still lands in the view before the bucket launches
(the parameter is excluded from the direct path from then on).
"""
from __future__ import annotations

import os

import torch

_ON = os.environ.get("APEX_AMD_DDP_DIRECT_GRAD", "1") == "1"
# lazy zeroing of bucket-view gradients (APEX_AMD_DDP_LAZY_ZERO=0: a zero kernel per step)
_LAZY = os.environ.get("APEX_AMD_DDP_LAZY_ZERO", "1") == "1"


_EPOCH = {}  # id(reducer) -> (use-count epoch, reducer.backwards() when it started)


def forward_epoch(red):
    """DistributedDataParallel.forward: start a new use count for ``red``'s parameters
    if a backward has completed since the current count started, else keep counting
    (two forwards before one backward: each parameter then shows two uses)."""
    b = red.backwards()
    e = _EPOCH.get(id(red))
    if e is None or e[1] != b:
        _EPOCH[id(red)] = ((e[0] + 1) if e is not None else 1, b)


def _epoch(red):
    e = _EPOCH.get(id(red))
    return e[0] if e is not None else 0


def note_use(*params):
    """Count one forward use of each DDP-registered parameter in this iteration (called
    by the own ops' forwards for the parameters they may later announce)."""
    if not _ON:
        return
    for p in params:
        slot = getattr(p, "_amd_ddp_slot", None) if p is not None else None
        if slot is None:
            continue
        red = slot[0]()
        if red is None:
            continue
        it = _epoch(red)
        u = getattr(p, "_amd_ddp_uses", None)
        p._amd_ddp_uses = (it, u[1] + 1) if (u is not None and u[0] == it) else (it, 1)


def slot(p):
    """(reducer, index) when ``p.grad`` is a bucket view (or the bucket view was lazily
    zeroed, ``grad_target``) its reducer will take an early ready mark for this iteration
    and ``p`` had exactly one counted forward use, else None."""
    s = getattr(p, "_amd_ddp_slot", None) if p is not None else None
    if s is None:
        return None
    red = s[0]()
    if red is None or not red.async_ready_ok() or not red.direct_ok(s[1]):
        return None
    if p.grad is None and red.lazy_view(s[1]) is None:
        return None
    u = getattr(p, "_amd_ddp_uses", None)
    if u is None or u[1] != 1 or u[0] != _epoch(red):
        return None
    return red, s[1]


def slots(*params):
    """[(reducer, index)] when every param's .grad is a bucket view its reducer will take
    an early ready mark for this iteration (``slot``), else None."""
    if not _ON:
        return None
    out = []
    for p in params:
        sl = slot(p)
        if sl is None:
            return None
        out.append(sl)
    if params[0].is_cuda and torch.cuda.is_current_stream_capturing():
        return None
    return out


def grad_target(p):
    """(tensor, accumulate) where a direct-path kernel puts ``p``'s gradient (after
    ``slot(p)`` succeeded): ``p.grad`` to accumulate into, or - the bucket was lazily
    zeroed by the optimizer's zero_grad (csrc/torch/reducer.cpp lazy_zero) - the stale
    bucket view to OVERWRITE (beta = 0; no memset of the buckets per step)."""
    g = p.grad
    if g is not None:
        return g, True
    s = p._amd_ddp_slot
    return s[0]().lazy_view(s[1]), False


def lazy_zero(params):
    """zero_grad for bucket-view gradients: detach them from their views and mark the
    views stale (the reducer's lazy_zero) where the reducer sees the next backward
    through; returns the gradients that still need a zeroing kernel."""
    rest = []
    by_red = {}
    for p in params:
        s = getattr(p, "_amd_ddp_slot", None) if _LAZY else None
        red = s[0]() if s is not None else None
        if red is None or p.grad is None or not red.lazy_zero_ok():
            if p.grad is not None:
                rest.append(p.grad)
            continue
        ent = by_red.setdefault(id(red), (red, []))
        ent[1].append(s[1])
    for red, idx in by_red.values():
        red.lazy_zero(idx)
    return rest


def mark_ready(sl):
    """Announce the parameters of ``slots()`` as ready (accumulated on the compute
    stream, which every bucket launch waits for anyway: no per-parameter event)."""
    for red, i in sl:
        red.mark_ready_direct(i)
