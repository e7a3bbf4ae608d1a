"""Sync-free overflow skipping for NON-fused optimizers (torch.optim.SGD & co.).

Apex decides "skip this step?" on the host: ``update_scale()`` reads the overflow
flag back (one device->host sync per iteration) and swaps
``optimizer.step`` for a no-op.  For a small model that sync serialises the host and
the GPU: the reference program (test_apex_distributed_spawn.py:119-164, torch SGD
under amp O2) measured 2.0 ms/step on MI355X, slower than the stock GradScaler path.

The fused optimizers of this package skip on the device (their kernels read the flag).
Any other optimizer gets a *step guard* instead: a snapshot of the tensors the step
may write (the (master) parameters and every CUDA tensor of their optimizer state) is
copied on the device before the step (one multi-tensor launch), the optimizer's own
step runs unconditionally, and a second launch (``mt.copy_if``) copies the snapshot
back iff the overflow flag is set - bitwise the same result as not stepping, with no
host round trip.  The loss scaler runs in its sync-free mode and prints the Apex
overflow message asynchronously.

Exactness conditions, checked per step:
  * every state value is a CUDA tensor or None (no host-side counters such as
    Adam's CPU ``step``: those would advance on a skipped step) - otherwise the step
    falls back to one host read of the flag;
  * a step that CREATES state (torch SGD's momentum buffer, first step) also reads
    the flag on the host once and, on overflow, drops the new state entries (the
    skipped step must not initialise them).
``APEX_AMD_GUARDED_STEP=0`` keeps Apex's host-synchronous skip for such optimizers.
"""
from __future__ import annotations

import os

import torch

from .. import _native

ENABLED = os.environ.get("APEX_AMD_GUARDED_STEP", "1") == "1"


def guardable(optimizer):
    from ..parallel.LARC import LARC

    return (ENABLED and isinstance(optimizer, torch.optim.Optimizer)
            and not isinstance(optimizer, LARC) and not getattr(optimizer, "_amp_fused", False))


def _state_tensors(opt, params):
    """(tensors, host_only): the CUDA tensors of the params' state, and whether some
    state value lives on the host (a counter the guard cannot roll back)."""
    ts, host = [], False
    for p in params:
        st = opt.state.get(p)
        if not st:
            continue
        for v in st.values():
            if v is None:
                continue
            if torch.is_tensor(v) and v.is_cuda:
                ts.append(v)
            else:
                host = True
    return ts, host


def install(optimizer):
    """Wrap ``optimizer.step`` (the optimizer's own step, before amp patches it)."""
    inner = optimizer.step
    cache = {}

    def guarded_step(*args, **kwargs):
        stash = getattr(optimizer, "_amp_stash", None)
        sc = getattr(stash, "last_scaler", None) if stash is not None else None
        if sc is None or not sc.sync_free or not sc.dynamic:
            return inner(*args, **kwargs)
        flag = sc._overflow_buf
        params = [p for g in optimizer.param_groups for p in g["params"]
                  if p.grad is not None and p.is_cuda]
        if not params:
            return inner(*args, **kwargs)
        states, host = _state_tensors(optimizer, params)
        if host:
            # host-side state (e.g. Adam's CPU step count): Apex's host decision
            if int(flag.item()):
                return None
            return inner(*args, **kwargs)
        tensors = params + states
        key = tuple(map(id, tensors))
        snap = cache.get("snap")
        if cache.get("key") != key:
            snap = [torch.empty_like(t) for t in tensors]
            cache["key"], cache["snap"] = key, snap
            cache["dummy"] = torch.zeros(1, dtype=torch.int32, device=flag.device)
        mt = _native.require().mt
        mt.scale_any(cache["dummy"], [[t.detach() for t in tensors], snap], 1.0)
        before = {id(p): set(optimizer.state[p].keys()) if p in optimizer.state else set()
                  for p in params}
        out = inner(*args, **kwargs)
        mt.copy_if(flag, [snap, [t.detach() for t in tensors]])
        created = [p for p in params
                   if (set(optimizer.state[p].keys()) if p in optimizer.state else set())
                   - before[id(p)]]
        if created:
            new_ts, _ = _state_tensors(optimizer, created)
            if new_ts and int(flag.item()):  # first step of lazily created state
                for p in created:
                    for k in set(optimizer.state[p].keys()) - before[id(p)]:
                        del optimizer.state[p][k]
        return out

    optimizer.step = guarded_step
    optimizer._amp_step_guard = True
    return optimizer
