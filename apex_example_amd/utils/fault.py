"""Deterministic fault injection for the numerical-failure path.

Apex's tests poison gradients by hand; this makes the same thing a switch, so a
training script can be driven through the overflow-skip path without edits:

    APEX_AMD_INJECT="inf@step=5"                  every rank, step 5, first grad
    APEX_AMD_INJECT="nan@step=3,rank=1,param=7"   rank 1 only, 8th grad in the list
    APEX_AMD_INJECT="inf@step=2,every=10"         steps 2, 12, 22, ...

``step`` counts ``amp.scale_loss`` exits (backward passes) from 0.  The value
is written into element 0 of the chosen gradient right after backward and
before amp's unscale / overflow check, i.e. exactly where a real fp16
overflow would appear.  Python API: :func:`configure` / :func:`disable`.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch


@dataclass
class FaultSpec:
    value: float
    step: int
    rank: Optional[int] = None
    param: int = 0
    every: int = 0

    def fires(self, step: int, rank: int) -> bool:
        if self.rank is not None and rank != self.rank:
            return False
        if self.every > 0:
            return step >= self.step and (step - self.step) % self.every == 0
        return step == self.step


def parse(spec: str) -> FaultSpec:
    """Parse ``"<inf|-inf|nan>@step=N[,rank=R][,param=I][,every=K]"``."""
    try:
        kind, _, rest = spec.partition("@")
        value = {"inf": float("inf"), "+inf": float("inf"), "-inf": float("-inf"),
                 "nan": float("nan")}[kind.strip().lower()]
        kv = dict(item.split("=", 1) for item in rest.split(",") if item.strip())
        kv = {k.strip(): int(v) for k, v in kv.items()}
        unknown = set(kv) - {"step", "rank", "param", "every"}
        if unknown or "step" not in kv:
            raise ValueError
        return FaultSpec(value, kv["step"], kv.get("rank"), kv.get("param", 0),
                         kv.get("every", 0))
    except (KeyError, ValueError):
        raise ValueError("bad fault-injection spec %r; expected e.g. 'inf@step=5,rank=1,param=0'"
                         % spec) from None


class _State:
    spec: Optional[FaultSpec] = None
    env_checked = False
    step = 0
    fired = 0


_state = _State()


def configure(spec):
    """Enable injection from a spec string or FaultSpec (overrides the env var)."""
    _state.spec = parse(spec) if isinstance(spec, str) else spec
    _state.env_checked = True
    _state.step = 0
    _state.fired = 0


def disable():
    _state.spec = None
    _state.env_checked = True
    _state.step = 0


def fired() -> int:
    return _state.fired


def _active() -> Optional[FaultSpec]:
    if not _state.env_checked:
        _state.env_checked = True
        env = os.environ.get("APEX_AMD_INJECT")
        if env:
            _state.spec = parse(env)
    return _state.spec


def _rank() -> int:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.get_rank()
    return int(os.environ.get("RANK", "0"))


def on_backward_end(optimizers):
    """Called by amp.scale_loss after backward, before unscale."""
    spec = _active()
    if spec is None:
        return
    step = _state.step
    _state.step += 1
    if not spec.fires(step, _rank()):
        return
    grads = []
    for opt in optimizers:
        stash = getattr(opt, "_amp_stash", None)
        if stash is not None and getattr(stash, "master_weights", False) and \
                getattr(stash, "lazy_init_called", False):
            grads += [p.grad for p in stash.all_fp16_params if p.grad is not None]
            grads += [p.grad for p in stash.all_fp32_from_fp32_params if p.grad is not None]
        else:
            grads += [p.grad for g in opt.param_groups for p in g["params"] if p.grad is not None]
    if not grads:
        return
    g = grads[min(spec.param, len(grads) - 1)]
    with torch.no_grad():
        g.view(-1)[0] = spec.value
    _state.fired += 1
