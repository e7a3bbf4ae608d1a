"""Shared machinery of the fused optimizers.

Every fused optimizer of this package:

* groups the tensors of a param group into launch sets of identical dtype
  signature (grad, param[, 16-bit model copy]) and issues ONE multi-tensor
  launch per set (usually one per group);
* under amp master weights it reads the masters from the amp stash and writes
  the 16-bit model copy inside the same kernel (``_amp_writes_model_copy``), so
  amp's separate master->model copy pass disappears; with
  ``materialize_master_grads=False`` it also reads the 16-bit model grads
  directly and folds the 1/loss_scale multiply into the kernel;
* in amp sync-free mode passes the loss scaler's device overflow flag as the
  kernels' noop flag, and keeps step counters / first-run flags on the device,
  so a skipped step never needs a host round trip.
"""
from __future__ import annotations

import functools
import itertools
import operator
from collections import OrderedDict

import torch

from .. import _native


_GRAD = operator.attrgetter("grad")
# native StepPlan launches from the second step on (tests turn it off to compare with the
# per-step Python launch path)
_STEP_PLAN = True


class FusedOptimizerBase(torch.optim.Optimizer):
    _amp_fused = True
    _amp_writes_model_copy = True
    # amp O1 16-bit weight copies written by the step (fused_dense.cast_params_once); the
    # optimizers whose kernels take a copy list opt in
    _o1_copies = False

    def __init__(self, params, defaults, set_grad_none=True, materialize_master_grads=True):
        super().__init__(params, defaults)
        self.set_grad_none = set_grad_none
        self.materialize_master_grads = materialize_master_grads
        self._dev_steps = {}
        self._dev_flags = {}
        self._dummy_bufs = {}
        self.most_recent_scale = 1.0
        self.scale_set_by_backward = False
        self._set_cache = {}

    @staticmethod
    def profile_hook_step(func):
        """torch's step wrapper opens a record_function (pytree-walking its
        arguments) on every call - ~10 us of host time per step.  Take that path
        only when something can observe it: a running profiler or a registered
        step hook; otherwise call the step directly."""
        hooked = torch.optim.Optimizer.profile_hook_step(func)
        from torch.autograd import profiler as _prof
        from torch.optim import optimizer as _optmod

        @functools.wraps(func)
        def wrapper(*args, **kwargs):
            self = args[0]
            if (_prof._is_profiler_enabled or self._optimizer_step_pre_hooks
                    or self._optimizer_step_post_hooks or _optmod._global_optimizer_pre_hooks
                    or _optmod._global_optimizer_post_hooks):
                return hooked(*args, **kwargs)
            return func(*args, **kwargs)
        return wrapper

    # ------------------------------------------------------------------ helpers
    def _dummy(self, device):
        key = str(device)
        b = self._dummy_bufs.get(key)
        if b is None:
            dev = key.split(":scratch")[0]
            b = self._dummy_bufs[key] = torch.zeros(1, dtype=torch.int32, device=dev)
        return b

    def _amp(self):
        stash = getattr(self, "_amp_stash", None)
        return stash

    def _noop(self, device):
        """The flag the kernels check: the amp scaler's overflow flag (sync-free
        dynamic scaling) or a zero buffer."""
        stash = self._amp()
        if stash is not None and stash.sync_free and stash.last_scaler is not None:
            sc = stash.last_scaler
            if sc.dynamic and sc._overflow_buf.device == torch.device(device):
                return sc._overflow_buf
        return self._dummy(device)

    def _sync_free(self):
        stash = self._amp()
        return stash is not None and stash.sync_free and stash.last_scaler is not None

    def _fold_scale(self):
        """Scale argument for launch sets that read raw (loss-scaled) grads: the scale
        the grads were PRODUCED with (``grads_scale``), not the current one, which
        update_scale() has already grown on a window's last step."""
        stash = self._amp()
        if stash is None or stash.last_scaler is None:
            return 1.0, False
        s = stash.last_scaler.grads_scale()
        if isinstance(s, torch.Tensor):
            return s, True
        return 1.0 / s, False

    def _amp_key(self, gid):
        """(key, grad sources) of group gid: which tensors own the grads the kernels read."""
        stash = self._amp()
        amp_path = bool(stash is not None and getattr(stash, "master_weights", False)
                        and stash.lazy_init_called)
        fold = not self.materialize_master_grads
        if amp_path:
            srcs = (stash.fp16_groups[gid] if fold else stash.fp32_from_fp16_groups[gid],
                    stash.fp32_from_fp32_groups[gid])
        else:
            srcs = (self.param_groups[gid]["params"],)
        # amp O1 folded unscale: the (fp32) grads still carry the loss scale
        o1_scaled = bool(not amp_path and stash is not None
                         and getattr(stash, "grads_scaled", False))
        return (amp_path, fold, o1_scaled), srcs

    def _launch_sets(self, gid, group):
        """OrderedDict key -> dict(grads, params, copies, scaled, owners).

        Cached per group.  Steady state: every set carries a native ``StepPlan``
        (``_set_plans``) that reads the grads from their owners in C++, so the step
        never walks the parameters in Python - ``refresh()`` (one call per set) checks
        that every owner still has a grad of the planned dtype / size and that no
        other parameter gained one.  Without plans (CPU-less native build, first step)
        a C-speed identity check of the current grads against the cached ones decides;
        rebuilding costs ~1 us per tensor of Python, which for ResNet-50's 161 tensors
        was more host time than the 0.1 ms the kernel runs."""
        key, srcs = self._amp_key(gid)
        c = self._set_cache.get(gid)
        grads = None
        if c is not None and c[0] == key:
            if c[3]:
                if all(s["_plan"].refresh() for s in c[2].values()):
                    return c[2]
            else:
                grads = list(itertools.chain.from_iterable(map(_GRAD, s) for s in srcs))
                if len(c[1]) == len(grads) and all(map(operator.is_, c[1], grads)):
                    return c[2]
        if grads is None:
            grads = list(itertools.chain.from_iterable(map(_GRAD, s) for s in srcs))
        stash = self._amp()
        sets = self._build_launch_sets(gid, group, stash, key[0], key[1], key[2])
        absent = [t for src in srcs for t in src if t.grad is None]
        self._set_cache[gid] = [key, grads, sets, False, absent]
        return sets

    def _set_plans(self, gid, sets, fixed):
        """Attach a native StepPlan to every set of group gid (``fixed(s)`` -> the
        non-grad lists of the set's launch); from the next step on the group takes
        the plan path (CPU tensors too: the plan calls the CPU kernels).  No-op
        without the extension."""
        c = self._set_cache.get(gid)
        if c is None or c[2] is not sets or c[3] or not _STEP_PLAN or not _native.available():
            return
        plans = [_native.require().mt.StepPlan(s["owners"], fixed(s)) for s in sets.values()]
        for s, pl in zip(sets.values(), plans):
            s["_plan"] = pl
        if plans:
            plans[0].set_absent(c[4])
            c[3] = True

    def _state_lists(self, s, names, init=torch.zeros_like):
        """Per-set lists of optimizer state tensors (``self.state[p][name]``),
        created with ``init(p)`` on first use and cached on the (cached) set."""
        cached = s.get("_state")
        if cached is not None and cached[0] == names:
            return cached[1]
        out = tuple([] for _ in names)
        for p in s["params"]:
            st = self.state[p]
            for lst, name in zip(out, names):
                t = st.get(name)
                if t is None:
                    t = st[name] = init(p)
                lst.append(t)
        s["_state"] = (names, out)
        return out

    def _build_launch_sets(self, gid, group, stash, amp_path, fold, o1_scaled=False):
        sets = OrderedDict()

        def add(key, g, p, c, scaled, owner):
            s = sets.get(key)
            if s is None:
                s = sets[key] = {"grads": [], "params": [], "copies": [] if c is not None else None,
                                 "scaled": scaled, "owners": []}
            s["owners"].append(owner)
            s["grads"].append(g)
            s["params"].append(p)
            if c is not None:
                s["copies"].append(c)

        if amp_path:
            for model_p, master in zip(stash.fp16_groups[gid], stash.fp32_from_fp16_groups[gid]):
                g = model_p.grad if fold else master.grad
                if g is None:
                    continue
                if g.is_sparse:
                    raise RuntimeError("fused optimizers do not support sparse gradients")
                add((g.dtype, master.dtype, model_p.dtype, fold), g, master, model_p, fold,
                    model_p if fold else master)
            for p in stash.fp32_from_fp32_groups[gid]:
                if p.grad is None:
                    continue
                add((p.grad.dtype, p.dtype, None, False), p.grad, p, None, False, p)
        else:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("fused optimizers do not support sparse gradients")
                cp = None
                if self._o1_copies and p.dtype == torch.float32 and p.is_cuda:
                    # amp O1: the step also writes the 16-bit copy the next forward's
                    # cast_params_once would otherwise re-cast (fused_dense.o1_copy_of)
                    from ..fused_dense import o1_copy_of
                    cp = o1_copy_of(p)
                add((p.grad.dtype, p.dtype, cp.dtype if cp is not None else None, o1_scaled),
                    p.grad, p, cp, o1_scaled, p)
                if cp is not None:
                    sets[(p.grad.dtype, p.dtype, cp.dtype, o1_scaled)]["o1"] = True
        return sets

    def _scale_args(self, scaled):
        if not scaled:
            return 1.0, False
        return self._fold_scale()

    def _plan_scale(self, scaled):
        """(value, tensor or None, invert) of the scale argument, for StepPlan calls."""
        v, inv = self._scale_args(scaled)
        if isinstance(v, torch.Tensor):
            return 1.0, v, inv
        return float(v), None, inv

    def _dev_step(self, gid, device):
        """int32 device counter of completed steps for group gid (sync-free mode)."""
        t = self._dev_steps.get(gid)
        if t is None:
            t = torch.tensor([int(self.param_groups[gid].get("step", 0))], dtype=torch.int32,
                             device=device)
            self._dev_steps[gid] = t
        return t

    def _dev_flag(self, key, device, init_first_run):
        """int32 device 'initialised' flag (0 => first run) for momentum-style state."""
        t = self._dev_flags.get(key)
        if t is None:
            t = torch.tensor([0 if init_first_run else 1], dtype=torch.int32, device=device)
            self._dev_flags[key] = t
        return t

    def _step_value(self, gid, group, device):
        """(host step, device step tensor or None) for this step; increments host step."""
        if self._sync_free() and device.type == "cuda":
            return 0, self._dev_step(gid, device)
        group["step"] = group.get("step", 0) + 1
        return group["step"], None

    def _after_step(self, gid, device, step_t, noop):
        if step_t is not None:
            _native.require().mt.advance_step(step_t, noop)

    # ------------------------------------------------------------------ API
    def zero_grad(self, set_to_none=None):
        """Apex semantics (set_grad_none -> None, else zero in place).  Grads that
        are DDP bucket views are always zeroed in place so they stay views
        (one multi-tensor launch); the amp stash learns that they are zero."""
        if set_to_none is None:
            set_to_none = self.set_grad_none
        grads, views = [], []
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if getattr(p, "_amd_grad_is_bucket_view", False):
                    views.append(p)  # zeroed lazily where the DDP reducer allows it
                    continue
                if set_to_none:
                    p.grad = None
                    continue
                if p.grad.requires_grad:
                    p.grad = p.grad.detach()
                grads.append(p.grad)
        if views:
            from ..ops import _ddp_direct
            grads.extend(_ddp_direct.lazy_zero(views))
        if grads:
            _native.require().mt.zero(grads)
        stash = self._amp()
        if stash is not None:
            stash.model_grads_zeroed = True
            stash.grads_scaled = False  # nothing loss-scaled is pending any more

    def _materialize_steps(self):
        for gid, t in self._dev_steps.items():
            self.param_groups[gid]["step"] = int(t.item())

    def state_dict(self):
        self._materialize_steps()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dev_steps = {}
        self._dev_flags = {}
        self._set_cache = {}

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        self._set_cache = {}
