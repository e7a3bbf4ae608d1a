"""FusedAdam (apex@f3a960f8 apex/optimizers/fused_adam.py).

``adam_w_mode=True`` (default) is decoupled weight decay (AdamW); False adds
``weight_decay * p`` to the gradient (L2).  ``group['step']`` is kept per param
group (Apex checkpoint format).  Under amp O2 the depth-5 kernel reads the grad,
updates the fp32 master / exp_avg / exp_avg_sq and writes the 16-bit model copy
in one pass; in amp sync-free mode the step counter lives on the device and is
only advanced for non-skipped steps.
"""
from __future__ import annotations

import torch

from .. import amp_C
from ..fused_dense import o1_mark_fresh
from ._base import FusedOptimizerBase


class FusedAdam(FusedOptimizerBase):
    _o1_copies = True
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 adam_w_mode=True, weight_decay=0., amsgrad=False, set_grad_none=True,
                 materialize_master_grads=True):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay)
        super().__init__(params, defaults, set_grad_none=set_grad_none,
                         materialize_master_grads=materialize_master_grads)
        self.adam_w_mode = 1 if adam_w_mode else 0

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=None, grad_norms=None):
        if any(p is not None for p in [grads, output_params, scale, grad_norms]):
            raise RuntimeError("FusedAdam has been updated.  Simply initialize it identically to "
                               "torch.optim.Adam, and call step() with no arguments.")
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()

        for gid, group in enumerate(self.param_groups):
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            sets = self._launch_sets(gid, group)
            if not sets:
                continue
            dev = next(iter(sets.values()))["params"][0].device
            step, step_t = self._step_value(gid, group, dev)
            noop = self._noop(dev)
            planned, last = True, len(sets) - 1
            for i, (key, s) in enumerate(sets.items()):
                if s.get("o1"):
                    # the depth-5 launch below refreshes the amp O1 16-bit weight copies
                    o1_mark_fresh(s["params"], s["copies"])
                # exponential moving averages of the gradient and its square
                m, v = self._state_lists(s, ("exp_avg", "exp_avg_sq"))
                plan = s.get("_plan")
                if plan is not None:
                    sv, st, inv = self._plan_scale(s["scaled"])
                    lr = group["lr"]
                    lv, lt = (1.0, lr) if isinstance(lr, torch.Tensor) else (float(lr), None)
                    # the last set also advances the device step counter (same launch order
                    # as _after_step)
                    if not plan.adam(noop, lv, lt, beta1, beta2, group["eps"], step, step_t,
                                     self.adam_w_mode, bool(bias_correction),
                                     group["weight_decay"], sv, st, inv, i == last):
                        raise RuntimeError("FusedAdam: launch set changed inside step()")
                    continue
                planned = False
                lists = [s["grads"], s["params"], m, v]
                if s["copies"] is not None:
                    lists.append(s["copies"])
                scale_v, inv = self._scale_args(s["scaled"])
                amp_C.multi_tensor_adam(65536, noop, lists, group["lr"], beta1, beta2,
                                        group["eps"], step_t if step_t is not None else step,
                                        self.adam_w_mode, bias_correction,
                                        group["weight_decay"], scale=scale_v, scale_inv=inv)
            if not planned:
                self._after_step(gid, dev, step_t, noop)
                self._set_plans(gid, sets, lambda s: [s["params"]] + list(s["_state"][1]) + (
                    [s["copies"]] if s["copies"] is not None else []))
        return loss
