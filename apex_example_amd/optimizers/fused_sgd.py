"""FusedSGD (apex@f3a960f8 apex/optimizers/fused_sgd.py).

One multi-tensor launch per (param group, dtype signature).  Under amp O2 the
launch set is (grad, fp32 master, fp32 momentum, 16-bit model copy) - the
depth-4 kernel updates the master and momentum and writes the bf16/fp16 model
weight in one pass (20 B/param with ``materialize_master_grads=False``, where
the grad read is the raw 16-bit model grad and 1/loss_scale is applied
in-kernel).
"""
from __future__ import annotations

import torch
from torch.optim.optimizer import required

from .. import amp_C
from ._base import FusedOptimizerBase


class FusedSGD(FusedOptimizerBase):
    r"""Implements stochastic gradient descent (optionally with momentum).

    Same constructor as ``apex.optimizers.FusedSGD``::

        FusedSGD(params, lr, momentum=0, dampening=0, weight_decay=0, nesterov=False,
                 wd_after_momentum=False, materialize_master_grads=True, set_grad_none=False)

    Nesterov momentum follows Sutskever et al. as in torch.optim.SGD:
    v = mu*v + (1-dampening)*g ; p = p - lr*(g + mu*v) (nesterov) or p - lr*v.
    """

    def __init__(self, params, lr=required, momentum=0, dampening=0, weight_decay=0,
                 nesterov=False, wd_after_momentum=False, materialize_master_grads=True,
                 set_grad_none=False):
        if lr is not required and lr < 0.0:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if momentum < 0.0:
            raise ValueError("Invalid momentum value: {}".format(momentum))
        if weight_decay < 0.0:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening,
                        weight_decay=weight_decay, nesterov=nesterov)
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, defaults, set_grad_none=set_grad_none,
                         materialize_master_grads=materialize_master_grads)
        self.wd_after_momentum = wd_after_momentum

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("nesterov", False)

    def get_momentums(self, params):
        momentums = []
        first_run = True
        for p in params:
            param_state = self.state[p]
            # torch.optim.SGD initializes momentum in the main loop, we have
            # to do it here, and track whether or not we've done so, so that
            # momentum application can be skipped in the main kernel.
            if "momentum_buffer" not in param_state:
                first_run = True
                buf = param_state["momentum_buffer"] = torch.zeros_like(p)
                momentums.append(buf)
            else:
                first_run = False
                momentums.append(param_state["momentum_buffer"])
        return momentums, first_run

    def _step_pair(self, sets, wd, momentum, lr, nesterov):
        """amp O2's two launch sets of a group (16-bit-copy set + fp32 set) in ONE
        native launch (StepPlan.sgd_pair), once both carry plans and their momentum
        buffers exist.  False: launch them one by one."""
        if len(sets) != 2:
            return False
        a, b = sets.values()
        if a["copies"] is None:
            a, b = b, a
        pa, pb = a.get("_plan"), b.get("_plan")
        if (pa is None or pb is None or a["copies"] is None or b["copies"] is not None
                or "_moms" not in a or "_moms" not in b):
            return False
        dev = a["params"][0].device
        sa, ta, ia = self._plan_scale(a["scaled"])
        sb, tb, ib = self._plan_scale(b["scaled"])
        return pa.sgd_pair(pb, self._noop(dev), wd, momentum, 0.0, lr, nesterov,
                           self.wd_after_momentum, sa, ta, ia, sb, tb, ib)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()

        for gid, group in enumerate(self.param_groups):
            weight_decay = group["weight_decay"]
            momentum = group["momentum"]
            dampening = group["dampening"]
            nesterov = group["nesterov"]
            lr = group["lr"]
            sets = self._launch_sets(gid, group)
            if dampening == 0 and self._step_pair(sets, weight_decay, momentum, lr, nesterov):
                continue
            planned = True
            for key, s in sets.items():
                params = s["params"]
                dev = params[0].device
                cached = s.get("_moms")
                if cached is None:
                    moms, first_run = self.get_momentums(params)
                    s["_moms"] = moms
                else:
                    moms, first_run = cached, False
                noop = self._noop(dev)
                flag = None
                if dampening == 0:
                    # the momentum buffers start at zero, so mom*0 + (1-0)*g == g bitwise:
                    # Apex's first-run initialisation needs no flag (and no per-step
                    # mark_step_done launch) when there is no dampening
                    first_run = False
                elif self._sync_free() and dev.type == "cuda" and momentum != 0:
                    flag = self._dev_flag((gid, key), dev, first_run)
                plan = s.get("_plan")
                if plan is not None:
                    sv, st, inv = self._plan_scale(s["scaled"])
                    if not plan.sgd(noop, weight_decay, momentum, dampening, lr, nesterov,
                                    first_run, flag, self.wd_after_momentum, sv, st, inv):
                        raise RuntimeError("FusedSGD: launch set changed inside step()")
                else:
                    planned = False
                    lists = [s["grads"], params, moms]
                    if s["copies"] is not None:
                        lists.append(s["copies"])
                    scale, inv = self._scale_args(s["scaled"])
                    amp_C.multi_tensor_sgd(65536, noop, lists, weight_decay, momentum, dampening,
                                           lr, nesterov, first_run, self.wd_after_momentum, scale,
                                           scale_inv=inv, first_run_flag=flag)
                if flag is not None:
                    from .. import _native

                    _native.require().mt.mark_step_done(flag, noop)
            if not planned:
                self._set_plans(gid, sets, lambda s: [s["params"], s["_moms"]] + (
                    [s["copies"]] if s["copies"] is not None else []))

        self.most_recent_scale = 1.0
        self.scale_set_by_backward = False
        return loss
