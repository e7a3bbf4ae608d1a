"""FusedNovoGrad (apex@f3a960f8 apex/optimizers/fused_novograd.py).

Per-tensor second moment stored as a norm (so L2 and inf norms share one
update): L2: v = sqrt(b2*v^2 + (1-b2)*||g||^2), inf: v = b2*v + (1-b2)*||g||_inf.
``init_zero=False`` seeds v with the first step's grad norm.  The update is
g_hat = g / (v/sqrt(bc2) + eps); moment_mode 1 (default, decoupled):
m = b1*m + b3*g_hat, p -= lr*(m/bc1 + wd*p); moment_mode 0
(reg_inside_moment=True): the wd*p term is added to g_hat inside the moment.
Per-tensor grad norms come from the deterministic multi-tensor norm kernel,
the blend + update from one fused launch each - no host sync.
"""
from __future__ import annotations

import torch

from .. import _native
from ._base import FusedOptimizerBase


class FusedNovoGrad(FusedOptimizerBase):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0., amsgrad=False, reg_inside_moment=False, grad_averaging=True,
                 norm_type=2, init_zero=False, set_grad_none=True,
                 materialize_master_grads=True):
        if amsgrad:
            raise RuntimeError("FusedNovoGrad does not support the AMSGrad variant.")
        if norm_type not in (0, 2):
            raise RuntimeError("FusedNovoGrad only support l2/inf norm now.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay, grad_averaging=grad_averaging,
                        norm_type=norm_type, init_zero=init_zero)
        super().__init__(params, defaults, set_grad_none=set_grad_none,
                         materialize_master_grads=materialize_master_grads)
        self.moment_mode = 0 if reg_inside_moment else 1

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        C = _native.require().mt
        for gid, group in enumerate(self.param_groups):
            sets = self._launch_sets(gid, group)
            if not sets:
                continue
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            grad_averaging = 1 if group["grad_averaging"] else 0
            dev = next(iter(sets.values()))["params"][0].device
            step, step_t = self._step_value(gid, group, dev)
            noop = self._noop(dev)
            scratch = self._dummy(str(dev) + ":scratch")
            first = "exp_avg_sq" not in group
            if first:
                group["exp_avg_sq"] = []
            for k, (key, s) in enumerate(sets.items()):
                m, = self._state_lists(s, ("exp_avg",))
                _, gnorms = C.norm(scratch, s["grads"], True, group["norm_type"] == 0)
                scale_v, inv = self._scale_args(s["scaled"])
                if s["scaled"]:
                    gnorms = gnorms / scale_v if isinstance(scale_v, torch.Tensor) else gnorms * scale_v
                if first:
                    group["exp_avg_sq"].append(torch.zeros(len(s["params"]), dtype=torch.float32,
                                                           device=dev))
                v = group["exp_avg_sq"][k]
                assert v.numel() == len(s["params"])
                first_blend = first and not group["init_zero"]
                lists = [s["grads"], s["params"], m]
                lv = group["lr"]
                sv, st = (1.0, scale_v) if isinstance(scale_v, torch.Tensor) else (float(scale_v), None)
                C.novograd(noop, lists, v, gnorms, bool(first_blend), float(lv), None, float(beta1),
                           float(beta2), float(group["eps"]), int(step), step_t,
                           bool(bias_correction), float(group["weight_decay"]),
                           bool(grad_averaging), int(self.moment_mode), int(group["norm_type"]),
                           sv, st, inv)
                if s["copies"] is not None:
                    from .. import amp_C

                    amp_C.multi_tensor_scale(65536, scratch, [s["params"], s["copies"]], 1.0)
            self._after_step(gid, dev, step_t, noop)
        return loss
