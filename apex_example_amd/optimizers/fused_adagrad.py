"""FusedAdagrad (apex fused_adagrad).

h += g^2 ; p -= lr * g / (sqrt(h) + eps).  ``adagrad_w_mode=False`` adds
weight_decay*p to the gradient (L2), True applies decoupled decay.
"""
from __future__ import annotations

import torch

from .. import amp_C
from ._base import FusedOptimizerBase


class FusedAdagrad(FusedOptimizerBase):
    def __init__(self, params, lr=1e-2, eps=1e-10, weight_decay=0., set_grad_none=True,
                 adagrad_w_mode=False, materialize_master_grads=True):
        defaults = dict(lr=lr, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults, set_grad_none=set_grad_none,
                         materialize_master_grads=materialize_master_grads)
        self.adagrad_w_mode = 1 if adagrad_w_mode else 0

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gid, group in enumerate(self.param_groups):
            for key, s in self._launch_sets(gid, group).items():
                dev = s["params"][0].device
                h, = self._state_lists(s, ("sum",))
                scale_v, inv = self._scale_args(s["scaled"])
                noop = self._noop(dev)
                amp_C.multi_tensor_adagrad(65536, noop, [s["grads"], s["params"], h], group["lr"],
                                           group["eps"], self.adagrad_w_mode,
                                           group["weight_decay"], scale=scale_v, scale_inv=inv)
                if s["copies"] is not None:
                    amp_C.multi_tensor_scale(65536, self._dummy(str(dev) + ":scratch"),
                                             [s["params"], s["copies"]], 1.0)
        return loss
