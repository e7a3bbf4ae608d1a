"""LARC: layer-wise adaptive rate clipping / scaling (apex@f3a960f8
apex/parallel/LARC.py).

Per parameter: adaptive_lr = trust_coefficient * ||p|| / (||g|| + wd*||p|| + eps);
clip mode uses min(adaptive_lr / lr, 1).  The wrapped optimizer's weight decay
is folded into the gradient and zeroed for the inner step, then restored.

MI355X design: Apex computes two norms per parameter with host-side
comparisons (2 syncs per parameter).  Here all parameter norms and all grad
norms come from two multi-tensor per-tensor-norm launches, the adaptive factors
are computed on the device as vectors, and the gradients are rescaled with
multi-tensor foreach ops - no host synchronisation at all.
"""
from __future__ import annotations

import torch

from .. import _native


class LARC(object):
    def __init__(self, optimizer, trust_coefficient=0.02, clip=True, eps=1e-8):
        self.optim = optimizer
        self.trust_coefficient = trust_coefficient
        self.eps = eps
        self.clip = clip

    def __getstate__(self):
        return self.optim.__getstate__()

    def __setstate__(self, state):
        self.optim.__setstate__(state)

    @property
    def state(self):
        return self.optim.state

    def __repr__(self):
        return self.optim.__repr__()

    @property
    def param_groups(self):
        return self.optim.param_groups

    @param_groups.setter
    def param_groups(self, value):
        self.optim.param_groups = value

    def state_dict(self):
        return self.optim.state_dict()

    def load_state_dict(self, state_dict):
        self.optim.load_state_dict(state_dict)

    def zero_grad(self, *a, **k):
        self.optim.zero_grad(*a, **k)

    def add_param_group(self, param_group):
        self.optim.add_param_group(param_group)

    @torch.no_grad()
    def _rescale_group(self, group, weight_decay):
        params = [p for p in group["params"] if p.grad is not None]
        if not params:
            return
        grads = [p.grad for p in params]
        if _native.available():
            mt = _native.require().mt
            flag = torch.zeros(1, dtype=torch.int32, device=params[0].device)
            _, pn = mt.norm(flag, params, True, False)
            _, gn = mt.norm(flag, grads, True, False)
        else:
            pn = torch.stack([p.float().norm() for p in params])
            gn = torch.stack([g.float().norm() for g in grads])
        ok = (pn != 0) & (gn != 0)
        adaptive = self.trust_coefficient * pn / (gn + pn * weight_decay + self.eps)
        if self.clip:
            adaptive = torch.clamp(adaptive / group["lr"], max=1.0)
        factor = torch.where(ok, adaptive, torch.ones_like(adaptive))
        wd = torch.where(ok, torch.full_like(adaptive, weight_decay), torch.zeros_like(adaptive))
        if weight_decay != 0:
            wds = list(wd.unbind())
            terms = torch._foreach_mul([p.to(g.dtype) for p, g in zip(params, grads)], wds)
            torch._foreach_add_(grads, terms)
        factors = list(factor.unbind())
        torch._foreach_mul_(grads, [f.to(g.dtype) for f, g in zip(factors, grads)])

    def step(self, closure=None):
        weight_decays = []
        for group in self.optim.param_groups:
            # absorb weight decay control from optimizer
            weight_decay = group["weight_decay"] if "weight_decay" in group else 0
            weight_decays.append(weight_decay)
            group["weight_decay"] = 0
            self._rescale_group(group, weight_decay)
        try:
            ret = self.optim.step(closure) if closure is not None else self.optim.step()
        finally:
            # return weight decay control to optimizer
            for i, group in enumerate(self.optim.param_groups):
                group["weight_decay"] = weight_decays[i]
        return ret
