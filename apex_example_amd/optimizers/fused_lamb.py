"""FusedLAMB (apex@f3a960f8 apex/optimizers/fused_lamb.py).

Per step:
  1. global grad norm = ||[||g_fp32||, ||g_16||]|| computed on the device with the
     deterministic multi-tensor l2norm (no host sync), divided by the loss scale
     when the grads are still scaled;
  2. one fused launch per dtype set: stage 1 (clip by global_norm/max_grad_norm,
     Adam(W) moments, per-chunk ||p||^2 and ||u||^2 partials in the same pass;
     u itself is not stored) -> per-tensor norm finalize -> stage 2 (u
     recomputed from p, m, v; trust ratio ||p||/||u||, p -= lr*ratio*u, 16-bit
     model copy written in-pass under amp O2).  No fp32 update workspace: the
     optimizer's persistent memory is exactly m and v.

``max_grad_norm`` is honoured per param group (Apex reads only the constructor
default; a group without its own value gets that default, so Apex behaviour is
unchanged).  The clip factor comes from the global norm over every group.
"""
from __future__ import annotations

import torch

from .. import _native, amp_C
from ._base import FusedOptimizerBase


class FusedLAMB(FusedOptimizerBase):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-6,
                 weight_decay=0.01, amsgrad=False, adam_w_mode=True, grad_averaging=True,
                 set_grad_none=True, max_grad_norm=1.0, use_nvlamb=False,
                 materialize_master_grads=True):
        if amsgrad:
            raise RuntimeError("FusedLAMB does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay, grad_averaging=grad_averaging,
                        max_grad_norm=max_grad_norm)
        super().__init__(params, defaults, set_grad_none=set_grad_none,
                         materialize_master_grads=materialize_master_grads)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.use_nvlamb = use_nvlamb

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()

        all_sets = [self._launch_sets(gid, group) for gid, group in enumerate(self.param_groups)]
        if all(s.get("_plan") is not None for sets in all_sets for s in sets.values()) and any(
                all_sets):
            self._planned_step(all_sets)
            return loss
        # global grad norm over every group (Apex: blend of the fp32 and fp16 norms)
        scaled, unscaled = [], []
        for sets in all_sets:
            for s in sets.values():
                (scaled if s["scaled"] else unscaled).extend(s["grads"])
        if not scaled and not unscaled:
            return loss
        dev = (scaled or unscaled)[0].device
        noop = self._noop(dev)
        # norms only WRITE their flag: give them a scratch flag, never the noop flag
        dummy = self._dummy(str(dev) + ":scratch")
        C = _native.require().mt
        parts = []
        if unscaled:
            parts.append(C.norm(dummy, unscaled, False, False)[0])
        if scaled:
            n = C.norm(dummy, scaled, False, False)[0]
            sv, inv = self._fold_scale()
            if isinstance(sv, torch.Tensor):
                n = n / sv
            else:
                n = n * sv
            parts.append(n)
        global_grad_norm = parts[0] if len(parts) == 1 else torch.stack(parts).norm().reshape(1)

        for gid, group in enumerate(self.param_groups):
            sets = all_sets[gid]
            if not sets:
                continue
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            grad_averaging = 1 if group["grad_averaging"] else 0
            step, step_t = self._step_value(gid, group, dev)
            for key, s in sets.items():
                m, v = self._state_lists(s, ("exp_avg", "exp_avg_sq"))
                scale_v, inv = self._scale_args(s["scaled"])
                amp_C.multi_tensor_lamb(65536, noop, [s["grads"], s["params"], m, v], group["lr"],
                                        beta1, beta2, group["eps"],
                                        step_t if step_t is not None else step, bias_correction,
                                        group["weight_decay"], grad_averaging, self.adam_w_mode,
                                        global_grad_norm,
                                        group.get("max_grad_norm", self.defaults["max_grad_norm"]),
                                        self.use_nvlamb, model_copies=s["copies"], scale=scale_v,
                                        scale_inv=inv)
            self._after_step(gid, dev, step_t, noop)
            self._set_plans(gid, sets, lambda s: [s["params"]] + list(s["_state"][1]) + (
                [s["copies"]] if s["copies"] is not None else []))
        return loss

    def _planned_step(self, all_sets):
        """Steady state: every launch set on its native StepPlan (csrc/torch/amp_ops.cpp) -
        the global grad norm is one norm per set written into one device vector (unscaled
        in the same call) and one norm of that vector; each set's two LAMB stages are one
        C++ call with scalar arguments (no tensor lists cross from Python)."""
        flat = [s for sets in all_sets for s in sets.values()]
        dev = flat[0]["params"][0].device
        noop = self._noop(dev)
        dummy = self._dummy(str(dev) + ":scratch")
        bufs = self.__dict__.setdefault("_norm_bufs", {})
        buf = bufs.get((str(dev), len(flat)))
        if buf is None:
            buf = bufs[(str(dev), len(flat))] = torch.empty(len(flat), dtype=torch.float32,
                                                            device=dev)
        for i, s in enumerate(flat):
            if s["scaled"]:
                sv, _inv = self._fold_scale()
                ok = s["_plan"].grad_norm_into(buf, i, dummy, 1.0 if isinstance(
                    sv, torch.Tensor) else float(sv), sv if isinstance(sv, torch.Tensor) else None)
            else:
                ok = s["_plan"].grad_norm_into(buf, i, dummy, 1.0, None)
            if not ok:
                raise RuntimeError("FusedLAMB: launch set changed inside step()")
        global_grad_norm = buf if len(flat) == 1 else buf.norm().reshape(1)
        for gid, group in enumerate(self.param_groups):
            sets = all_sets[gid]
            if not sets:
                continue
            beta1, beta2 = group["betas"]
            step, step_t = self._step_value(gid, group, dev)
            last = len(sets) - 1
            for i, s in enumerate(sets.values()):
                sv, st, inv = self._plan_scale(s["scaled"])
                lr = group["lr"]
                lv, lt = (1.0, lr) if isinstance(lr, torch.Tensor) else (float(lr), None)
                if not s["_plan"].lamb(noop, lv, lt, beta1, beta2, group["eps"], step, step_t,
                                       bool(group["bias_correction"]), group["weight_decay"],
                                       bool(group["grad_averaging"]), self.adam_w_mode,
                                       global_grad_norm,
                                       group.get("max_grad_norm", self.defaults["max_grad_norm"]),
                                       self.use_nvlamb, sv, st, inv, i == last):
                    raise RuntimeError("FusedLAMB: launch set changed inside step()")
