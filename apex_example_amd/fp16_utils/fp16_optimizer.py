"""Legacy ``FP16_Optimizer`` (apex@f3a960f8 apex/fp16_utils/fp16_optimizer.py).

Wraps an optimizer over 16-bit params: keeps fp32 master copies, scales the
loss, copies/unscales grads into the masters with one multi-tensor launch,
skips the step on overflow, and copies masters back.  Superseded by amp O2 but
kept for API parity.
"""
from __future__ import annotations

import torch

from ..amp._amp_state import is_half_dtype, maybe_print
from .fp16util import clip_grad_norm, master_params_to_model_params  # noqa: F401
from .loss_scaler import DynamicLossScaler, LossScaler


class FP16_Optimizer(object):
    def __init__(self, init_optimizer, static_loss_scale=1.0, dynamic_loss_scale=False,
                 dynamic_loss_args=None, verbose=True):
        self.verbose = verbose
        self.optimizer = init_optimizer
        self.fp16_groups = []
        self.fp32_from_fp16_groups = []
        self.fp32_from_fp32_groups = []
        for i, param_group in enumerate(self.optimizer.param_groups):
            self.maybe_print("FP16_Optimizer processing param group {}:".format(i))
            fp16_params_this_group = []
            fp32_params_this_group = []
            fp32_from_fp16_params_this_group = []
            for j, param in enumerate(param_group["params"]):
                if param.requires_grad:
                    if is_half_dtype(param.dtype):
                        self.maybe_print("FP16_Optimizer received {} with {}".format(
                            param.dtype, tuple(param.size())))
                        fp16_params_this_group.append(param)
                        master_param = param.detach().clone().float()
                        master_param.requires_grad = True
                        param_group["params"][j] = master_param
                        fp32_from_fp16_params_this_group.append(master_param)
                        if param in self.optimizer.state:
                            self.optimizer.state[master_param] = self.optimizer.state.pop(param)
                    elif param.dtype == torch.float32:
                        self.maybe_print("FP16_Optimizer received torch.float32 with {}".format(
                            tuple(param.size())))
                        fp32_params_this_group.append(param)
                        param_group["params"][j] = param
                    else:
                        raise TypeError("Wrapped parameters must be either half/bfloat16 or "
                                        "float32 tensors. Received {}".format(param.dtype))
            self.fp16_groups.append(fp16_params_this_group)
            self.fp32_from_fp16_groups.append(fp32_from_fp16_params_this_group)
            self.fp32_from_fp32_groups.append(fp32_params_this_group)

        self.all_fp16_params = [p for g in self.fp16_groups for p in g]
        self.all_fp32_from_fp16_params = [p for g in self.fp32_from_fp16_groups for p in g]
        self.all_fp32_from_fp32_params = [p for g in self.fp32_from_fp32_groups for p in g]
        self.optimizer.load_state_dict(self.optimizer.state_dict())

        if dynamic_loss_scale:
            self.dynamic_loss_scale = True
            if dynamic_loss_args is not None:
                self.loss_scaler = DynamicLossScaler(**dynamic_loss_args)
            else:
                self.loss_scaler = DynamicLossScaler()
        else:
            self.dynamic_loss_scale = False
            self.loss_scaler = LossScaler(static_loss_scale)
        self.overflow = False
        self.first_closure_call_this_step = True
        self.clip_grad_norm = clip_grad_norm
        dev = self.all_fp16_params[0].device if self.all_fp16_params else torch.device("cpu")
        self._overflow_buf = torch.zeros(1, dtype=torch.int32, device=dev)

    def maybe_print(self, msg):
        if self.verbose:
            print(msg)

    def __getstate__(self):
        raise RuntimeError("FP16_Optimizer should be serialized using state_dict().")

    def __setstate__(self, state):
        raise RuntimeError("FP16_Optimizer should be deserialized using load_state_dict().")

    def zero_grad(self, set_grads_to_None=False):
        for group in self.optimizer.param_groups:
            for p in group["params"]:
                if set_grads_to_None:
                    p.grad = None
                elif p.grad is not None:
                    p.grad = p.grad.detach()
                    p.grad.zero_()
        for fp16_group in self.fp16_groups:
            for param in fp16_group:
                if set_grads_to_None:
                    param.grad = None
                elif param.grad is not None:
                    param.grad = param.grad.detach()
                    param.grad.zero_()

    def _master_params_to_model_params(self):
        from .. import amp_C

        if self.all_fp16_params:
            amp_C.multi_tensor_scale(65536, self._overflow_buf,
                                     [self.all_fp32_from_fp16_params, self.all_fp16_params], 1.0)

    def clip_master_grads(self, max_norm, norm_type=2):
        if not self.overflow:
            fp32_params = []
            for param_group in self.optimizer.param_groups:
                for param in param_group["params"]:
                    fp32_params.append(param)
            return self.clip_grad_norm(fp32_params, max_norm, norm_type)
        else:
            return -1

    def state_dict(self):
        state_dict = {}
        state_dict["loss_scaler"] = self.loss_scaler
        state_dict["dynamic_loss_scale"] = self.dynamic_loss_scale
        state_dict["overflow"] = self.overflow
        state_dict["first_closure_call_this_step"] = self.first_closure_call_this_step
        state_dict["optimizer_state_dict"] = self.optimizer.state_dict()
        state_dict["fp32_from_fp16"] = self.fp32_from_fp16_groups
        return state_dict

    def load_state_dict(self, state_dict):
        self.loss_scaler = state_dict["loss_scaler"]
        self.dynamic_loss_scale = state_dict["dynamic_loss_scale"]
        self.overflow = state_dict["overflow"]
        self.first_closure_call_this_step = state_dict["first_closure_call_this_step"]
        self.optimizer.load_state_dict(state_dict["optimizer_state_dict"])
        for current_group, saved_group in zip(self.fp32_from_fp16_groups,
                                              state_dict["fp32_from_fp16"]):
            for current, saved in zip(current_group, saved_group):
                current.data.copy_(saved.data)

    def step(self, closure=None):
        scale = self.loss_scaler.loss_scale
        if self.overflow:
            maybe_print("Gradient overflow.  Skipping step, reducing loss scale to {}".format(
                self.loss_scaler.loss_scale))
            return
        if closure is not None:
            retval = self._step_with_closure(closure)
        else:
            retval = self.optimizer.step()
        self._master_params_to_model_params()
        return retval

    def _step_with_closure(self, closure):
        def wrapped_closure():
            if self.first_closure_call_this_step:
                self.first_closure_call_this_step = False
            else:
                self._master_params_to_model_params()
            temp_loss = closure()
            while self.overflow:
                scale = self.loss_scaler.loss_scale
                print("OVERFLOW within closure! Skipping step, reducing loss scale to {}".format(
                    self.loss_scaler.loss_scale))
                temp_loss = closure()
            return temp_loss

        retval = self.optimizer.step(wrapped_closure)
        self.first_closure_call_this_step = True
        return retval

    def backward(self, loss, update_master_grads=True, retain_graph=False):
        scaled_loss = loss.float() * self.loss_scaler.loss_scale
        scaled_loss.backward(retain_graph=retain_graph)
        if update_master_grads:
            self.update_master_grads()

    def update_master_grads(self):
        from .. import amp_C

        self._overflow_buf.zero_()
        model_grads, master_grads = [], []
        for mp, p in zip(self.all_fp32_from_fp16_params, self.all_fp16_params):
            if p.grad is not None:
                if mp.grad is None:
                    mp.grad = torch.empty_like(mp)
                model_grads.append(p.grad)
                master_grads.append(mp.grad)
        fp32_grads = [p.grad for p in self.all_fp32_from_fp32_params if p.grad is not None]
        inv = 1.0 / self.loss_scaler.loss_scale
        if model_grads:
            amp_C.multi_tensor_scale(65536, self._overflow_buf, [model_grads, master_grads], inv)
        if fp32_grads:
            amp_C.multi_tensor_scale(65536, self._overflow_buf, [fp32_grads, fp32_grads], inv)
        if self.dynamic_loss_scale:
            self.overflow = bool(self._overflow_buf.item())
            self.loss_scaler.update_scale(self.overflow)
        else:
            self.overflow = False

    def inspect_master_grad_data(self):
        if self.overflow:
            print("Warning:  calling FP16_Optimizer.inspect_master_grad_data while in an overflow "
                  "state.  Gradients are currently invalid (may be inf, nan, or stale).  Returning "
                  "None.")
            return None
        master_grads_data = []
        for param_group in self.optimizer.param_groups:
            master_grads_data.append([p.grad.data if p.grad is not None else None
                                      for p in param_group["params"]])
        return master_grads_data

    def _get_loss_scale(self):
        return self.loss_scaler.loss_scale

    def _set_loss_scale(self, value):
        self.loss_scaler.cur_scale = value

    loss_scale = property(_get_loss_scale, _set_loss_scale)

    def _get_state(self):
        return self.optimizer.state

    def _set_state(self, value):
        self.optimizer.state = value

    state = property(_get_state, _set_state)

    def _get_param_groups(self):
        return self.optimizer.param_groups

    def _set_param_groups(self, value):
        self.optimizer.param_groups = value

    param_groups = property(_get_param_groups, _set_param_groups)
