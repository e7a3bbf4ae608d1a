"""Optimizer patching for amp (apex@f3a960f8 apex/amp/_process_optimizer.py,
SURVEY.md A-03).

With master weights (O2) the optimizer's half-precision params are replaced by
fp32 masters (lazily, at the first backward, as in Apex, so a checkpoint loaded
into the model after ``amp.initialize`` seeds the masters).  After backward the
16-bit model grads are unscaled into fp32 master grads with ONE multi-tensor
launch (fused overflow check); after ``step`` the masters are copied back into
the model params with one launch.

MI355X fast path (``materialize_master_grads=False`` on this package's fused
optimizers): no fp32 master grads are materialised.  Backward only runs a
read-only overflow check over the 16-bit grads; the fused optimizer kernel
reads the 16-bit grads directly, multiplies by 1/loss_scale (a device scalar),
updates the fp32 master + state and writes the 16-bit model copy in the same
pass (apex FusedSGD depth-4 semantics, extended to Adam / LAMB).
"""
from __future__ import annotations

import itertools
import operator
import types

import torch

from ..fp16_utils import master_params_to_model_params
from ..multi_tensor_apply import multi_tensor_applier
from ._amp_state import is_half_dtype, maybe_print


class AmpOptimizerState(object):
    def __init__(self):
        pass


_GRAD = operator.attrgetter("grad")

def _fused(opt):
    return getattr(opt, "_amp_fused", False)


def _folds_unscale(opt):
    return _fused(opt) and not getattr(opt, "materialize_master_grads", True)


def _zero_or_none(params):
    """Prepare 16-bit model grads for a fresh backward.

    Apex sets them to None (grad copy elision).  Grads that are DDP bucket views
    are zeroed in place instead so they stay views (one launch for all)."""
    vparams = []
    for p in params:
        if p.grad is None:
            continue
        if getattr(p, "_amd_grad_is_bucket_view", False):
            vparams.append(p)
        else:
            p.grad = None
    views = _lazy_zero(vparams)
    if views:
        from .. import amp_C

        amp_C.multi_tensor_zero(65536, None, [views])


def _lazy_zero(params):
    """Bucket-view grads zeroed lazily by their DDP reducer where it allows (the grads are
    detached and the next backward overwrites the views, ops/_ddp_direct.py); returns
    the grads that still need a zero kernel."""
    if not params:
        return []
    from ..ops import _ddp_direct
    return _ddp_direct.lazy_zero(params)


def _stash_grad(stash, param):
    """Take a param's current grad out of the way of the next backward (Apex
    grad-copy elision) and return what must be added back after unscaling.

    A grad that is a DDP bucket view must stay attached (the reducer all-reduces
    the bucket in place), so it cannot simply be set to None: if it is known to
    be zero (zero_grad ran since the last backward) nothing is stashed;
    otherwise its (already unscaled) content is saved and the view zeroed."""
    g = param.grad
    if g is None:
        return None
    if getattr(param, "_amd_grad_is_bucket_view", False):
        if getattr(stash, "model_grads_zeroed", False):
            return None
        saved = g.detach().clone()
        with torch.no_grad():
            g.zero_()
        return saved
    param.grad = None
    return g


def _master_params_to_model_params(self):
    stash = self._amp_stash
    if multi_tensor_applier.available:
        if len(stash.all_fp16_params) > 0:
            from .. import amp_C

            multi_tensor_applier(amp_C.multi_tensor_scale, stash.dummy_overflow_buf,
                                 [stash.all_fp32_from_fp16_params, stash.all_fp16_params], 1.0)
    else:
        for fp16_group, fp32_from_fp16_group in zip(stash.fp16_groups, stash.fp32_from_fp16_groups):
            master_params_to_model_params(fp16_group, fp32_from_fp16_group)


def lazy_init_with_master_weights(self):
    stash = self._amp_stash
    stash.fp16_groups = []
    stash.fp32_from_fp16_groups = []
    stash.fp32_from_fp32_groups = []
    for i, param_group in enumerate(self.param_groups):
        fp16_params_this_group = []
        fp32_params_this_group = []
        fp32_from_fp16_params_this_group = []
        for j, param in enumerate(param_group["params"]):
            if param.requires_grad:
                if is_half_dtype(param.dtype):
                    fp16_params_this_group.append(param)
                    master_param = param.detach().clone().float()
                    master_param.requires_grad = True
                    param_group["params"][j] = master_param
                    fp32_from_fp16_params_this_group.append(master_param)
                    # Reset existing state dict key to the new master param.
                    if param in self.state:
                        self.state[master_param] = self.state.pop(param)
                elif param.dtype == torch.float32:
                    fp32_params_this_group.append(param)
                    param_group["params"][j] = param
                else:
                    raise TypeError("Optimizer's parameters must be half/bfloat16 or float32 "
                                    "tensors.  Received {}".format(param.dtype))
        stash.fp16_groups.append(fp16_params_this_group)
        stash.fp32_from_fp16_groups.append(fp32_from_fp16_params_this_group)
        stash.fp32_from_fp32_groups.append(fp32_params_this_group)

    stash.all_fp16_params = [p for g in stash.fp16_groups for p in g]
    stash.all_fp32_from_fp16_params = [p for g in stash.fp32_from_fp16_groups for p in g]
    stash.all_fp32_from_fp32_params = [p for g in stash.fp32_from_fp32_groups for p in g]
    stash.all_fp16_grad_stash = [None for _ in stash.all_fp16_params]
    stash.all_fp32_from_fp32_grad_stash = [None for _ in stash.all_fp32_from_fp32_params]
    stash.master_grad_bufs = [None for _ in stash.all_fp32_from_fp16_params]

    for param in stash.all_fp32_from_fp16_params:
        param.grad = None
    for param in stash.all_fp32_from_fp32_params:
        param.grad = None

    # Leverage state_dict() and load_state_dict() to recast preexisting per-param state tensors
    self.load_state_dict(self.state_dict())


def post_backward_models_are_masters(scaler, params, stashed_grads, scale_override=None):
    # (never read scaler.loss_scale() here: in sync-free mode that is a host sync)
    grads_have_scale, out_scale = None, 1.0
    if scale_override is not None:
        grads_have_scale, _, out_scale = scale_override

    # This is a lot of python overhead...
    grads_needing_unscale = []
    grads_needing_unscale_with_stash = []
    stashed = []
    for param, stashed_grad in zip(params, stashed_grads):
        if param.grad is None and stashed_grad is not None:
            param.grad = stashed_grad
        elif param.grad is not None and stashed_grad is None:
            grads_needing_unscale.append(param.grad)
        elif param.grad is not None and stashed_grad is not None:
            grads_needing_unscale_with_stash.append(param.grad)
            stashed.append(stashed_grad)
        else:  # param.grad is None and stashed_grad is None
            continue

    # unscale() implements grads*(1/scale), so "scale" should be grads_have_scale/out_scale.
    if len(grads_needing_unscale) > 0:
        scaler.unscale(grads_needing_unscale, grads_needing_unscale, None,
                       models_are_masters=True,
                       scale_override=None if scale_override is None
                       else grads_have_scale / out_scale)
    if len(grads_needing_unscale_with_stash) > 0:
        scaler.unscale_with_stashed(grads_needing_unscale_with_stash, stashed,
                                    grads_needing_unscale_with_stash,
                                    scale_override=scale_override)

    # Clear the stash.
    for i in range(len(stashed_grads)):
        stashed_grads[i] = None


def prepare_backward_with_master_weights(self):
    stash = self._amp_stash
    self._amp_lazy_init()
    _zero_or_none(stash.all_fp16_params)
    for i, param in enumerate(stash.all_fp32_from_fp32_params):
        stash.all_fp32_from_fp32_grad_stash[i] = _stash_grad(stash, param)


def post_backward_with_master_weights(self, scaler):
    stash = self._amp_stash
    self._amp_lazy_init()

    stash.model_grads_zeroed = False
    if _folds_unscale(self):
        # fused optimizer reads the 16-bit grads itself: overflow check only
        grads = [p.grad for p in stash.all_fp16_params if p.grad is not None]
        if grads:
            scaler.check_overflow(grads)
        post_backward_models_are_masters(scaler, stash.all_fp32_from_fp32_params,
                                         stash.all_fp32_from_fp32_grad_stash)
        return

    fp16_grads_needing_unscale = []
    new_fp32_grads = []
    fp16_grads_needing_unscale_with_stash = []
    preexisting_fp32_grads = []
    for i, (fp16_param, fp32_param) in enumerate(zip(stash.all_fp16_params,
                                                     stash.all_fp32_from_fp16_params)):
        if fp16_param.grad is None and fp32_param.grad is not None:
            continue
        elif fp16_param.grad is not None and fp32_param.grad is None:
            buf = stash.master_grad_bufs[i]
            if buf is None:
                buf = stash.master_grad_bufs[i] = torch.empty_like(fp32_param)
            fp32_param.grad = buf
            fp16_grads_needing_unscale.append(fp16_param.grad)
            new_fp32_grads.append(fp32_param.grad)
        elif fp16_param.grad is not None and fp32_param.grad is not None:
            fp16_grads_needing_unscale_with_stash.append(fp16_param.grad)
            preexisting_fp32_grads.append(fp32_param.grad)
        else:  # fp16_param.grad is None and fp32_param.grad is None:
            continue

    if len(fp16_grads_needing_unscale) > 0:
        scaler.unscale(fp16_grads_needing_unscale, new_fp32_grads, scaler.loss_scale,
                       models_are_masters=False)
    if len(fp16_grads_needing_unscale_with_stash) > 0:
        scaler.unscale_with_stashed(fp16_grads_needing_unscale_with_stash,
                                    preexisting_fp32_grads, preexisting_fp32_grads)

    # fp32 params can be treated as they would be in the "no_master_weights" case.
    post_backward_models_are_masters(scaler, stash.all_fp32_from_fp32_params,
                                     stash.all_fp32_from_fp32_grad_stash)


def lazy_init_no_master_weights(self):
    stash = self._amp_stash
    stash.all_fp16_params = []
    stash.all_fp32_params = []
    for i, param_group in enumerate(self.param_groups):
        for i, param in enumerate(param_group["params"]):
            if is_half_dtype(param.dtype):
                stash.all_fp16_params.append(param)
            elif param.dtype == torch.float32:
                stash.all_fp32_params.append(param)
            else:
                raise TypeError("Optimizer's parameters must be half/bfloat16 or float32 "
                                "tensors.  Received {}".format(param.dtype))
    stash.all_fp16_grad_stash = [None for _ in stash.all_fp16_params]
    stash.all_fp32_grad_stash = [None for _ in stash.all_fp32_params]


def _unscale_pending(opt):
    """Grads left loss-scaled by a folded-unscale backward (see
    post_backward_no_master_weights) meet another backward before a step:
    unscale them in place by the scale they carry, so stashing / accumulation
    sees unscaled values as in Apex."""
    stash = opt._amp_stash
    stash.grads_scaled = False
    grads = [p.grad for p in stash.all_fp16_params + stash.all_fp32_params if p.grad is not None]
    if not grads or stash.last_scaler is None:
        return
    from .. import amp_C

    s = stash.last_scaler.grads_scale()
    dummy = torch.zeros(1, dtype=torch.int32, device=grads[0].device)
    if isinstance(s, torch.Tensor):
        amp_C.multi_tensor_scale(65536, dummy, [grads, grads], s, scale_inv=True)
    else:
        amp_C.multi_tensor_scale(65536, dummy, [grads, grads], 1.0 / s)


def prepare_backward_no_master_weights(self):
    stash = self._amp_stash
    self._amp_lazy_init()
    if getattr(stash, "grads_scaled", False):
        _unscale_pending(self)
    for i, param in enumerate(stash.all_fp16_params):
        stash.all_fp16_grad_stash[i] = _stash_grad(stash, param)
    for i, param in enumerate(stash.all_fp32_params):
        stash.all_fp32_grad_stash[i] = _stash_grad(stash, param)


def post_backward_no_master_weights(self, scaler):
    stash = self._amp_stash
    self._amp_lazy_init()
    stash.model_grads_zeroed = False
    if (_folds_unscale(self) and multi_tensor_applier.available
            and not any(g is not None for g in stash.all_fp16_grad_stash)
            and not any(g is not None for g in stash.all_fp32_grad_stash)):
        # amp O1 with a fused optimizer and materialize_master_grads=False: the
        # optimizer kernel multiplies by 1/scale itself (as under O2), so the
        # separate in-place unscale pass over every fp32 grad becomes a read-only
        # overflow check.  The grads stay scaled until the step (or the next
        # backward, which unscales them first).
        grads = [p.grad for p in stash.all_fp16_params + stash.all_fp32_params
                 if p.grad is not None]
        if grads:
            scaler.check_overflow(grads)
        stash.grads_scaled = True
        return
    stash.grads_scaled = False
    split_types = ((stash.all_fp16_params, stash.all_fp16_grad_stash),
                   (stash.all_fp32_params, stash.all_fp32_grad_stash))
    for params, stashed_grads in split_types:
        post_backward_models_are_masters(scaler, params, stashed_grads)


def _amp_lazy_init(self):
    stash = self._amp_stash
    if not stash.lazy_init_called:
        self._lazy_init_maybe_master_weights()
        stash.lazy_init_called = True


def _process_optimizer(optimizer, properties):
    if hasattr(optimizer, "_amp_stash"):
        raise RuntimeError("A given optimizer should only be passed through amp.initialize once.")
    else:
        optimizer._amp_stash = AmpOptimizerState()

    optimizer._amp_stash.lazy_init_called = False
    optimizer._amp_stash.already_patched = False
    optimizer._amp_stash.params_have_scaled_gradients = False
    optimizer._amp_stash.sync_free = False
    optimizer._amp_stash.last_scaler = None
    optimizer._amp_stash.master_weights = bool(properties.master_weights)

    for name in ("_lazy_init_maybe_master_weights", "_master_params_to_model_params",
                 "_prepare_amp_backward", "_post_amp_backward", "_amp_lazy_init"):
        if hasattr(optimizer, name):
            raise RuntimeError("Incoming optimizer already has {} defined.".format(name))

    if multi_tensor_applier.available:
        from .. import amp_C

        optimizer._amp_stash.multi_tensor_scale = amp_C.multi_tensor_scale
        optimizer._amp_stash.multi_tensor_l2norm = amp_C.multi_tensor_l2norm
        dev = None
        for g in optimizer.param_groups:
            for p in g["params"]:
                dev = p.device
                break
            if dev is not None:
                break
        optimizer._amp_stash.dummy_overflow_buf = torch.zeros(
            1, dtype=torch.int32, device=dev if dev is not None else "cpu")

    if properties.master_weights:
        optimizer._lazy_init_maybe_master_weights = types.MethodType(
            lazy_init_with_master_weights, optimizer)
        optimizer._master_params_to_model_params = types.MethodType(
            _master_params_to_model_params, optimizer)

        old_step = optimizer.step

        def new_step(self, closure=None):
            if closure is not None:
                raise RuntimeError("Currently, Amp does not support closure use with optimizers.")
            self._amp_lazy_init()
            retval = old_step()
            if not getattr(self, "_amp_writes_model_copy", False):
                self._master_params_to_model_params()
            # Clear the master grads that wouldn't be zeroed by model.zero_grad()
            # (C-speed scan first: with folded unscale the masters never get grads)
            masters = self._amp_stash.all_fp32_from_fp16_params
            if not all(map(operator.is_, map(_GRAD, masters), itertools.repeat(None))):
                for param in masters:
                    param.grad = None
            return retval

        optimizer.step = types.MethodType(new_step, optimizer)

        def new_zero_grad(self, set_to_none=None):
            stash = self._amp_stash
            self._amp_lazy_init()
            # Zero the model grads.
            views, vparams = [], []
            for param in stash.all_fp16_params + stash.all_fp32_from_fp32_params:
                if param.grad is not None:
                    if param.grad.requires_grad:  # (bucket views never require grad)
                        param.grad = param.grad.detach()
                    if getattr(param, "_amd_grad_is_bucket_view", False):
                        vparams.append(param)
                    else:
                        views.append(param.grad)
            views.extend(_lazy_zero(vparams))
            if views:
                from .. import amp_C

                if multi_tensor_applier.available:
                    amp_C.multi_tensor_zero(65536, None, [views])
                else:
                    for v in views:
                        v.zero_()
            stash.model_grads_zeroed = True
            # Clear the master grads that are independent of model grads
            for param in self._amp_stash.all_fp32_from_fp16_params:
                param.grad = None

        optimizer.zero_grad = types.MethodType(new_zero_grad, optimizer)
        optimizer._prepare_amp_backward = types.MethodType(prepare_backward_with_master_weights,
                                                           optimizer)
        optimizer._post_amp_backward = types.MethodType(post_backward_with_master_weights,
                                                        optimizer)
    else:
        optimizer._lazy_init_maybe_master_weights = types.MethodType(
            lazy_init_no_master_weights, optimizer)
        optimizer._prepare_amp_backward = types.MethodType(prepare_backward_no_master_weights,
                                                           optimizer)
        optimizer._post_amp_backward = types.MethodType(post_backward_no_master_weights,
                                                        optimizer)

    optimizer._amp_lazy_init = types.MethodType(_amp_lazy_init, optimizer)

    old_add_param_group = optimizer.add_param_group

    def new_add_param_group(self, new_group):
        stash = self._amp_stash
        if not stash.lazy_init_called:
            self._lazy_init_maybe_master_weights()
            stash.lazy_init_called = True

        assert isinstance(new_group, dict), "param group must be a dict"
        new_params = new_group["params"]
        if isinstance(new_params, torch.Tensor):
            new_group["params"] = [new_params]
        elif isinstance(new_params, set):
            raise TypeError("optimizer parameters need to be organized in ordered collections, "
                            "but the ordering of tensors in sets will change between runs. "
                            "Please use a list instead.")
        else:
            new_group["params"] = list(new_params)

        if properties.master_weights:
            # Mutate new_group in-place to use FP32 master params
            fp16_params_this_group = []
            fp32_params_this_group = []
            fp32_from_fp16_params_this_group = []
            for i, param in enumerate(new_group["params"]):
                if param.requires_grad:
                    if is_half_dtype(param.dtype):
                        fp16_params_this_group.append(param)
                        master_param = param.detach().clone().float()
                        master_param.requires_grad = True
                        new_group["params"][i] = master_param
                        fp32_from_fp16_params_this_group.append(master_param)
                    elif param.dtype == torch.float32:
                        fp32_params_this_group.append(param)
                        new_group["params"][i] = param
                    else:
                        raise TypeError("Optimizer's parameters must be half/bfloat16 or "
                                        "float32 tensors.  Received {}".format(param.dtype))
            stash.fp16_groups.append(fp16_params_this_group)
            stash.fp32_from_fp16_groups.append(fp32_from_fp16_params_this_group)
            stash.fp32_from_fp32_groups.append(fp32_params_this_group)
            stash.all_fp16_params += fp16_params_this_group
            stash.all_fp32_from_fp16_params += fp32_from_fp16_params_this_group
            stash.all_fp32_from_fp32_params += fp32_params_this_group
            stash.all_fp32_from_fp32_grad_stash += [None for _ in fp32_params_this_group]
            stash.master_grad_bufs += [None for _ in fp32_from_fp16_params_this_group]
        else:
            for param in new_group["params"]:
                if is_half_dtype(param.dtype):
                    stash.all_fp16_params.append(param)
                    stash.all_fp16_grad_stash.append(None)
                elif param.dtype == torch.float32:
                    stash.all_fp32_params.append(param)
                    stash.all_fp32_grad_stash.append(None)
                else:
                    raise TypeError("Optimizer's parameters must be half/bfloat16 or float32 "
                                    "tensors.  Received {}".format(param.dtype))

        old_add_param_group(new_group)

    optimizer.add_param_group = types.MethodType(new_add_param_group, optimizer)
    return optimizer


__all__ = ["_process_optimizer", "AmpOptimizerState", "maybe_print"]
