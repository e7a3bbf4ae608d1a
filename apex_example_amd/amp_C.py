"""Drop-in facade for Apex's ``amp_C`` extension module.

Every function keeps the positional signature of apex@f3a960f8
csrc/amp_C_frontend.cpp and dispatches to the native gfx950 / C++ CPU kernels in
``apex_example_amd._C.mt``.  Extensions over Apex (keyword-only):

* any ``scale`` / ``lr`` argument may be a 1-element float32 *device tensor*
  (no host sync - this is how the dynamic loss scale reaches the kernels);
* ``step`` may be an int32 device tensor holding the number of completed steps;
* ``scale_inv=True`` means "multiply by 1/scale" (loss-scale unscaling).
"""
from __future__ import annotations

import torch

from . import _native


def _C():
    return _native.require().mt


def _split(v):
    """(float_value, tensor_or_None) for a scalar that may live on the device."""
    if isinstance(v, torch.Tensor):
        return 1.0, v
    return float(v), None


def multi_tensor_scale(chunk_size, noop_flag, tensor_lists, scale, *, scale_inv=False):
    s, st = _split(scale)
    _C().scale_any(noop_flag, tensor_lists, s, st, scale_inv)


def multi_tensor_check_finite(chunk_size, noop_flag, tensor_lists):
    """Read-only overflow check (sets noop_flag on inf/nan)."""
    lst = tensor_lists[0] if tensor_lists and isinstance(tensor_lists[0], (list, tuple)) else tensor_lists
    _C().check_finite(noop_flag, list(lst))


def multi_tensor_axpby(chunk_size, noop_flag, tensor_lists, a, b, arg_to_check, *, a_inv=False,
                       b_inv=False):
    av, at = _split(a)
    bv, bt = _split(b)
    _C().axpby(noop_flag, tensor_lists, av, at, a_inv, bv, bt, b_inv, int(arg_to_check))


def multi_tensor_zero(chunk_size, noop_flag, tensor_lists):
    lst = tensor_lists[0] if tensor_lists and isinstance(tensor_lists[0], (list, tuple)) else tensor_lists
    _C().zero(list(lst))


def multi_tensor_l2norm(chunk_size, noop_flag, tensor_lists, per_tensor=False):
    lst = tensor_lists[0]
    return _C().norm(noop_flag, list(lst), bool(per_tensor), False)


def multi_tensor_maxnorm(chunk_size, noop_flag, tensor_lists, per_tensor=False):
    return _C().norm(noop_flag, list(tensor_lists[0]), bool(per_tensor), True)


def multi_tensor_norm_out_cuda(chunk_size, noop_flag, tensor_lists, out, alpha, beta, norm_type):
    """Per-tensor norms blended into ``out``:
    L2 (norm_type=2): out = sqrt(alpha*out^2 + beta*norm^2); inf (0): out = alpha*out + beta*norm."""
    _, per = _C().norm(noop_flag, list(tensor_lists[0]), True, norm_type == 0)
    with torch.no_grad():
        if norm_type == 0:
            out.mul_(alpha).add_(per, alpha=beta)
        else:
            out.copy_((out.pow(2).mul_(alpha) + per.pow(2).mul_(beta)).sqrt_())


def multi_tensor_sgd(chunk_size, noop_flag, tensor_lists, wd, momentum, dampening, lr, nesterov,
                     first_run, wd_after_momentum, scale, *, scale_inv=False,
                     first_run_flag=None):
    lv, lt = _split(lr)
    sv, st = _split(scale)
    _C().sgd(noop_flag, tensor_lists, float(wd), float(momentum), float(dampening), lv, lt,
             bool(nesterov), bool(first_run), first_run_flag, bool(wd_after_momentum), sv, st,
             scale_inv)


def multi_tensor_adam(chunk_size, noop_flag, tensor_lists, lr, beta1, beta2, epsilon, step, mode,
                      bias_correction, weight_decay, *, scale=1.0, scale_inv=False):
    lv, lt = _split(lr)
    sv, st = _split(scale)
    if isinstance(step, torch.Tensor):
        step_v, step_t = 0, step
    else:
        step_v, step_t = int(step), None
    _C().adam(noop_flag, tensor_lists, lv, lt, float(beta1), float(beta2), float(epsilon), step_v,
              step_t, int(mode), bool(bias_correction), float(weight_decay), sv, st, scale_inv)


def multi_tensor_lamb(chunk_size, noop_flag, tensor_lists, lr, beta1, beta2, epsilon, step,
                      bias_correction, weight_decay, grad_averaging, mode, global_grad_norm,
                      max_grad_norm, use_nvlamb=False, *, update_buffers=None, model_copies=None,
                      scale=1.0, scale_inv=False):
    """tensor_lists = [grads, params, exp_avg, exp_avg_sq] (Apex).  The update
    direction is recomputed from (p, m, v) in the second stage on the device, so
    no fp32 workspace exists; ``update_buffers`` is accepted for API
    compatibility and ignored."""
    del update_buffers
    g, p, m, v = tensor_lists[:4]
    lists = [list(g), list(p), list(m), list(v)]
    if model_copies is not None:
        lists.append(list(model_copies))
    lv, lt = _split(lr)
    sv, st = _split(scale)
    if isinstance(step, torch.Tensor):
        step_v, step_t = 0, step
    else:
        step_v, step_t = int(step), None
    gn = global_grad_norm if isinstance(global_grad_norm, torch.Tensor) else None
    if gn is None:
        dev = p[0].device
        gn = torch.tensor([float(global_grad_norm)], dtype=torch.float32, device=dev)
    _C().lamb(noop_flag, lists, lv, lt, float(beta1), float(beta2), float(epsilon), step_v, step_t,
              bool(bias_correction), float(weight_decay), bool(grad_averaging), int(mode), gn,
              float(max_grad_norm), bool(use_nvlamb), sv, st, scale_inv)


def _dev_scalar(v, device):
    """A python number or 1-element tensor as a 0-dim fp32 device tensor (no sync)."""
    if isinstance(v, torch.Tensor):
        return v.reshape(()).to(device=device, dtype=torch.float32)
    return torch.tensor(float(v), dtype=torch.float32, device=device)


def _per_tensor(vals, n, dev):
    """Per-tensor scalars (a tensor or a list of numbers / 1-element tensors) as a
    contiguous fp32 device array [n] (no host sync for device inputs)."""
    if isinstance(vals, torch.Tensor):
        t = vals.reshape(-1)
    elif all(isinstance(v, torch.Tensor) for v in vals):
        t = torch.stack([v.reshape(()) for v in vals])
    else:
        t = torch.tensor([float(v) for v in vals], dtype=torch.float32)
    t = t.to(device=dev, dtype=torch.float32).contiguous()
    assert t.numel() == n, "one value per tensor expected"
    return t


def multi_tensor_lamb_stage1_cuda(chunk_size, noop_flag, tensor_lists, per_tensor_decay, step,
                                  beta1, beta2, epsilon, global_grad_norm, max_global_grad_norm):
    """Legacy two-stage LAMB, stage 1 (apex csrc/multi_tensor_lamb_stage_1.cu): Adam
    moments of the clipped grad and the update u = m^/(sqrt(v^)+eps) + decay_i * p
    written into tensor_lists[4].  API parity for callers of the old interface (the
    fused path is multi_tensor_lamb).  GPU: one multi-tensor launch
    (csrc/hip/mt_optim.hip lamb_legacy1_kernel) reading the overflow flag and the global
    norm on the device; CPU: the same math from tensor ops."""
    g, p, m, v, u = tensor_lists
    if not g:
        return
    dev = p[0].device
    if dev.type == "cuda" and _native.available():
        _C().lamb_legacy_stage1(noop_flag, [list(g), list(p), list(m), list(v), list(u)],
                                _per_tensor(per_tensor_decay, len(g), dev), int(step),
                                float(beta1), float(beta2), float(epsilon),
                                _dev_scalar(global_grad_norm, dev).reshape(1),
                                float(max_global_grad_norm))
        return
    keep = noop_flag.reshape(()).to(dev).eq(0)
    gn = _dev_scalar(global_grad_norm, dev)
    mx = float(max_global_grad_norm)
    clip = torch.where(gn > mx, gn / mx, torch.ones_like(gn))
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    with torch.no_grad():
        for i in range(len(g)):
            d = per_tensor_decay[i]
            d = d.reshape(()).to(dev, torch.float32) if isinstance(d, torch.Tensor) else float(d)
            gi = g[i].float() / clip
            mn = m[i].float() * beta1 + gi * (1 - beta1)
            vn = v[i].float() * beta2 + gi * gi * (1 - beta2)
            upd = (mn / bc1) / ((vn / bc2).sqrt() + epsilon) + d * p[i].float()
            m[i].copy_(torch.where(keep, mn, m[i].float()))
            v[i].copy_(torch.where(keep, vn, v[i].float()))
            u[i].copy_(torch.where(keep, upd, u[i].float()))


def multi_tensor_lamb_stage2_cuda(chunk_size, noop_flag, tensor_lists, per_tensor_param_norm,
                                  per_tensor_update_norm, lr, weight_decay=0.0, use_nvlamb=False):
    """Legacy LAMB stage 2: p -= lr * (||p|| / ||u||) * u per tensor (trust ratio 1
    when a norm is zero, plain lr when neither weight decay nor nvlamb applies).
    GPU: one launch (lamb_legacy2_kernel); CPU: tensor ops.  No host sync either way."""
    p, u = tensor_lists[:2]
    if not p:
        return
    dev = p[0].device
    if dev.type == "cuda" and _native.available():
        _C().lamb_legacy_stage2(noop_flag, [list(p), list(u)],
                                _per_tensor(per_tensor_param_norm, len(p), dev),
                                _per_tensor(per_tensor_update_norm, len(p), dev), float(lr),
                                float(weight_decay), bool(use_nvlamb))
        return
    keep = noop_flag.reshape(()).to(dev).eq(0)
    with torch.no_grad():
        for i in range(len(p)):
            if use_nvlamb or weight_decay != 0.0:
                pn = _dev_scalar(per_tensor_param_norm[i], dev)
                un = _dev_scalar(per_tensor_update_norm[i], dev)
                ratio = torch.where((pn != 0) & (un != 0), lr * pn / un,
                                    torch.full_like(pn, float(lr)))
            else:
                ratio = _dev_scalar(lr, dev)
            step_i = u[i].float() * (ratio * keep)
            p[i].sub_(step_i.to(p[i].dtype))


def multi_tensor_novograd(chunk_size, noop_flag, tensor_lists, grad_norms, lr, beta1, beta2,
                          epsilon, step, bias_correction, weight_decay, grad_averaging, mode,
                          norm_type, *, scale=1.0, scale_inv=False):
    """Apex semantics: ``grad_norms`` already holds the blended per-tensor second
    moment (see multi_tensor_norm_out_cuda)."""
    lv, lt = _split(lr)
    sv, st = _split(scale)
    if isinstance(step, torch.Tensor):
        step_v, step_t = 0, step
    else:
        step_v, step_t = int(step), None
    # first_step=True with grad_norms == v makes the in-kernel blend the identity
    _C().novograd(noop_flag, tensor_lists, grad_norms, grad_norms, True, lv, lt, float(beta1),
                  float(beta2), float(epsilon), step_v, step_t, bool(bias_correction),
                  float(weight_decay), bool(grad_averaging), int(mode), int(norm_type), sv, st,
                  scale_inv)


def multi_tensor_adagrad(chunk_size, noop_flag, tensor_lists, lr, epsilon, mode, weight_decay, *,
                         scale=1.0, scale_inv=False):
    lv, lt = _split(lr)
    sv, st = _split(scale)
    _C().adagrad(noop_flag, tensor_lists, lv, lt, float(epsilon), int(mode), float(weight_decay),
                 sv, st, scale_inv)
