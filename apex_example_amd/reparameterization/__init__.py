"""Weight-norm reparameterization (apex@f3a960f8 apex/reparameterization/,
SURVEY.md A-22): ``apply_weight_norm(module, name='', dim=0, hook_child=True)``
replaces ``name`` (every >=2-D parameter when ``name == ''``) by ``name_g`` and
``name_v`` with w = g * v / ||v|| (norm over every dim except ``dim``),
recomputed before each forward; ``remove_weight_norm`` folds it back.
The recompute is ATen's fused ``_weight_norm`` (one norm + one scale pass).
"""
from __future__ import annotations

import torch
from torch.nn import Parameter

__all__ = ["WeightNorm", "Reparameterization", "apply_weight_norm", "remove_weight_norm",
           "apply_reparameterization", "remove_reparameterization"]


def _norm_except(v, dim):
    if dim is None or dim == -1 and v.dim() == 1:
        return v.norm()
    dims = [d for d in range(v.dim()) if d != dim]
    return v.norm(2, dim=dims, keepdim=True)


class Reparameterization(object):
    """Base class: ``compute_weight`` builds the weight from the new parameters
    before every forward (apex ``Reparameterization``)."""

    def __init__(self, name, dim, module, retain_forward=True):
        self.name = name
        self.dim = dim
        self.evaluated = False
        self.retain_forward = retain_forward
        self.reparameterization_names = []
        self.backward_hook_key = None
        self.module = module

    def compute_weight(self, module=None, name=None):
        raise NotImplementedError

    def reparameterize(self, name, weight, dim):
        raise NotImplementedError

    @staticmethod
    def apply(module, name, dim, reparameterization=None, hook_child=True):
        if reparameterization is None:
            reparameterization = WeightNorm
        names = [name] if name else [n for n, p in module.named_parameters(recurse=False)
                                     if p.dim() > 1]
        fns = []
        for n in names:
            fn = reparameterization(n, dim, module)
            weight = getattr(module, n)
            del module._parameters[n]
            new_names, new_params = fn.reparameterize(n, weight, dim)
            for nn_, p in zip(new_names, new_params):
                module.register_parameter(nn_, p)
            fn.reparameterization_names = new_names
            setattr(module, n, fn.compute_weight(module, n))
            module.register_forward_pre_hook(fn)
            fns.append(fn)
        if hook_child:
            for child in module.children():
                Reparameterization.apply(child, name, dim, reparameterization, hook_child)
        return fns

    def remove(self, module):
        weight = self.compute_weight(module, self.name)
        delattr(module, self.name)
        for n in self.reparameterization_names:
            del module._parameters[n]
        module.register_parameter(self.name, Parameter(weight.detach()))

    def __call__(self, module, inputs):
        setattr(module, self.name, self.compute_weight(module, self.name))


class WeightNorm(Reparameterization):
    def compute_weight(self, module=None, name=None):
        module = self.module if module is None else module
        name = self.name if name is None else name
        g = getattr(module, name + "_g")
        v = getattr(module, name + "_v")
        if self.dim is None or (self.dim == -1 and v.dim() == 1):
            return v * (g / v.norm())
        return torch._weight_norm(v, g, self.dim)

    def reparameterize(self, name, weight, dim):
        g = Parameter(_norm_except(weight.data, dim).detach().clone())
        v = Parameter(weight.data.detach().clone())
        return [name + "_g", name + "_v"], [g, v]


def apply_reparameterization(module, reparameterization=None, name="", dim=0, hook_child=True):
    return Reparameterization.apply(module, name, dim, reparameterization, hook_child)


def apply_weight_norm(module, name="", dim=0, hook_child=True):
    """Apply weight normalization to ``name`` of ``module`` (all >=2-D parameters
    when ``name == ''``; children too when ``hook_child``)."""
    Reparameterization.apply(module, name, dim, WeightNorm, hook_child)
    return module


def remove_reparameterization(module, reparameterization=Reparameterization, name="",
                              remove_all=False):
    for k, hook in list(module._forward_pre_hooks.items()):
        if isinstance(hook, reparameterization) and (remove_all or not name or
                                                     hook.name == name):
            hook.remove(module)
            del module._forward_pre_hooks[k]
    if remove_all or not name:
        for child in module.children():
            remove_reparameterization(child, reparameterization, name, remove_all)
    return module


def remove_weight_norm(module, name="", remove_all=False):
    return remove_reparameterization(module, WeightNorm, name, remove_all)
