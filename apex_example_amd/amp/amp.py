"""O1 ("patch torch functions") on top of ``torch.autocast``, plus the user cast
registries (apex@f3a960f8 apex/amp/amp.py + wrap.py + utils.py).

Apex O1 monkey-patches every function in its FP16/FP32/promote tables
(amp/lists/).  On PyTorch 2.10 nearly all of that policy is implemented
natively (in C++, no Python per call) by the autocast dispatch key, so
``init()`` enables autocast for the calling thread - the scope of Apex's global
patching - and ``disable_casts()`` turns it off for a region.  The entries of
Apex's tables on which autocast decides differently are found by
``amp.lists.audit`` (every table entry is called and its output dtype checked;
tests/test_amp_o1_tables.py) and patched here with Apex's decision
(``APEX_POLICY_OVERRIDES``), active only while autocast is on in the calling
thread.  The user registries keep Apex's decorator API.
"""
from __future__ import annotations

import functools
import itertools

import torch

from ._amp_state import _amp_state
from .handle import AmpHandle, NoOpHandle

_DECORATOR_HANDLE = None
_USER_CAST_REGISTRY = set()
_USER_PROMOTE_REGISTRY = set()
_APPLIED = {}


def _half_dtype():
    h = _amp_state.handle if hasattr(_amp_state, "handle") else None
    return getattr(h, "_dtype", torch.float16)


def _cast(x, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(dtype) if x.is_floating_point() else x
    if isinstance(x, (list, tuple)):
        return type(x)(_cast(v, dtype) for v in x)
    if isinstance(x, dict):
        return {k: _cast(v, dtype) for k, v in x.items()}
    return x


def _widest(args):
    order = {torch.float16: 0, torch.bfloat16: 1, torch.float32: 2, torch.float64: 3}
    best = None
    for a in itertools.chain(args):
        if isinstance(a, torch.Tensor) and a.is_floating_point():
            if best is None or order.get(a.dtype, 2) > order.get(best, 2):
                best = a.dtype
    return best


def _no_autocast(fn_call):
    prev = {d: torch.is_autocast_enabled(d) for d in ("cuda", "cpu")}
    for d in prev:
        torch.set_autocast_enabled(d, False)
    try:
        return fn_call()
    finally:
        for d, v in prev.items():
            torch.set_autocast_enabled(d, v)


def half_function(fn):
    """Decorator: run ``fn`` with floating tensor args cast to the half dtype."""
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        dt = _half_dtype()
        return _no_autocast(lambda: fn(*_cast(args, dt), **_cast(kwargs, dt)))
    return wrapper


def float_function(fn):
    """Decorator: run ``fn`` with floating tensor args cast to fp32."""
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        return _no_autocast(lambda: fn(*_cast(args, torch.float32), **_cast(kwargs, torch.float32)))
    return wrapper


def promote_function(fn):
    """Decorator: cast floating tensor args to the widest floating type present."""
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        dt = _widest(list(args) + list(kwargs.values()))
        if dt is None:
            return fn(*args, **kwargs)
        return _no_autocast(lambda: fn(*_cast(args, dt), **_cast(kwargs, dt)))
    return wrapper


def _autocast_on():
    return torch.is_autocast_enabled("cuda") or torch.is_autocast_enabled("cpu")


def _policy_float(fn):
    """Apex FP32_FUNCS entry that autocast leaves in the input dtype: under
    autocast, run it in fp32 (floating args cast, autocast off inside)."""
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        if not _autocast_on():
            return fn(*args, **kwargs)
        return _no_autocast(lambda: fn(*_cast(args, torch.float32),
                                       **_cast(kwargs, torch.float32)))
    wrapper._amp_policy_original = fn
    return wrapper


# Apex FP32_FUNCS entries whose autocast (CUDA, fp16 and bf16) policy differs:
# autocast runs them in the input dtype.  Found by amp.lists.audit.
APEX_POLICY_OVERRIDES = (
    ("torch", "std"), ("torch", "var"),
    ("tensor", "std"), ("tensor", "var"),
    ("F", "gelu"), ("F", "grid_sample"), ("F", "ctc_loss"),
)
_POLICY_APPLIED = []


def _ns(name):
    import torch.nn.functional as F
    return {"torch": torch, "tensor": torch.Tensor, "F": F}[name]


def _apply_policy_overrides():
    if _POLICY_APPLIED:
        return
    for ns, name in APEX_POLICY_OVERRIDES:
        mod = _ns(ns)
        orig = getattr(mod, name)
        setattr(mod, name, _policy_float(orig))
        _POLICY_APPLIED.append((mod, name, orig))


def _restore_policy_overrides():
    while _POLICY_APPLIED:
        mod, name, orig = _POLICY_APPLIED.pop()
        setattr(mod, name, orig)


def _register(module, name, kind):
    if not hasattr(module, name):
        raise ValueError("No function named {} in module {}.".format(name, module))
    if kind == "promote":
        _USER_PROMOTE_REGISTRY.add((module, name))
    else:
        _USER_CAST_REGISTRY.add((module, name, kind))
    if hasattr(_amp_state, "handle") and isinstance(_amp_state.handle, AmpHandle):
        _apply_registries()


def register_half_function(module, name):
    _register(module, name, "half")


def register_float_function(module, name):
    _register(module, name, "float")


def register_promote_function(module, name):
    _register(module, name, "promote")


def _apply_registries():
    for module, name, kind in list(_USER_CAST_REGISTRY):
        key = (id(module), name)
        if key in _APPLIED:
            continue
        orig = getattr(module, name)
        _APPLIED[key] = (module, name, orig)
        setattr(module, name, half_function(orig) if kind == "half" else float_function(orig))
    for module, name in list(_USER_PROMOTE_REGISTRY):
        key = (id(module), name)
        if key in _APPLIED:
            continue
        orig = getattr(module, name)
        _APPLIED[key] = (module, name, orig)
        setattr(module, name, promote_function(orig))


def _restore_registries():
    for module, name, orig in _APPLIED.values():
        setattr(module, name, orig)
    _APPLIED.clear()


def init(enabled=True, loss_scale="dynamic", enable_caching=True, verbose=False,
         allow_banned=False, dtype=torch.float16, device_type=None):
    """Activate O1 casting for this thread (apex.amp.init)."""
    global _DECORATOR_HANDLE
    if not enabled:
        handle = NoOpHandle()
        _DECORATOR_HANDLE = handle
        return handle
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cpu" and dtype == torch.float16:
        dtype = torch.bfloat16  # CPU autocast policy is defined for bf16
    handle = AmpHandle(loss_scale, enable_caching, verbose, dtype=dtype, device_type=device_type)
    torch.set_autocast_dtype(device_type, dtype)
    torch.set_autocast_enabled(device_type, True)
    torch.set_autocast_cache_enabled(enable_caching)
    if allow_banned:
        import torch.nn.functional as F

        register_float_function(F, "binary_cross_entropy")
    _amp_state.handle = handle
    _apply_policy_overrides()
    _apply_registries()
    _DECORATOR_HANDLE = handle
    return handle


def deinit():
    """Undo ``init`` (used by tests and by re-initialisation)."""
    h = getattr(_amp_state, "handle", None)
    if h is not None:
        h._deactivate()
    _restore_policy_overrides()
    _restore_registries()
