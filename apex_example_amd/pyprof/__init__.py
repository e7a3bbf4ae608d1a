"""Op-level profiling for rocprofv3 (apex.pyprof re-targeted).

Apex's pyprof monkey-patched every torch function to push an NVTX range with
the op name, shapes and dtypes, then post-processed nvprof SQLite.  Here:

* :func:`init` / :class:`annotate` - a ``TorchFunctionMode`` (no monkey
  patching) that brackets every torch op called from Python with a roctx range
  ``"<op>(shape dtype, ...)"``; module-level ranges via :func:`annotate_modules`
  (forward hooks push ``"module:<name>"``).  roctx = ``torch.cuda.nvtx`` on ROCm.
* :mod:`.parse` - reads a ``rocprofv3 --kernel-trace --marker-trace`` CSV run,
  attributes each kernel to the innermost enclosing op range on its thread and
  aggregates time per op signature and per kernel (with FLOP estimates for
  matmul-like ops), as apex.pyprof.prof did for nvprof.

    from apex_example_amd import pyprof
    with pyprof.annotate():
        loss = model(x).sum(); loss.backward()
    # rocprofv3 --kernel-trace --marker-trace --output-format csv -d out -- python train.py
    # python -m apex_example_amd.pyprof.parse out
"""
from __future__ import annotations

import contextlib

import torch
from torch.overrides import TorchFunctionMode

from .flops import op_flops  # noqa: F401

_SKIP = {"__get__", "__set__", "size", "dim", "numel", "is_contiguous", "stride", "data_ptr",
         "element_size", "__len__", "__format__", "__repr__", "shape", "dtype", "device",
         "is_floating_point", "requires_grad_", "__hash__", "__eq__", "__bool__", "item",
         "tolist", "storage_offset", "is_complex", "layout", "grad", "_version",
         "requires_grad", "is_leaf", "grad_fn", "names", "__iter__"}


def _fmt(a):
    if isinstance(a, torch.Tensor):
        return "%s %s" % ("x".join(str(s) for s in a.shape) or "scalar",
                          str(a.dtype).replace("torch.", ""))
    if isinstance(a, (list, tuple)) and a and isinstance(a[0], torch.Tensor):
        return "[%d tensors]" % len(a)
    return None


def signature(func, args, kwargs=None):
    name = getattr(func, "__name__", None) or str(func)
    parts = [p for p in (_fmt(a) for a in args) if p]
    for k, v in (kwargs or {}).items():
        p = _fmt(v)
        if p:
            parts.append("%s=%s" % (k, p))
    return "%s(%s)" % (name, ", ".join(parts))


class annotate(TorchFunctionMode):
    """Context manager: every torch op inside gets a roctx range."""

    def __init__(self, enabled=True, record_shapes=True):
        super().__init__()
        self.enabled = enabled and torch.cuda.is_available()
        self.record_shapes = record_shapes

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = getattr(func, "__name__", "")
        if not self.enabled or name in _SKIP:
            return func(*args, **kwargs)
        label = signature(func, args, kwargs) if self.record_shapes else name
        torch.cuda.nvtx.range_push(label)
        try:
            return func(*args, **kwargs)
        finally:
            torch.cuda.nvtx.range_pop()


_global_mode = None


def init(record_shapes=True):
    """Enable op annotation for the rest of the program (apex.pyprof.nvtx.init)."""
    global _global_mode
    if _global_mode is None:
        _global_mode = annotate(record_shapes=record_shapes)
        _global_mode.__enter__()
    return _global_mode


def stop():
    global _global_mode
    if _global_mode is not None:
        _global_mode.__exit__(None, None, None)
        _global_mode = None


def annotate_modules(model, prefix="module"):
    """Push/pop a roctx range around every submodule's forward."""
    handles = []
    if not torch.cuda.is_available():
        return handles
    for name, mod in model.named_modules():
        label = "%s:%s" % (prefix, name or type(mod).__name__)

        def pre(m, inp, _label=label):
            torch.cuda.nvtx.range_push(_label)

        def post(m, inp, out):
            torch.cuda.nvtx.range_pop()

        handles.append(mod.register_forward_pre_hook(pre))
        handles.append(mod.register_forward_hook(post))
    return handles


@contextlib.contextmanager
def range(name):  # noqa: A001  (mirrors torch.cuda.nvtx.range)
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_pop()
