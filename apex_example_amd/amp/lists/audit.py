"""Audit of the O1 cast policy against Apex's tables (apex@f3a960f8
apex/amp/lists/{torch,tensor,functional}_overrides.py and tests/L0/run_amp/
test_basic_casts.py / test_promotion.py).

Every entry of every Apex table gets a small call recipe; ``audit()`` runs each
recipe under the active O1 state and compares the output dtype with what Apex's
policy prescribes:

* FP16_FUNCS   - fp32 inputs      -> the half dtype (fp16, or bf16 when amp runs bf16)
* FP32_FUNCS   - half inputs      -> fp32
* CASTS        - (half, fp32) mix -> the widest type (fp32); comparisons -> bool;
                 in-place ops keep the dtype of their first operand
* SEQUENCE_CASTS - cat / stack of (half, fp32) -> fp32
* BANNED_FUNCS - raise under O1 (unless ``allow_banned``)

``audit`` works on real GPU tensors and, for the CUDA autocast policy on a
CPU-only host, on FakeTensorMode "cuda" tensors (no device needed).
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn.functional as F

from . import functional_overrides as FO
from . import tensor_overrides as TO
from . import torch_overrides as TT

# entries whose Apex behaviour is deliberately not reproduced (with the reason)
KNOWN_DIFFERENCES = {
    ("tensor", "cpu"): "Apex's O1 made Tensor.cpu() return fp32 copies of half tensors; "
                       "patching the device-transfer method changes checkpoint / logging "
                       "dtypes for every caller, so it stays a plain copy here",
    ("tensor", "__ipow__"): "Apex's fp32 wrapper turned `x **= y` on a half tensor into an "
                            "OUT-of-place fp32 result (other aliases of x never see the "
                            "update); here it stays in place in x's dtype",
}


# FakeTensorMode cannot run these (data-dependent / device-only kernels); the GPU
# audit covers them on real tensors
FAKE_UNVERIFIABLE = (("torch", "equal"), ("tensor", "equal"), ("F", "ctc_loss"))


def _mk(device):
    def t(shape, dtype, positive=False, requires_grad=False):
        x = torch.rand(shape, device=device) + 0.5 if positive else \
            torch.randn(shape, device=device)
        return x.to(dtype)
    return t


def _long(shape, high, device):
    return torch.randint(0, high, shape, device=device)


def _recipes(device):
    """name -> fn(t, half, full) returning the op's output (t: tensor factory)."""
    L = lambda s, h: _long(s, h, device)  # noqa: E731
    r = {}
    # ---------------------------------------------------------------- fp16 (torch / F)
    conv = {
        "conv1d": lambda t, d: torch.conv1d(t((1, 4, 8), d), t((4, 4, 3), d)),
        "conv2d": lambda t, d: torch.conv2d(t((1, 4, 8, 8), d), t((4, 4, 3, 3), d)),
        "conv3d": lambda t, d: torch.conv3d(t((1, 4, 4, 4, 4), d), t((4, 4, 3, 3, 3), d)),
        "conv_transpose1d": lambda t, d: torch.conv_transpose1d(t((1, 4, 8), d), t((4, 4, 3), d)),
        "conv_transpose2d": lambda t, d: torch.conv_transpose2d(t((1, 4, 8, 8), d),
                                                                t((4, 4, 3, 3), d)),
        "conv_transpose3d": lambda t, d: torch.conv_transpose3d(t((1, 4, 4, 4, 4), d),
                                                                t((4, 4, 3, 3, 3), d)),
        "conv_tbc": lambda t, d: torch.conv_tbc(t((8, 1, 4), d), t((3, 4, 4), d), t((4,), d), 1),
    }
    for k, f in conv.items():
        r[("torch", k)] = f
    r[("F", "conv_tbc")] = lambda t, d: F.conv_tbc(t((8, 1, 4), d), t((3, 4, 4), d),
                                                   t((4,), d), 1)
    r[("F", "conv1d")] = lambda t, d: F.conv1d(t((1, 4, 8), d), t((4, 4, 3), d))
    r[("F", "conv2d")] = lambda t, d: F.conv2d(t((1, 4, 8, 8), d), t((4, 4, 3, 3), d))
    r[("F", "conv3d")] = lambda t, d: F.conv3d(t((1, 4, 4, 4, 4), d), t((4, 4, 3, 3, 3), d))
    r[("F", "conv_transpose1d")] = lambda t, d: F.conv_transpose1d(t((1, 4, 8), d),
                                                                   t((4, 4, 3), d))
    r[("F", "conv_transpose2d")] = lambda t, d: F.conv_transpose2d(t((1, 4, 8, 8), d),
                                                                   t((4, 4, 3, 3), d))
    r[("F", "conv_transpose3d")] = lambda t, d: F.conv_transpose3d(t((1, 4, 4, 4, 4), d),
                                                                   t((4, 4, 3, 3, 3), d))
    r[("F", "linear")] = lambda t, d: F.linear(t((2, 4), d), t((3, 4), d), t((3,), d))
    r[("torch", "prelu")] = lambda t, d: torch.prelu(t((2, 4, 3), d), t((1,), d))
    r[("torch", "addmm")] = lambda t, d: torch.addmm(t((4, 4), d), t((4, 4), d), t((4, 4), d))
    r[("torch", "addmv")] = lambda t, d: torch.addmv(t((4,), d), t((4, 4), d), t((4,), d))
    r[("torch", "addr")] = lambda t, d: torch.addr(t((4, 4), d), t((4,), d), t((4,), d))
    r[("torch", "matmul")] = lambda t, d: torch.matmul(t((4, 4), d), t((4, 4), d))
    r[("torch", "mm")] = lambda t, d: torch.mm(t((4, 4), d), t((4, 4), d))
    r[("torch", "mv")] = lambda t, d: torch.mv(t((4, 4), d), t((4,), d))
    r[("tensor", "__matmul__")] = lambda t, d: t((4, 4), d).__matmul__(t((4, 4), d))
    for k in ("prelu", "addmm", "addmv", "addr", "matmul", "mm", "mv"):
        r[("tensor", k)] = (lambda k_: lambda t, d: (lambda a: getattr(a[0], k_)(*a[1:]))(
            _tensor_self_args(k_, t, d)))(k)
    # ---------------------------------------------------------------- fp32 (torch)
    for k in ("acos", "asin", "cosh", "erfinv", "exp", "expm1", "log", "log10", "log2", "log1p",
              "reciprocal", "rsqrt", "sinh", "tan"):
        pos = k not in ("acos", "asin", "erfinv")
        r[("torch", k)] = (lambda k_, p_: lambda t, d: getattr(torch, k_)(
            t((4, 4), d, positive=p_) * (1.0 if p_ else 0.5)))(k, pos)
        r[("tensor", k)] = (lambda k_, p_: lambda t, d: getattr(
            t((4, 4), d, positive=p_) * (1.0 if p_ else 0.5), k_)())(k, pos)
    r[("torch", "pow")] = lambda t, d: torch.pow(t((4, 4), d, positive=True), 2)
    r[("tensor", "pow")] = lambda t, d: t((4, 4), d, positive=True).pow(2)
    for k in ("cumprod", "cumsum"):
        r[("torch", k)] = (lambda k_: lambda t, d: getattr(torch, k_)(t((4, 4), d), 0))(k)
        r[("tensor", k)] = (lambda k_: lambda t, d: getattr(t((4, 4), d), k_)(0))(k)
    r[("torch", "dist")] = lambda t, d: torch.dist(t((4, 4), d), t((4, 4), d))
    r[("tensor", "dist")] = lambda t, d: t((4, 4), d).dist(t((4, 4), d))
    for k in ("norm", "prod", "std", "sum", "var"):
        r[("torch", k)] = (lambda k_: lambda t, d: getattr(torch, k_)(t((4, 4), d)))(k)
        r[("tensor", k)] = (lambda k_: lambda t, d: getattr(t((4, 4), d), k_)())(k)
    r[("torch", "renorm")] = lambda t, d: torch.renorm(t((4, 4), d), 2, 0, 1.0)
    r[("tensor", "renorm")] = lambda t, d: t((4, 4), d).renorm(2, 0, 1.0)
    r[("tensor", "__pow__")] = lambda t, d: t((4, 4), d, positive=True).__pow__(2)
    r[("tensor", "__rpow__")] = lambda t, d: t((4, 4), d).__rpow__(2)
    r[("tensor", "__ipow__")] = lambda t, d: t((4, 4), d, positive=True).__ipow__(2)
    r[("tensor", "cpu")] = lambda t, d: t((4, 4), d).cpu()
    # ---------------------------------------------------------------- fp32 (F)
    f32 = {
        "interpolate": lambda t, d: F.interpolate(t((1, 4, 8, 8), d), scale_factor=2,
                                                  mode="bilinear", align_corners=False),
        "grid_sample": lambda t, d: F.grid_sample(t((1, 4, 8, 8), d),
                                                  t((1, 8, 8, 2), d).clamp(-1, 1),
                                                  align_corners=False),
        "softplus": lambda t, d: F.softplus(t((4, 4), d)),
        "softmin": lambda t, d: F.softmin(t((4, 4), d), dim=1),
        "log_softmax": lambda t, d: F.log_softmax(t((4, 4), d), dim=1),
        "softmax": lambda t, d: F.softmax(t((4, 4), d), dim=1),
        "gelu": lambda t, d: F.gelu(t((4, 4), d)),
        "layer_norm": lambda t, d: F.layer_norm(t((4, 4), d), (4,)),
        "group_norm": lambda t, d: F.group_norm(t((2, 4, 8), d), 2),
        "local_response_norm": lambda t, d: F.local_response_norm(t((1, 4, 8, 8), d), 2),
        "normalize": lambda t, d: F.normalize(t((4, 4), d)),
        "cosine_similarity": lambda t, d: F.cosine_similarity(t((4, 4), d), t((4, 4), d)),
        "poisson_nll_loss": lambda t, d: F.poisson_nll_loss(t((4, 4), d), t((4, 4), d,
                                                                          positive=True)),
        "cosine_embedding_loss": lambda t, d: F.cosine_embedding_loss(
            t((4, 4), d), t((4, 4), d), torch.ones(4, device=t((1,), d).device)),
        "cross_entropy": lambda t, d: F.cross_entropy(t((4, 4), d), L((4,), 4)),
        "hinge_embedding_loss": lambda t, d: F.hinge_embedding_loss(
            t((4, 4), d), torch.ones(4, 4, device=t((1,), d).device)),
        "kl_div": lambda t, d: F.kl_div(t((4, 4), d), t((4, 4), d, positive=True),
                                        reduction="batchmean"),
        "l1_loss": lambda t, d: F.l1_loss(t((4, 4), d), t((4, 4), d)),
        "mse_loss": lambda t, d: F.mse_loss(t((4, 4), d), t((4, 4), d)),
        "margin_ranking_loss": lambda t, d: F.margin_ranking_loss(
            t((4,), d), t((4,), d), torch.ones(4, device=t((1,), d).device)),
        "multilabel_margin_loss": lambda t, d: F.multilabel_margin_loss(t((4, 4), d),
                                                                        L((4, 4), 4)),
        "multilabel_soft_margin_loss": lambda t, d: F.multilabel_soft_margin_loss(
            t((4, 4), d), t((4, 4), d, positive=True).round().clamp(0, 1)),
        "multi_margin_loss": lambda t, d: F.multi_margin_loss(t((4, 4), d), L((4,), 4)),
        "nll_loss": lambda t, d: F.nll_loss(t((4, 4), d), L((4,), 4)),
        "binary_cross_entropy_with_logits": lambda t, d: F.binary_cross_entropy_with_logits(
            t((4, 4), d), t((4, 4), d, positive=True).clamp(0, 1)),
        "smooth_l1_loss": lambda t, d: F.smooth_l1_loss(t((4, 4), d), t((4, 4), d)),
        "soft_margin_loss": lambda t, d: F.soft_margin_loss(
            t((4, 4), d), torch.ones(4, 4, device=t((1,), d).device)),
        "triplet_margin_loss": lambda t, d: F.triplet_margin_loss(t((4, 4), d), t((4, 4), d),
                                                                  t((4, 4), d)),
        "ctc_loss": lambda t, d: F.ctc_loss(
            F.log_softmax(t((6, 2, 5), torch.float32), 2).to(d), L((2, 3), 4) + 1,
            torch.full((2,), 6, dtype=torch.long), torch.full((2,), 3, dtype=torch.long)),
    }
    for k, f in f32.items():
        r[("F", k)] = f
    # ---------------------------------------------------------------- promote / casts
    two = {"add": "add", "div": "div", "mul": "mul", "atan2": "atan2", "eq": "eq", "ge": "ge",
           "gt": "gt", "le": "le", "lt": "lt", "ne": "ne", "equal": "equal"}
    for k in two:
        r[("torch", k)] = (lambda k_: lambda t, h, f: getattr(torch, k_)(t((4, 4), h),
                                                                          t((4, 4), f)))(k)
        r[("tensor", k)] = (lambda k_: lambda t, h, f: getattr(t((4, 4), h), k_)(
            t((4, 4), f)))(k)
    r[("torch", "addcdiv")] = lambda t, h, f: torch.addcdiv(t((4, 4), h), t((4, 4), f),
                                                            t((4, 4), f, positive=True))
    r[("torch", "addcmul")] = lambda t, h, f: torch.addcmul(t((4, 4), h), t((4, 4), f),
                                                            t((4, 4), f))
    r[("torch", "cross")] = lambda t, h, f: torch.cross(t((4, 3), h), t((4, 3), f), dim=1)
    r[("torch", "bilinear")] = lambda t, h, f: torch.bilinear(t((2, 4), h), t((2, 4), f),
                                                              t((3, 4, 4), f), t((3,), f))
    r[("torch", "dot")] = lambda t, h, f: torch.dot(t((4,), h), t((4,), f))
    for k in ("addcdiv", "addcmul", "cross", "dot"):
        r[("tensor", k)] = (lambda k_: lambda t, h, f: r[("torch", k_)](t, h, f))(k)
    dunder = {"__add__", "__div__", "__eq__", "__ge__", "__gt__", "__le__", "__lt__", "__mul__",
              "__ne__", "__radd__", "__rdiv__", "__rmul__", "__rsub__", "__rtruediv__",
              "__sub__", "__truediv__"}
    for k in dunder:
        r[("tensor", k)] = (lambda k_: lambda t, h, f: _dunder(t((4, 4), h, positive=True), k_,
                                                               t((4, 4), f, positive=True)))(k)
    for k in ("__iadd__", "__idiv__", "__imul__", "__isub__", "__itruediv__"):
        r[("tensor", k)] = (lambda k_: lambda t, h, f: _dunder(t((4, 4), h, positive=True), k_,
                                                               t((4, 4), f, positive=True)))(k)
    r[("torch", "cat")] = lambda t, h, f: torch.cat([t((2, 4), h), t((2, 4), f)])
    r[("torch", "stack")] = lambda t, h, f: torch.stack([t((2, 4), h), t((2, 4), f)])
    # ---------------------------------------------------------------- banned
    r[("F", "binary_cross_entropy")] = lambda t, d: F.binary_cross_entropy(
        torch.sigmoid(t((4, 4), d)), t((4, 4), d, positive=True).clamp(0, 1))
    return r


def _tensor_self_args(k, t, d):
    shapes = {"prelu": ((2, 4, 3), (1,)), "addmm": ((4, 4), (4, 4), (4, 4)),
              "addmv": ((4,), (4, 4), (4,)), "addr": ((4, 4), (4,), (4,)),
              "matmul": ((4, 4), (4, 4)), "mm": ((4, 4), (4, 4)), "mv": ((4, 4), (4,))}
    return [t(s, d) for s in shapes[k]]


def _dunder(a, name, b):
    if name in ("__div__", "__rdiv__", "__idiv__"):
        # Python 3 spells these __truediv__ / __rtruediv__ / __itruediv__
        name = {"__div__": "__truediv__", "__rdiv__": "__rtruediv__",
                "__idiv__": "__itruediv__"}[name]
    return getattr(a, name)(b)


def _tables():
    """[(namespace, name, kind)] for every entry of Apex's tables."""
    out = []
    for n in TT.FP16_FUNCS:
        out.append(("torch", n, "fp16"))
    for n in TT.FP32_FUNCS:
        out.append(("torch", n, "fp32"))
    for n in TT.CASTS:
        out.append(("torch", n, "promote"))
    for n in TT.SEQUENCE_CASTS:
        out.append(("torch", n, "sequence"))
    for n in FO.FP16_FUNCS:
        out.append(("F", n, "fp16"))
    for n in FO.FP32_FUNCS:
        out.append(("F", n, "fp32"))
    for n, _ in FO.BANNED_FUNCS:
        out.append(("F", n, "banned"))
    # Apex only patched the Tensor methods that exist (hasattr check)
    for n in TO.FP16_FUNCS:
        if hasattr(torch.Tensor, n):
            out.append(("tensor", n, "fp16"))
    for n in TO.FP32_FUNCS:
        if hasattr(torch.Tensor, n):
            out.append(("tensor", n, "fp32"))
    for n in TO.CASTS:
        if hasattr(torch.Tensor, n) or n in ("__div__", "__rdiv__", "__idiv__"):
            out.append(("tensor", n, "promote"))
    seen, uniq = set(), []
    for e in out:
        if e[:2] not in seen:
            seen.add(e[:2])
            uniq.append(e)
    return uniq


def expected(kind, name, half):
    if kind == "fp16":
        return half
    if kind == "fp32":
        return torch.float32
    if kind == "sequence":
        return torch.float32
    if kind == "promote":
        if name.lstrip("_").rstrip("_") in ("eq", "ge", "gt", "le", "lt", "ne"):
            return torch.bool
        if name == "equal":
            return bool
        if name.startswith("__i"):
            return half  # in-place: the first operand keeps its dtype
        return torch.float32
    return "raises"


def audit(device="cuda", half=torch.float16, fake=False, skip_known=True):
    """Run every table entry under the CURRENT amp state (call after
    ``amp.init`` / ``amp.initialize(opt_level="O1")``).  Returns a list of
    mismatches ``(namespace, name, kind, expected, got)``; empty = parity."""
    ctx = contextlib.nullcontext()
    unverifiable = ()
    if fake:
        unverifiable = FAKE_UNVERIFIABLE
        from torch._subclasses.fake_tensor import FakeTensorMode
        ctx = FakeTensorMode(allow_non_fake_inputs=True)
    bad = []
    with ctx:
        t = _mk(device)
        recipes = _recipes(device)
        for ns, name, kind in _tables():
            if (skip_known and (ns, name) in KNOWN_DIFFERENCES) or (ns, name) in unverifiable:
                continue
            fn = recipes.get((ns, name))
            if fn is None:
                bad.append((ns, name, kind, "a recipe", "none"))
                continue
            want = expected(kind, name, half)
            try:
                if kind in ("promote", "sequence"):
                    out = fn(t, half, torch.float32)
                elif kind == "fp16":
                    out = fn(t, torch.float32)
                else:
                    out = fn(t, half)
            except Exception as e:  # noqa: BLE001
                got = "raises" if kind == "banned" else "error: %s" % str(e).splitlines()[0][:80]
                if got != want:
                    bad.append((ns, name, kind, want, got))
                continue
            got = type(out) if not isinstance(out, torch.Tensor) else out.dtype
            if got != want:
                bad.append((ns, name, kind, want, got))
    return bad
