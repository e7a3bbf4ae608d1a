"""Fused dense layers (apex.fused_dense API: ``FusedDense``, ``FusedDenseGeluDense``,
``DenseNoBias`` and the ``fused_dense_function`` / ``fused_dense_gelu_dense_function``
functionals), MI355X-native.

Forward: hipBLASLt GEMMs with the bias in the GEMM (``addmm``).  Backward: the
data / weight gradients are hipBLASLt GEMMs; the bias gradients (column sums of
dY, which PyTorch's generic reduction runs at ~1 TB/s) and the GELU backward of
the FFN run on ``csrc/hip/bias_grad.hip``: one split-row column-sum pass at HBM
rate, and for the FFN one pass that forms dpre = dh * gelu'(pre) AND its column
sums (no extra read of dpre for the first bias).

Under autocast (amp O1) the operands are cast once in forward and the casted
copies saved, so backward runs plain half-precision GEMMs (no second weight
cast); bias gradients are reduced in fp32 and written in the bias's dtype.

``FusedDenseGeluDense(approximate="tanh")`` - apex's semantics: its cuBLASLt GELU
epilogues are the tanh approximation - runs the GELU inside hipBLASLt epilogues
both ways (csrc/torch/lt_ops.cpp): forward GELU_AUX_BIAS (h and the
pre-activation from one GEMM), backward DGELU_BGRAD (dpre and the first bias
gradient from the dh GEMM).  Shapes / dtypes the library has no algorithm for
fall back to GEMM + the kernels above.
"""
from __future__ import annotations

import collections
import os
import threading

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native
from ..ops import _bias_handoff, _ddp_direct
from ..ops.conv import _SideWgrad, _side_out

__all__ = ["FusedDense", "FusedDenseGeluDense", "DenseNoBias", "fused_dense_function", "cast_params_once",
           "fused_dense_gelu_dense_function", "dense_no_bias_function", "fused_dense_skip_function",
           "fused_dense_gelu_dense_skip_function"]


def _compute_dtype(x):
    if torch.is_autocast_enabled("cuda") and x.is_cuda:
        return torch.get_autocast_dtype("cuda")
    return x.dtype


# Per-thread state (nn.DataParallel runs replica forwards in threads):
#   active: {id(param): (param, 16-bit copy)} while a cast_params_once() block runs
#   bufs:   persistent flat buffers, one per parameter list (LRU of _MAX_BUFS)
_TLS = threading.local()
_MAX_BUFS = 4


def _tls():
    if not hasattr(_TLS, "active"):
        _TLS.active, _TLS.bufs = None, collections.OrderedDict()
        _TLS.copy_of, _TLS.fresh = {}, {}
    return _TLS


def _cast(t, dt):
    if t is None or t.dtype == dt:
        return t
    active = _tls().active
    if active is not None:
        e = active.get(id(t))
        # identity + shape check: a recycled id() never matches a stale copy
        if e is not None and e[0] is t and e[1].dtype == dt and e[1].shape == t.shape:
            return e[1]
    return t.to(dt)


# The 16-bit copies of cast_params_once written by the fused optimizer's step (FusedAdam
# depth-5 launch) instead of a separate cast pass over every parameter at the next forward
# (GPT-2-medium O1: one 2.1 GB multi-tensor pass, ~340 us per step).  A/B switch.
_O1_FUSED_COPIES = os.environ.get("APEX_AMD_O1_FUSED_COPIES", "1") == "1"
O1_CAST_SKIPPED = [0]


def o1_copy_of(p):
    """The 16-bit copy cast_params_once keeps for fp32 parameter p, or None."""
    if not _O1_FUSED_COPIES:
        return None
    e = _tls().copy_of.get(id(p))
    return e[1] if e is not None and e[0] is p and e[1].shape == p.shape else None


def o1_mark_fresh(params, copies):
    """The optimizer step just wrote ``copies`` from the updated ``params``."""
    fresh = _tls().fresh
    for p, c in zip(params, copies):
        fresh[id(p)] = (p, p._version, c.data_ptr())


class cast_params_once:
    """amp O1 weight casts for a whole forward in ONE multi-tensor launch: the fp32
    parameters are written as 16-bit copies into one flat buffer (``mt.scale``
    with factor 1: plain round-to-nearest casts, the same values ``.to()`` gives),
    and the dense layers' ``_cast`` picks them up instead of launching one cast
    kernel per weight and bias (~200 small launches per GPT-2-medium step).
    Re-cast on every entry, so an optimizer step between forwards is seen.

    The flat buffer (and the zeroed no-op flag) persist per parameter list, so
    the data pointers - and with them the cached multi-tensor launch plan - are
    the same every step.  Contract that follows: the copies a graph saved for
    backward are refreshed by the next forward of the same parameter list, so
    run a graph's backward before changing the weights and re-running forward
    (every ordinary training loop does).  With grad disabled (eval / no_grad)
    nothing is batched: per-layer casts are freed right after their GEMM
    instead of keeping every 16-bit copy live for the whole forward."""

    def __init__(self, params, dtype):
        self.params, self.dtype, self.prev = params, dtype, None

    def __enter__(self):
        st = _tls()
        self.prev = st.active
        if not torch.is_grad_enabled():
            return self
        ps = [p for p in self.params if p.is_cuda and p.dtype == torch.float32]
        if not ps or not _native.available():
            return self
        key = (self.dtype, ps[0].device, tuple(id(p) for p in ps))
        ent = st.bufs.get(key)
        if ent is None or any(a is not b or o.shape != b.shape
                              for a, b, o in zip(ent[0], ps, ent[1])):
            # each copy starts 16-byte aligned (8 halves): the kernel's vector path
            pad = [(p.numel() + 7) // 8 * 8 for p in ps]
            flat = torch.empty(sum(pad), dtype=self.dtype, device=ps[0].device)
            outs, off = [], 0
            for p, n in zip(ps, pad):
                outs.append(flat[off:off + p.numel()].view(p.shape))
                off += n
            noop = torch.zeros(1, dtype=torch.int32, device=ps[0].device)
            ent = (list(ps), outs, noop)
            st.bufs[key] = ent
            while len(st.bufs) > _MAX_BUFS:
                st.bufs.popitem(last=False)
        st.bufs.move_to_end(key)
        # a fused optimizer that wrote these very copies in its step (o1_mark_fresh) and
        # nothing modified a parameter since (version counters unchanged): no re-cast
        fresh = st.fresh
        if not (_O1_FUSED_COPIES and all(
                (f := fresh.get(id(p))) is not None and f[0] is p and f[1] == p._version
                and f[2] == o.data_ptr() for p, o in zip(ps, ent[1]))):
            _native.require().mt.scale(ent[2], [[p.detach() for p in ps], ent[1]], 1.0)
        else:
            O1_CAST_SKIPPED[0] += 1
        for p in ps:
            fresh.pop(id(p), None)
        for p, o in zip(ps, ent[1]):
            st.copy_of[id(p)] = (p, o)
        st.active = {id(p): (p, o) for p, o in zip(ps, ent[1])}
        return self

    def __exit__(self, *exc):
        _tls().active = self.prev
        return False


# Split-K for the dense weight gradients (tools/microbench.py wgrad-dense,
# profiles/microbench_wgrad_dense.txt): dW[out, in] = dY^T X reduces over all T tokens
# into only 16-64 output tiles of 256 x 256, too few workgroups for 256 CUs, so one
# GEMM runs at 300-870 TF.  Cutting T into S chunks (>= 2048 tokens each, S x tiles
# <= 256) gives one batched GEMM with fp32 partials + the slab reduction kernel
# writing the weight dtype: BERT-large (T = 16384) 101 -> 53 us for 1024 x 1024,
# 163 -> 130 us for 3072 x 1024, 168 -> 150 us for 4096 x 1024; GPT-2 O1 (T = 8192,
# fp32 dW) 57 -> 39 us / 91 -> 83 us, but slower at 64 tiles there.
_DENSE_SPLITK = True


def _splitk_chunks(T, o, i, in_dtype, out_dtype):
    tiles = -(-o // 256) * -(-i // 256)
    if tiles > (64 if out_dtype == in_dtype else 48):
        return 1
    S = 1
    while S < 16 and T % (2 * S) == 0 and T // (2 * S) >= 2048 and 2 * S * tiles <= 256:
        S *= 2
    return S


# O1 fp32 bucket-view weight gradients accumulate inside the GEMM (torch.addmm
# out_dtype=fp32, beta = 1) instead of mm + add: GPT-2-medium with forced world-1
# collectives 227.2 / 227.3 -> 229.5 / 229.2 k tok/s (same box).  Cleared on the first
# failure.
_ADDMM_F32 = True


# Dense weight gradients on the own transposed-operand MFMA kernel (csrc/hip/wgrad4w.hip):
# fp32 partials per row split + the slab reduction, for weights with both dimensions
# multiples of 256 and >= 48 output tiles of 256 x 256 (the FFN and QKV projections).
# Same box (profiles/r5/wgrad_dense.md): BERT FFN 114.5 vs 136.8 us, QKV 103.5 vs 107.6 us,
# GPT-2 FFN 69.7 vs 83.5 us against the hipBLASLt split-K path; the 1024 x 1024 attention
# output projection (16 tiles) stays on hipBLASLt (57.8 vs 47.8 us).
_DENSE_W4W = True
_W4W_MIN_TILES = 48


# workgroups per weight-gradient launch: 256 (one 256 x 256 tile per CU) on the main
# stream; on the weight-gradient SIDE stream at most 128 - the kernel holds 128 KB of LDS
# per workgroup for its whole K loop, so a full grid there keeps the main stream's
# kernels (LayerNorm backward, attention, the data-gradient GEMMs) off every CU until a
# tile finishes.  GPT-2-medium O1 (fp32 weight gradients on the side stream), same box:
# 260.9 / 260.4 k tok/s with 256, 268.3 / 267.6 k with 128 (profiles/r5/ab_wg/).
_W4W_MAX_WG = 256
_W4W_MAX_WG_SIDE = 128


def _w4w_splits(T, o, i, max_wg=None):
    """Row splits for wgrad4w: the largest power of two with splits x tiles <= max_wg (256:
    one 256 x 256 tile per CU), at least 1024 rows (16 K-tiles) per split."""
    cap = _W4W_MAX_WG if max_wg is None else max_wg
    tiles = (o // 256) * (i // 256)
    S = 1
    while 2 * S * tiles <= cap and T % (2 * S * 64) == 0 and T // (2 * S) >= 1024:
        S *= 2
    return S


# The bias gradient of a wgrad4w layer from the kernel's own dY fragments (column sums via
# v_dot2 next to the MFMAs, csrc/hip/wgrad4w.hip variant 4) instead of a separate
# column-sum pass over dy.
_W4W_BIAS = True


def _wgrad_w4w(dy2, x2, dtype, out, accumulate, side=False, b_dtype=None):
    """wgrad4w when the shapes / dtypes fit, else None; with ``b_dtype`` the pair
    (dW, db) with db = column sums of dy2 formed inside the same kernel."""
    if not (_DENSE_W4W and dy2.is_cuda and dtype in (torch.bfloat16, torch.float32)
            and dy2.dtype in (torch.bfloat16, torch.float16) and x2.dtype == dy2.dtype
            and _native.available()):
        return None
    T, o = dy2.shape
    i = x2.shape[1]
    if o % 256 or i % 256 or (o // 256) * (i // 256) < _W4W_MIN_TILES:
        return None
    dn = _native.require().dense
    S = _w4w_splits(T, o, i, _W4W_MAX_WG_SIDE if side else None)
    if not dn.wgrad4w_ok(dy2, x2, S):
        return None
    if out is not None and not out.is_contiguous():
        return None
    if b_dtype is not None:
        if b_dtype not in (torch.float32, torch.bfloat16, torch.float16):
            return None
        r, db = dn.wgrad4w_bias(dy2, x2, S, dtype, out=out, accumulate=accumulate,
                                bias_dtype=b_dtype)
        return (out if out is not None else r), db
    r = dn.wgrad4w(dy2, x2, S, dtype, out=out, accumulate=accumulate)
    return out if out is not None else r


def _wgrad(dy2, x2, dtype, out=None, accumulate=True, side=False):
    """dW = dy2^T x2 written in the parameter's dtype by the GEMM itself (amp O1:
    fp16 operands, fp32 weight -> no separate fp16->fp32 cast of dW); split-K over
    the tokens when the output has too few tiles to fill the GPU.  ``out``: accumulate
    into that [o, i]-contiguous tensor (a DDP bucket view, see _direct_slots) and
    return it - the slab reduction or the GEMM's beta = 1 does the add; with
    ``accumulate=False`` (a lazily zeroed bucket view) overwrite it (beta = 0)."""
    got = _wgrad_w4w(dy2, x2, dtype, out, accumulate, side)
    if got is not None:
        return got
    if (_DENSE_SPLITK and dy2.is_cuda and dtype in (torch.bfloat16, torch.float32)
            and dy2.dtype in (torch.bfloat16, torch.float16) and x2.dtype == dy2.dtype
            and _native.available()):
        T, o = dy2.shape
        i = x2.shape[1]
        S = _splitk_chunks(T, o, i, dy2.dtype, dtype)
        if S > 1 and (o * i) % 4 == 0 and dy2.is_contiguous() and x2.is_contiguous():
            a = dy2.view(S, T // S, o).transpose(1, 2)
            b = x2.view(S, T // S, i)
            part = torch.bmm(a, b, out_dtype=torch.float32)
            return _native.require().conv.splitk_reduce(part, dtype, out=out,
                                                        accumulate=accumulate)
    if dtype != dy2.dtype and dy2.is_cuda and dtype == torch.float32:
        global _ADDMM_F32
        if out is not None and _ADDMM_F32:
            # fp32 C (+)= fp16 A @ B in the GEMM (beta = 1 / 0), no separate add pass
            o2 = out.view(dy2.size(1), x2.size(1))
            try:
                torch.addmm(o2, dy2.t(), x2, beta=1 if accumulate else 0,
                            out_dtype=torch.float32, out=o2)
                return out
            except (RuntimeError, TypeError):
                _ADDMM_F32 = False
        r = torch.mm(dy2.t(), x2, out_dtype=torch.float32)
        if out is None:
            return r
        return out.add_(r.view_as(out)) if accumulate else out.copy_(r.view_as(out))
    if out is not None:
        if out.dtype == dy2.dtype:
            return out.view(dy2.size(1), x2.size(1)).addmm_(
                dy2.t(), x2, beta=1 if accumulate else 0).view_as(out)
        r = (dy2.t() @ x2).view_as(out)
        return out.add_(r) if accumulate else out.copy_(r)
    return dy2.t() @ x2


def _direct_slots(side, weight, w_dtype):
    """DDP reducer slots when the weight gradient can accumulate straight into the
    weight's bucket view on the compute stream (ops/_ddp_direct.py: no AccumulateGrad
    add kernel per weight - GPT-2-medium O1 under DDP ran 96 of them, ~1.4 ms per step,
    `profiles/gpt2_medium_forced_collectives_r3.md`), else None."""
    if side is None or side.on or weight is None:
        return None
    sl = _ddp_direct.slots(weight)
    if sl is None:
        return None
    g, _acc = _ddp_direct.grad_target(weight)
    if g is None or not g.is_cuda or g.dtype != w_dtype or not g.is_contiguous():
        return None
    return sl


def _side_wgrad(side, weight, w_dtype, dy2, x2):
    """The weight-gradient closure for ``side.run``: under a DDP-mode side stream it
    writes the (possibly lazily zeroed) bucket view itself (ops/conv.py _side_out) - no
    fresh gradient + copy per weight (96 copies / 1.3 ms per GPT-2 step before)."""
    so, sa = _side_out(side, weight)
    if so is not None and so.dtype != w_dtype:
        so, sa = None, True
    on = bool(side is not None and side.on)
    return lambda: _wgrad(dy2, x2, w_dtype, out=so, accumulate=sa, side=on)


def _side_wgrad_bgrad(side, weight, w_dtype, b_dtype, dy2, x2):
    """As _side_wgrad for a (weight, bias) pair: dW into the bucket view, db fresh."""
    so, sa = _side_out(side, weight)
    if so is None or so.dtype != w_dtype:
        return lambda: _wgrad_bgrad(dy2, x2, w_dtype, b_dtype)
    on = bool(side is not None and side.on)
    return lambda: _wgrad_bgrad(dy2, x2, w_dtype, b_dtype, out=so, accumulate=sa, side=on)


def _wgrad_maybe_direct(side, weight, w_dtype, dy2, x2, *used):
    """The weight gradient for autograd, or None after accumulating it into the DDP
    bucket view and announcing the parameter to the reducer."""
    direct = _direct_slots(side, weight, w_dtype)
    if direct is None:
        return side.run(_side_wgrad(side, weight, w_dtype, dy2, x2), dy2, *used)
    tgt, acc = _ddp_direct.grad_target(weight)
    _wgrad(dy2, x2, w_dtype, out=tgt, accumulate=acc)
    _ddp_direct.mark_ready(direct)
    return None


def _bias_grad(g2, dtype):
    hs = _bias_handoff.take(g2, dtype)  # summed by the residual join's backward already
    if hs is not None:
        return hs
    if g2.is_cuda and _native.available():
        return _native.require().dense.bias_grad(g2, dtype)
    return g2.to(torch.promote_types(g2.dtype, torch.float32)).sum(0).to(dtype)


def _shares_storage(a, b):
    return a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()


def _dgrad(g2, w, xshape, dskip, dy=None):
    """dX = g2 @ W, accumulated IN PLACE into the residual-branch gradient ``dskip``
    (C += A @ B, hipBLASLt beta = 1) when the input also fed a residual: the sum
    autograd would otherwise launch over the input gradient disappears.  ``dskip``
    is the fresh gradient buffer the residual consumer's backward produced - except
    when autograd hands this layer's own output gradient to both branches (an
    unfused ``x + dense(x)``): then ``dskip`` IS ``dy``, which the weight gradient
    (possibly on the side stream) still reads, so the sum is formed out of place."""
    if dskip is not None:
        alias = _shares_storage(dskip, g2) or (dy is not None and _shares_storage(dskip, dy))
        if dskip.dtype == g2.dtype and dskip.is_contiguous() and not alias:
            return dskip.view(-1, w.size(1)).addmm_(g2, w).view(xshape)
        acc = torch.promote_types(dskip.dtype, torch.float32)
        return (dskip.to(acc) + (g2 @ w).view(xshape).to(acc)).to(dskip.dtype)
    return (g2 @ w).view(xshape)


def _dense_fwd(ctx, x, weight, bias):
    dt = _compute_dtype(x)
    with torch.autocast("cuda", enabled=False):
        xc, wc, bc = _cast(x, dt), _cast(weight, dt), _cast(bias, dt)
        x2 = xc.reshape(-1, xc.size(-1))
        y = torch.addmm(bc, x2, wc.t()) if bc is not None else x2 @ wc.t()
    ctx.save_for_backward(xc, wc)
    ctx.bias_dtype = bias.dtype if bias is not None else None
    ctx.w_dtype = weight.dtype
    ctx.params = (weight, bias)  # leaves: side-stream weight gradients check .grad
    if ctx.needs_input_grad[1]:
        _ddp_direct.note_use(weight)
    return y.view(*x.shape[:-1], weight.size(0))


def _side_dense(w_dtype, kind="attn"):
    """Dense weight gradients on the side stream (ops/conv.py _SideWgrad) only for fp32
    weights (amp O1: the fp32 weight-gradient GEMMs overlap the fp16 data-gradient
    chain): GPT-2-medium O1 239.5 / 239.9 k -> 246.5 / 249.0 k tok/s, while BERT-large
    O2 (bf16 weights) measured 666.6 / 666.7 -> 648.7 / 648.7 seq/s (same box); the
    attention-only / FFN-only splits for BERT measured 664.4 and 645.4 seq/s against
    664.5 (round 4) and 722-724 against 728 (round 5, profiles/r5/ab_bert_side_final/)."""
    del kind
    return w_dtype == torch.float32


def _dense_bwd(ctx, dy, dskip=None):
    xc, wc = ctx.saved_tensors
    dx = dw = db = None
    if dy is None:
        return dskip, None, None
    dy2 = dy.reshape(-1, dy.size(-1)).contiguous()
    if dy2.dtype != wc.dtype:
        dy2 = dy2.to(wc.dtype)
    need_b = ctx.bias_dtype is not None and ctx.needs_input_grad[2]
    side = _SideWgrad(*ctx.params, enable=_side_dense(ctx.w_dtype)) \
        if ctx.needs_input_grad[1] else None
    if ctx.needs_input_grad[0]:
        dx = _dgrad(dy2, wc, xc.shape, dskip, dy)
    x2 = xc.reshape(-1, xc.size(-1))
    direct = _direct_slots(side, ctx.params[0], ctx.w_dtype) if ctx.needs_input_grad[1] else None
    if direct is not None and need_b:
        # the weight gradient straight into its bucket view, db from the same kernel
        # where wgrad4w takes the layer (_wgrad_bgrad)
        tgt, acc = _ddp_direct.grad_target(ctx.params[0])
        _, db = _wgrad_bgrad(dy2, x2, ctx.w_dtype, ctx.bias_dtype, out=tgt, accumulate=acc)
        _ddp_direct.mark_ready(direct)
    elif direct is not None:
        dw = _wgrad_maybe_direct(side, ctx.params[0], ctx.w_dtype, dy2, x2, xc)
    elif ctx.needs_input_grad[1] and need_b:
        dw, db = side.run(_side_wgrad_bgrad(side, ctx.params[0], ctx.w_dtype, ctx.bias_dtype,
                                            dy2, x2), dy2, xc)
    elif ctx.needs_input_grad[1]:
        dw = side.run(_side_wgrad(side, ctx.params[0], ctx.w_dtype, dy2, x2), dy2, xc)
    elif need_b:
        db = _bias_grad(dy2, ctx.bias_dtype)
    return dx, dw, db


class FusedDenseFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        return _dense_fwd(ctx, x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        return _dense_bwd(ctx, dy)


class FusedDenseSkipFunc(torch.autograd.Function):
    """(dense(x), x): the dense layer whose input also feeds a residual branch
    (BERT's QKV projection and FFN input).  Backward receives both gradients and
    forms dx = dskip + dy @ W as one accumulating GEMM."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        return _dense_fwd(ctx, x, weight, bias), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dskip):
        return _dense_bwd(ctx, dy, dskip)


# hipBLASLt GELU epilogues (csrc/torch/lt_ops.cpp) for the tanh-GELU FFN where the own
# gemm4w epilogues do not apply (tests turn it off to compare with the unfused kernels)
_LT_GELU = True


def _lt_ok(*ts):
    return (_LT_GELU and all(t is not None and t.is_cuda for t in ts)
            and ts[0].dtype in (torch.bfloat16, torch.float16)
            and all(t.dtype == ts[0].dtype for t in ts) and _native.available())


# (op, shapes, dtypes) the library offered no algorithm for: not asked again
_LT_MISSING = set()


def _lt_call(name, *args):
    """Run a hipBLASLt epilogue op of csrc/torch/lt_ops.cpp; None when the library
    has no algorithm for this problem (remembered, so the fallback is direct)."""
    key = (name,) + tuple((tuple(a.shape), a.dtype) if isinstance(a, torch.Tensor) else a
                          for a in args)
    if key in _LT_MISSING:
        return None
    res = getattr(_native.require().dense, name)(*args)
    if not res:
        _LT_MISSING.add(key)
        return None
    return res


# BGRADB (bias gradient inside the weight-gradient GEMM) is opt-in: the library's
# BGRADB kernels for gfx950 are far slower than its plain GEMMs - BERT-large
# 592 -> 421 seq/s when enabled (same box) - so the plain GEMM + the column-sum
# kernel stay the default
_LT_BGRAD = False


def _wgrad_bgrad(dy2, x2, w_dtype, b_dtype, out=None, accumulate=True, side=False):
    """(dW, db): db handed over by a fused residual join (ops/_bias_handoff.py), else
    wgrad4w forming db from its own dY fragments, else the weight-gradient GEMM + the
    column-sum kernel, or (opt-in) one hipBLASLt GEMM with the BGRADB epilogue.  ``out`` /
    ``accumulate``: as _wgrad (a DDP bucket view)."""
    hs = _bias_handoff.take(dy2, b_dtype)
    if hs is None and _W4W_BIAS:
        got = _wgrad_w4w(dy2, x2, w_dtype, out, accumulate, side, b_dtype=b_dtype)
        if got is not None:
            return got
    if hs is None and out is None and _LT_BGRAD and _lt_ok(dy2, x2):
        res = _lt_call("wgrad_bgrad_lt", dy2, x2, w_dtype, b_dtype)
        if res is not None:
            return res
    dw = _wgrad(dy2, x2, w_dtype, out=out, accumulate=accumulate, side=side)
    return dw, (hs if hs is not None else _bias_grad(dy2, b_dtype))


# The FFN on the own MFMA GEMM with its epilogues: forward h = gelu(x W1^T + b1) keeping
# the pre-activation (no separate GELU pass), backward dpre = (dy W2) * gelu'(pre) with the
# b1 gradient's column sums (no dh round trip, no column-sum kernels).  bf16 / fp16
# operands, N % 256 == 0, K % 64 == 0.  Default on the one-wave-per-SIMD gemm4w
# (csrc/hip/gemm4w.hip): BERT-large FFN forward 152 us fused vs 164 us for hipBLASLt
# addmm + the GELU pass, backward 194 vs 217 us (profiles/r5/gemm4w_bench.md).


def _g4w_ok(a, b, *more):
    if not (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16)
            and b.dtype == a.dtype
            and all(t is None or t.dtype in (a.dtype, torch.float32) for t in more)
            and _native.available()):
        return False
    return _native.require().dense.gemm4w_ok(a, b)


_T_KERNEL = True


def _transposed(w):
    """w^T contiguous, built on every call.  No cache: the fused optimizers and amp's
    master -> model copy write weights through their data pointers without bumping the
    version counter, so a cache keyed on (version, data_ptr) would go stale silently;
    the transpose is one small pass (8 MB for a BERT-large W2) per backward - on the
    64 x 64 LDS-tiled transpose kernel (conv.transpose_weight): ATen's strided copy took
    25-33 us per layer for it (0.6 ms per BERT-large step, 0.8 ms per GPT-2-medium step)."""
    if (_T_KERNEL and w.is_cuda and w.dim() == 2 and w.element_size() == 2
            and w.is_contiguous() and _native.available()):
        o, i = w.shape
        return _native.require().conv.transpose_weight(w.view(o, i, 1, 1)).view(i, o)
    return w.t().contiguous()


def _gelu_dense_fwd(ctx, x, w1, b1, w2, b2, approximate):
    dt = _compute_dtype(x)
    with torch.autocast("cuda", enabled=False):
        xc = _cast(x, dt)
        w1c, b1c, w2c, b2c = _cast(w1, dt), _cast(b1, dt), _cast(w2, dt), _cast(b2, dt)
        x2 = xc.reshape(-1, xc.size(-1))
        res = None
        if approximate in ("tanh", "none") and _g4w_ok(x2, w1c, b1c):
            h, pre = _native.require().dense.gemm4w(x2, w1c, 1, bias=b1c, want_pre=True,
                                                    tanh=approximate == "tanh")
            res = (h, pre)
        elif approximate == "tanh" and _lt_ok(x2, w1c, b1c):
            # one GEMM: h = gelu(x W1^T + b1) with pre as the epilogue's aux output
            res = _lt_call("gelu_fwd_lt", x2, w1c, b1c)
        if res is not None:
            h, pre = res
        else:
            pre = torch.addmm(b1c, x2, w1c.t()) if b1c is not None else x2 @ w1c.t()
            if pre.is_cuda and _native.available():
                h = _native.require().dense.gelu(pre, approximate == "tanh")
            else:
                h = F.gelu(pre, approximate=approximate)
        y = torch.addmm(b2c, h, w2c.t()) if b2c is not None else h @ w2c.t()
    ctx.save_for_backward(xc, w1c, pre, h, w2c)
    ctx.b1_dtype = b1.dtype if b1 is not None else None
    ctx.b2_dtype = b2.dtype if b2 is not None else None
    ctx.tanh = approximate == "tanh"
    ctx.w_dtypes = (w1.dtype, w2.dtype)
    ctx.params = (w1, b1, w2, b2)
    _ddp_direct.note_use(*(w for w, k in ((w1, 1), (w2, 3)) if ctx.needs_input_grad[k]))
    return y.view(*x.shape[:-1], w2.size(0))


def _gelu_dense_bwd(ctx, dy, dskip=None):
    if dy is None:
        return dskip, None, None, None, None, None
    xc, w1c, pre, h, w2c = ctx.saved_tensors
    dy2 = dy.reshape(-1, dy.size(-1)).contiguous()
    if dy2.dtype != w2c.dtype:
        dy2 = dy2.to(w2c.dtype)
    need = ctx.needs_input_grad
    dw2 = db2 = None
    need_b2 = ctx.b2_dtype is not None and need[4]
    w1, b1, w2, b2 = ctx.params
    side2 = _SideWgrad(w2, b2, enable=_side_dense(ctx.w_dtypes[1], "ffn")) if need[3] else None
    if need[3] and _direct_slots(side2, w2, ctx.w_dtypes[1]) is not None:
        dw2 = _wgrad_maybe_direct(side2, w2, ctx.w_dtypes[1], dy2, h)
        if need_b2:
            db2 = _bias_grad(dy2, ctx.b2_dtype)
    elif need[3] and need_b2:
        dw2, db2 = side2.run(_side_wgrad_bgrad(side2, w2, ctx.w_dtypes[1], ctx.b2_dtype, dy2, h),
                             dy2, h)
    elif need[3]:
        dw2 = side2.run(_side_wgrad(side2, w2, ctx.w_dtypes[1], dy2, h), dy2, h)
    elif need_b2:
        db2 = _bias_grad(dy2, ctx.b2_dtype)
    res = None
    w2t = None
    if (dy2.dtype in (torch.bfloat16, torch.float16) and pre.dtype == dy2.dtype
            and w2c.dtype == dy2.dtype and pre.is_contiguous() and dy2.is_cuda):
        w2t = _transposed(w2c)
        if not _g4w_ok(dy2, w2t):
            w2t = None
    if w2t is not None:
        # one GEMM on the own kernel: dpre = (dy W2) * gelu'(pre) + the b1 column sums
        res = tuple(_native.require().dense.gemm4w(
            dy2, w2t, 2, aux=pre, tanh=ctx.tanh,
            bias_grad_dtype=ctx.b1_dtype or dy2.dtype))
    elif ctx.tanh and _lt_ok(dy2, w2c, pre):
        # one GEMM: dpre = (dy W2) * gelu'(pre) and its column sums, dh never stored
        res = _lt_call("dgelu_bgrad_lt", dy2, w2c, pre, ctx.b1_dtype or dy2.dtype)
    if res is not None:
        dpre, db1 = res
    elif dy2.is_cuda and _native.available():
        dh = dy2 @ w2c
        dpre, db1 = _native.require().dense.gelu_bwd_bias_grad(
            dh, pre, ctx.tanh, ctx.b1_dtype or dh.dtype)
    else:
        dh = dy2 @ w2c
        with torch.enable_grad():
            p = pre.detach().to(torch.promote_types(pre.dtype, torch.float32))
            p.requires_grad_(True)
            g, = torch.autograd.grad(F.gelu(p, approximate="tanh" if ctx.tanh else "none"),
                                     p, dh.to(p.dtype))
        dpre = g.to(dh.dtype)
        db1 = _bias_grad(dpre, ctx.b1_dtype or dh.dtype)
    side1 = _SideWgrad(w1, enable=_side_dense(ctx.w_dtypes[0], "ffn")) if need[1] else None
    dx = _dgrad(dpre, w1c, xc.shape, dskip, dy) if need[0] else None
    x2 = xc.reshape(-1, xc.size(-1))
    dw1 = _wgrad_maybe_direct(side1, w1, ctx.w_dtypes[0], dpre, x2, xc) if need[1] else None
    if ctx.b1_dtype is None or not need[2]:
        db1 = None
    return dx, dw1, db1, dw2, db2, None


class FusedDenseGeluDenseFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, approximate):
        return _gelu_dense_fwd(ctx, x, w1, b1, w2, b2, approximate)

    @staticmethod
    def backward(ctx, dy):
        return _gelu_dense_bwd(ctx, dy)


class FusedDenseGeluDenseSkipFunc(torch.autograd.Function):
    """(dense2(gelu(dense1(x))), x) with dx = dskip + dpre @ W1 in one GEMM."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, approximate):
        return _gelu_dense_fwd(ctx, x, w1, b1, w2, b2, approximate), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dskip):
        return _gelu_dense_bwd(ctx, dy, dskip)


def fused_dense_function(x, weight, bias):
    return FusedDenseFunc.apply(x, weight, bias)


def fused_dense_skip_function(x, weight, bias):
    """(dense(x), x) - use the second output as the residual so that the input
    gradient is one accumulating GEMM (see FusedDenseSkipFunc)."""
    return FusedDenseSkipFunc.apply(x, weight, bias)


def fused_dense_gelu_dense_skip_function(x, w1, b1, w2, b2, approximate="none"):
    return FusedDenseGeluDenseSkipFunc.apply(x, w1, b1, w2, b2, approximate)


def dense_no_bias_function(x, weight):
    return FusedDenseFunc.apply(x, weight, None)


def fused_dense_gelu_dense_function(x, w1, b1, w2, b2, approximate="none"):
    return FusedDenseGeluDenseFunc.apply(x, w1, b1, w2, b2, approximate)


class FusedDense(nn.Linear):
    """nn.Linear with the fused backward (same parameters / state dict)."""

    def forward(self, x):
        return fused_dense_function(x, self.weight, self.bias)


class DenseNoBias(nn.Linear):
    def __init__(self, in_features, out_features, device=None, dtype=None):
        super().__init__(in_features, out_features, bias=False, device=device, dtype=dtype)

    def forward(self, x):
        return dense_no_bias_function(x, self.weight)


class FusedDenseGeluDense(nn.Module):
    """Linear -> GELU -> Linear (apex naming: weight1/bias1/weight2/bias2)."""

    def __init__(self, in_features, intermediate_features, out_features, bias=True,
                 approximate="none"):
        super().__init__()
        self.in_features, self.intermediate_features = in_features, intermediate_features
        self.out_features, self.approximate = out_features, approximate
        l1 = nn.Linear(in_features, intermediate_features, bias=bias)
        l2 = nn.Linear(intermediate_features, out_features, bias=bias)
        self.weight1, self.bias1 = l1.weight, l1.bias
        self.weight2, self.bias2 = l2.weight, l2.bias

    def forward(self, x):
        return fused_dense_gelu_dense_function(x, self.weight1, self.bias1, self.weight2,
                                               self.bias2, self.approximate)
