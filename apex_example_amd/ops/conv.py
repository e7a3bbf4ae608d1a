"""1x1 convolution as a plain GEMM on channels-last activations.

A stride-1 1x1 convolution over an NHWC tensor is exactly
``y[M, Cout] = x[M, Cin] @ W[Cout, Cin]^T`` with M = N*H*W, and the activation is
already that matrix in memory (channels_last), so forward and data-gradient are
library GEMMs (hipBLASLt via ``torch.mm``) with no layout change.  Measured on
MI355X at ResNet-50 bs256 shapes (tools/microbench.py conv1x1, docs/PERF.md),
hipBLASLt beats MIOpen's 1x1 forward/dgrad kernels by 1.2-4x.

The weight gradient dW[co, ci] = sum_m dY[m, co] X[m, ci] is a long-K GEMM
(K = N*H*W up to 802,816) with a tiny output, which a single GEMM cannot spread
over 256 CUs.  It runs split-K: the M rows are cut into S chunks, one batched
hipBLASLt GEMM computes the S partial products with fp32 output, and one sum
reduces them - ~2x faster than MIOpen's wgrad on ResNet-50's layer2-4 shapes
(tools/microbench.py wgrad, profiles/microbench_wgrad.txt).  S targets ~3k rows
per chunk.
"""
from __future__ import annotations

import collections
import os
import threading

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native
from . import _ddp_direct
from .batch_norm import bn_src_of

# Weight gradients on a side stream (APEX_AMD_WGRAD_STREAM=0 disables; a documented
# debugging switch, docs/KNOBS.md): the data
# gradient stays on the critical path of the main stream while the weight gradient
# (MFMA-bound) runs beside it and beside the following BatchNorm backward passes
# (HBM-bound); the main stream joins the side stream once, at the end of the
# backward pass (an autograd final callback).  Used only where nothing reads the
# gradient on the main stream before that join: world size 1 (no DDP bucket hooks)
# and the weight's .grad is None (AccumulateGrad then stores the tensor without a
# kernel); never inside a graph capture.
_USE_WSTREAM = os.environ.get("APEX_AMD_WGRAD_STREAM", "1") == "1"
_SIDE = {}          # device index -> side stream
_JOIN = {}          # device index -> (main stream to join, autograd graph task id)
_LOCK = threading.Lock()


def _ddp_slot(p):
    """(reducer, index) when ``p.grad`` is a DDP bucket view whose reducer can take a
    side-stream gradient this iteration (parallel/distributed.py), else None."""
    return _ddp_direct.slot(p)


def _side_mode(params):
    """'free': every param's .grad is None (AccumulateGrad stores the side-stream tensor
    without a kernel; world size 1 only: no bucket hooks read it before the join);
    'ddp': every param's .grad is a DDP bucket view - the side stream accumulates into
    the view itself and announces it to the reducer (csrc/torch/reducer.cpp
    mark_ready_on_stream), which launches that bucket's all-reduce behind an event of
    the side stream instead of the compute stream; None: no side stream."""
    ps = [p for p in params if p is not None]
    if not _USE_WSTREAM or not ps or not ps[0].is_cuda:
        return None
    if torch.cuda.is_current_stream_capturing():
        return None
    if all(p.grad is None for p in ps) and not any(
            getattr(p, "_amd_grad_is_bucket_view", False) for p in ps):
        # (a DDP parameter whose bucket view was lazily zeroed also has no .grad, but its
        # ready hook copies the gradient on the compute stream: never 'free')
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return None
        return "free"
    if _DDP_SIDE and all(_ddp_slot(p) is not None for p in ps):
        return "ddp"
    return None


# Side-stream weight gradients under DDP (APEX_AMD_WGRAD_STREAM_DDP=0 disables): on a
# HIGH-priority side stream of their own (its wgrads then keep pace with the data
# gradients instead of trailing them; the last buckets wait for the side stream) with a
# bounded lag.  ResNet-50 with forced world-1 collectives, same box: 9,865 / 9,871 img/s
# without, 8,083 / 8,079 with a normal-priority side stream (exposed tail 0.9 ms),
# 10,418 / 10,417 with the high-priority one (tail 0.14 ms) - 98.6 % of the plain step
# (profiles/r4/).
_DDP_SIDE = os.environ.get("APEX_AMD_WGRAD_STREAM_DDP", "1") == "1"
# Bounded side-stream lag under DDP: the main stream waits for the weight gradient
# enqueued 4 launches earlier (the last buckets cannot launch before the side stream
# reaches their gradients); unbounded in the single-GPU 'free' mode.  The side stream has
# high priority under DDP, normal priority in the 'free' mode (same box: 10,565 / 10,534
# img/s normal vs 10,531 / 10,500 high there).  Measured and removed in round 6: a
# CU-masked side stream (1/4-3/4 of every XCD: GPT-2 247 -> 129-154 k tok/s, ResNet-50
# 10,566 -> 7,181 img/s, profiles/r4/m/) and gating the side stream behind the LayerNorm
# backward passes (neutral on GPT-2, profiles/r5/ab_wg/).
_SIDE_EVENTS = {}   # device index -> deque of side-stream events, oldest first


# test hook (tests/test_ddp_gpu.py race test): GPU cycles the side stream sleeps before
# each weight gradient, to skew it against the compute stream and the bucket streams
_TEST_SIDE_SLEEP = 0


def _join_side():
    with _LOCK:
        pending = list(_JOIN.items())
        _JOIN.clear()
        for idx, _ in pending:
            _SIDE_EVENTS.pop(idx, None)
    for idx, (main, _task) in pending:
        for key, side in list(_SIDE.items()):
            if key[0] == idx:
                main.wait_stream(side)


def _lag_for(mode):
    return 4 if mode == "ddp" else 0


def join_side_streams():
    """Make every main stream wait for the weight-gradient side stream now (also
    what the end-of-backward callback does).  Idempotent; for code that reads a
    weight gradient before its backward pass finished (e.g. after an exception)."""
    _join_side()


class _SideWgrad:
    """Fork point taken BEFORE the data gradient is enqueued, so the weight gradient
    launched afterwards on the side stream can overlap it."""

    def __init__(self, weight, *more, enable=True):
        self.params = (weight,) + more
        self.mode = _side_mode(self.params) if enable else None
        self.on = self.mode is not None
        if self.on:
            dev = weight.device
            self.main = torch.cuda.current_stream(dev)
            high = self.mode == "ddp"
            key = (dev.index, high)
            self.side = _SIDE.get(key)
            if self.side is None:
                prio = torch.cuda.Stream.priority_range()[1] if high else 0
                self.side = torch.cuda.Stream(dev, priority=prio)
                _SIDE[key] = self.side
            self.ev = self.main.record_event()

    def run(self, fn, *used):
        if not self.on:
            return fn()
        self.side.wait_event(self.ev)
        with torch.cuda.stream(self.side):
            if _TEST_SIDE_SLEEP:
                torch.cuda._sleep(_TEST_SIDE_SLEEP)
            dw = fn()
            outs = dw if isinstance(dw, tuple) else (dw,)
            if self.mode == "ddp":
                # accumulate into the bucket views on the side stream (what
                # AccumulateGrad would do on the compute stream), then hand autograd
                # None so nothing reads them on the compute stream before the join
                with torch.no_grad():
                    for p, g in zip(self.params, outs):
                        if g is None:
                            continue
                        tgt, acc = _ddp_direct.grad_target(p)
                        if g.data_ptr() == tgt.data_ptr():
                            continue  # written into the view by the kernel itself
                        if acc:
                            tgt.add_(g)
                        else:  # a lazily zeroed bucket view: overwrite
                            tgt.copy_(g)
        for t in used:
            t.record_stream(self.side)
        for t in outs:
            if t is not None:
                t.record_stream(self.main if self.mode == "free" else self.side)
        idx = self.main.device.index
        # one join per backward pass (graph task): a pass that raised before its final
        # callbacks ran leaves a stale entry behind; the next pass sees another task id
        # and queues its own callback, which joins everything pending
        task = torch._C._current_graph_task_id()
        lag = _lag_for(self.mode)
        wait_ev = None
        with _LOCK:
            ent = _JOIN.get(idx)
            fresh = ent is None or ent[1] != task
            if fresh:
                _JOIN[idx] = (self.main, task)
                _SIDE_EVENTS.pop(idx, None)
            if lag > 0:
                q = _SIDE_EVENTS.setdefault(idx, collections.deque())
                q.append(self.side.record_event())
                if len(q) > lag:
                    wait_ev = q.popleft()
        if wait_ev is not None:
            # the main stream may run at most `lag` weight gradients ahead of the side stream
            self.main.wait_event(wait_ev)
        if fresh:
            torch.autograd.Variable._execution_engine.queue_callback(_join_side)
        sid = self.side.cuda_stream
        if self.mode == "ddp":
            for p, g in zip(self.params, outs):
                if g is not None:
                    red, i = _ddp_slot(p)
                    red.mark_ready_on_stream(i, sid)
        else:
            # 'free': store the side-stream tensor as .grad here (what AccumulateGrad
            # would do without a kernel) and hand autograd None.  Another use of the
            # parameter (a penalty term, a second call of the module) then reaches
            # AccumulateGrad alone, whose pre-hook makes the compute stream wait for this
            # side stream before adding into .grad (csrc/torch/reducer.cpp
            # side_grad_announce); returning the tensor instead would let autograd sum
            # the two on the compute stream before the side stream has written it.
            if not all(g is None or (p.grad is None and g.dtype == p.dtype
                                     and g.shape == p.shape and g.device == p.device)
                       for p, g in zip(self.params, outs)):
                raise RuntimeError("side-stream weight gradient does not match its parameter")
            announce = _native.require().reducer.side_grad_announce
            for p, g in zip(self.params, outs):
                if g is not None:
                    p.grad = g
                    announce(p, sid)
        none = tuple(None for _ in outs)
        return none if isinstance(dw, tuple) else None


def _side_out(side, weight, cl=False):
    """(bucket view, accumulate) that a DDP-mode side-stream weight gradient writes into
    directly - same kernels and rounding as the main-stream direct path; a lazily zeroed
    bucket (``weight.grad`` None) is overwritten (accumulate False, GEMM beta = 0) -
    else (None, True).  Without it the side stream computed a fresh gradient and copied
    it into the view: 59 copies / 0.3 ms per ResNet-50 step and 96 / 1.3 ms per GPT-2
    step in the forced-collective profiles (`__amd_rocclr_copyBuffer`)."""
    if side is None or not side.on or side.mode != "ddp":
        return None, True
    g, acc = _ddp_direct.grad_target(weight)
    if g is None:
        return None, True
    ok = g.is_contiguous(memory_format=torch.channels_last) if cl else g.is_contiguous()
    return (g, acc) if ok else (None, True)


def _wgrad_1x1_w(dy, x, weight, out=None, accumulate=True):
    """1x1 weight gradient shaped like the weight, or accumulated into (written to, with
    ``accumulate=False``) ``out`` - returned as the very same tensor, so a DDP-mode side
    stream knows not to add it again."""
    r = wgrad_1x1(_as_rows(dy), _as_rows(x), weight.dtype, out=out, accumulate=accumulate)
    return r if out is not None else r.view(weight.shape)


# maximum row splits of the 1x1 weight gradients (A/B knob: the split-K GEMMs run on the
# weight-gradient side stream, where a smaller grid leaves more CUs to the main stream)
_SPLITK_MAX = int(os.environ.get("APEX_AMD_WGRAD1X1_SPLITS", "128"))


def _split_k(m):
    s = 1
    while s < _SPLITK_MAX and m % (2 * s) == 0 and m // (2 * s) >= 2048:
        s *= 2
    return s


def wgrad_1x1(dy_rows, x_rows, out_dtype, out=None, accumulate=True):
    """dW[co, ci] = dy_rows^T @ x_rows, split-K over the rows (fp32 partials).  ``out``:
    accumulate into that [co, ci]-contiguous gradient (a DDP bucket view) instead, or
    overwrite it (``accumulate=False``: a lazily zeroed bucket view)."""
    m, co = dy_rows.shape
    ci = x_rows.shape[1]
    S = _split_k(m)
    if S == 1:
        r = torch.mm(dy_rows.t(), x_rows, out_dtype=torch.float32).to(out_dtype)
    else:
        a = dy_rows.view(S, m // S, co).transpose(1, 2)
        b = x_rows.view(S, m // S, ci)
        part = torch.bmm(a, b, out_dtype=torch.float32)
        if (_USE_SPLITK_REDUCE and out_dtype in (torch.bfloat16, torch.float32)
                and (co * ci) % 4 == 0):
            # one two-stage slab reduction writing the weight dtype directly
            r = _native.require().conv.splitk_reduce(
                part, out_dtype, out.view(co, ci) if out is not None else None, accumulate)
            return out if out is not None else r
        r = part.sum(0).to(out_dtype)
    if out is not None:
        if accumulate:
            out.view(co, ci).add_(r)
        else:
            out.view(co, ci).copy_(r)
        return out
    return r


# Stride-1 1x1 convs on the own MFMA implicit-GEMM kernel (conv_tap_k, kFwd1) where
# it measured faster than hipBLASLt (tools/microbench.py conv1x1-own,
# profiles/microbench_conv1x1_own.txt; bit-identical results): the channel-
# reducing ResNet-50 shapes 256->64 @ 56x56 (97 vs 156 us) and 512->128 @ 28x28
# (50 vs 61 us), and 512->2048 @ 7x7 (46 vs 53 us).  A data gradient is the same
# 1x1 conv of dY with the transposed weight, so conv3's dgrads (256->64, 512->128)
# take it too.  (cin, cout) -> minimum rows M = N*H*W.
_OWN1X1 = {(256, 64): 200_000, (512, 128): 100_000, (512, 2048): 0}
_USE_OWN1X1 = True


def _own_1x1(x_rows_dtype, cin, cout, m):
    lim = _OWN1X1.get((cin, cout))
    return (_USE_OWN1X1 and lim is not None and m >= lim and m < (1 << 31)
            and x_rows_dtype == torch.bfloat16 and _native.available())


def _g4w_1x1(x, ci, co, m):
    """The native 1x1 forward runs this shape on gemm4w (csrc/hip/conv_igemm.hip
    conv1x1_g4w: the measured winners, with the statistics epilogue)."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and _native.available() and ci % 64 == 0
            and _native.require().conv.on_gemm4w_1x1(m, ci, co))


# Channel-reducing 1x1 forwards consumed by a BatchNorm that run on the own kernel with the
# statistics epilogue although hipBLASLt alone is faster: the saved statistics pass + its
# finalize outweigh it (round 6, tools/diag/own1x1_route.py vs the tuned library times of
# the serialized model profile, profiles/r6/route1x1/): 256 -> 128 @ 56 151 vs 144 + 63 + 7
# us, 512 -> 256 @ 28 103 vs 83 + 32 + 7, 1024 -> 256 @ 14 43 vs 32 + 11 + 6, 2048 -> 512
# @ 7 44 vs 38 + 6 + 8; 1024 -> 512 @ 14 stays on the library (77 vs 39 + 6 + 8).
_OWN1X1_BN = {(256, 128), (512, 256), (1024, 256), (2048, 512)}


def _conv1x1_fwd(x, weight, bn=None):
    """y = conv1x1(x) for a channels-last bf16 x: own MFMA kernel, gemm4w or hipBLASLt.
    With ``bn`` (a BatchNorm consuming y) the native kernel also writes its statistics
    wherever that beats hipBLASLt + a statistics pass (always for own-kernel and gemm4w
    shapes; channel-expanding / equal shapes, where the saved pass over the 4x larger
    output outweighs the library's edge: profiles/microbench_conv1x1_own.txt)."""
    n, ci, h, w = x.shape
    co = weight.shape[0]
    own = _own_1x1(x.dtype, ci, co, n * h * w) or _g4w_1x1(x, ci, co, n * h * w)
    if (bn is not None and weight.dtype == torch.bfloat16 and ci % 64 == 0 and co % 64 == 0
            and (own or co >= ci or (_USE_OWN1X1 and (ci, co) in _OWN1X1_BN))
            and n * h * w < (1 << 31)):
        return _conv_fwd(x, weight, 1, bn)
    if own and weight.dtype == torch.bfloat16:
        return _native.require().conv.conv_fwd(x, weight, 1)
    y2 = torch.mm(_as_rows(x), weight.reshape(co, ci).t())
    return y2.view(n, h, w, co).permute(0, 3, 1, 2)


def _transpose_1x1(weight):
    """W^T as a [Cin, Cout, 1, 1] filter: one LDS-tiled transpose kernel for 16-bit
    weights (ATen's strided copy took ~17 us per ResNet-50 weight, 14 per step)."""
    co, ci = weight.shape[0], weight.shape[1]
    if weight.is_cuda and weight.element_size() == 2 and _native.available():
        got = _prepared(weight)
        if got is not None:
            return got
        return _native.require().conv.transpose_weight(weight)
    return weight.reshape(co, ci).t().contiguous().view(ci, co, 1, 1)


def _conv1x1_dgrad(dy, weight, xshape):
    """dX = dY @ W (a 1x1 conv of dY with W^T)."""
    n, ci, h, w = xshape
    co = weight.shape[0]
    if _own_1x1(dy.dtype, co, ci, n * h * w) and weight.dtype == torch.bfloat16:
        return _native.require().conv.conv_fwd(dy, _transpose_1x1(weight), 1)
    dx2 = torch.mm(_as_rows(dy), weight.reshape(co, ci))
    return dx2.view(n, h, w, ci).permute(0, 3, 1, 2)


def _as_rows(t):
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


# ---------------------------------------------------------------- BN statistics in the
# conv epilogue.  A conv whose output feeds a training-mode BatchNorm (the model links
# them: ``conv._amd_stats_bn``) asks the own MFMA kernel to also write that BN's
# per-M-tile shifted sums (csrc/hip/conv_igemm.hip); the BN then finalizes from that
# slab (bn.slab_train_stats / slab_packed_stats) instead of re-reading its input with a
# statistics pass.  The slab travels to the BN as an attribute of the conv output,
# tagged with the BN module it was made for.  APEX_AMD_CONV_BN_STATS=0 disables.
_CONV_BN_STATS = os.environ.get("APEX_AMD_CONV_BN_STATS", "1") == "1"
_TLS = threading.local()


def _stats_bn(conv, x):
    """The BatchNorm module that will consume ``conv(x)`` if it can take epilogue
    statistics (training mode, running-stat shift available or not), else None."""
    if not (_CONV_BN_STATS and x.is_cuda and x.dtype == torch.bfloat16):
        return None
    link = getattr(conv, "_amd_stats_bn", None)
    owner = link() if link is not None else None
    bn = getattr(owner, "bn", None) if owner is not None else None
    if bn is None or not bn.training or not hasattr(bn, "_amd_accepts_slab"):
        return None
    if not bn._amd_accepts_slab():
        return None
    return bn


def _shift_of(bn):
    rm = bn.running_mean if bn.track_running_stats else None
    if rm is not None and rm.dtype == torch.float32 and rm.is_contiguous():
        return rm
    return None


def _conv_fwd(x, weight, stride, bn):
    """Own-kernel conv forward; with ``bn`` also the stats slab (thread-local hand-off
    to the module, which tags the output)."""
    cv = _native.require().conv
    if bn is None:
        return cv.conv_fwd(x, weight, stride)
    shift = _shift_of(bn)
    y, slab = cv.conv_fwd_stats(x, weight, stride, shift)
    _TLS.slab = (slab, shift, bn)
    return y


def _tag_stats(y):
    ent = getattr(_TLS, "slab", None)
    if ent is not None:
        _TLS.slab = None
        y._amd_bn_stats = ent
    return y


# ---------------------------------------------------------------- BN backward in the
# data-gradient epilogue.  A conv whose input is a fused BN's output (the BN tagged it
# with a BnBwdSrc, ops/batch_norm.py) computes its stride-1 data gradient on the own
# MFMA kernel with the ConvBnEpi epilogue (csrc/hip/conv_igemm.hip): it stores
# g = relu_mask * (dY W^T [+ the residual gradient]) and that BN's per-tile sums, and the
# BN's backward then runs only its elementwise pass.  APEX_AMD_CONV_BN_BWD=0 disables
# (ops/batch_norm.py).


# Where the epilogue pays (tools/microbench.py conv-bnbwd, profiles/microbench_conv_bnbwd.txt,
# one MI355X): with a residual gradient to add (the bottleneck's conv1 dgrad feeding the
# previous block's bn3) it replaces the hipBLASLt addmm + reduce pass + dz store and wins
# 10-260 us per layer; without one (bn1 / bn2) the extra read of the BN input in the
# epilogue costs more than the reduce pass it saves except on small layers (7x7: M =
# 12544), so those fuse only below 65,536 output pixels.  Round 4
# (32-deep K ring): 65536 takes the 14x14 layers (M = 50176) in too - ResNet-50 same box,
# two runs each: 10,582 / 10,576 img/s at 16384, 10,595 / 10,633 with the 14x14 layers,
# 10,613 / 10,549 with every layer (profiles/r4/i/).  Round 6 (halo / C^T / N-fastest
# kernels, the epilogue's early prefetch): every layer wins - 12,640 / 12,727 vs 12,581 /
# 12,656 img/s with the 65,536 cap (profiles/r6/bnbwd_all/), so no cap by default.
_BNBWD_MAX_M = int(os.environ.get("APEX_AMD_BNBWD_MAX_M", str((1 << 31) - 1)))
# the stride-2 3x3 data gradients (conv_dgrad_s2) with the same epilogue (A/B switch):
# correct (tests/test_conv_bn_bwd_gpu.py::test_dgrad_s2_bnbwd_epilogue) but neutral end to
# end - 12,593 / 12,625 vs 12,605 / 12,599 img/s same box (profiles/r6/bnbwd_s2/) - so off
_BNBWD_S2 = os.environ.get("APEX_AMD_BNBWD_S2", "0") == "1"


def _bnbwd_ok(dy, weight, src, xshape, has_add=False):
    m = xshape[0] * xshape[2] * xshape[3]
    return (src is not None and dy.is_cuda and dy.dtype == torch.bfloat16
            and weight.dtype == torch.bfloat16 and tuple(src.x.shape) == tuple(xshape)
            and dy.size(1) % 64 == 0 and xshape[1] % 64 == 0 and m < (1 << 31)
            and (has_add or m <= _BNBWD_MAX_M) and _native.available())


def _dgrad_bn(dy, wprep, add, src, add_stride2=False):
    """g = mask * (conv(dy, wprep) + add) with the BN sums; hands them to the BN.
    ``add_stride2``: ``add`` is the COMPACT [N, C, H/2, W/2] gradient of a stride-2 1x1
    conv over the same input, landing on the even pixels only."""
    g, slab = _native.require().conv.conv_fwd_bnbwd(
        dy, wprep, add, src.x, src.mask, src.mean, src.invstd, src.weight, src.bias,
        src.relu_mode, add_stride2)
    src.result = (g.data_ptr(), slab, g._version)
    return g


class Conv1x1GemmFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bn=None, src=None):
        ctx.save_for_backward(x, weight)
        ctx.src = src
        if ctx.needs_input_grad[1]:
            _ddp_direct.note_use(weight)
        n, ci, h, w = x.shape
        if ctx.needs_input_grad[0] and weight.dtype == torch.bfloat16 and (
                src is not None or _own_1x1(x.dtype, weight.shape[0], ci, n * h * w)):
            _register_prep(weight)  # its dgrad runs on the own kernel with W^T
        return _conv1x1_fwd(x, weight, bn)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        side = _SideWgrad(weight) if ctx.needs_input_grad[1] else None
        if ctx.needs_input_grad[0]:
            if _bnbwd_ok(dy, weight, ctx.src, x.shape):
                dx = _dgrad_bn(dy, _transpose_1x1(weight), None, ctx.src)
            else:
                dx = _conv1x1_dgrad(dy, weight, x.shape)
        ctx.src = None
        if ctx.needs_input_grad[1]:
            direct = None if side.on else _ddp_direct.slots(weight)
            tgt, acc = _ddp_direct.grad_target(weight) if direct is not None else (None, True)
            if direct is not None and tgt.is_contiguous():
                # accumulate straight into the DDP bucket view, no autograd add kernel
                wgrad_1x1(_as_rows(dy), _as_rows(x), weight.dtype, out=tgt, accumulate=acc)
                _ddp_direct.mark_ready(direct)
            else:
                so, sa = _side_out(side, weight)
                dw = side.run(lambda: _wgrad_1x1_w(dy, x, weight, so, sa), dy, x)
        return dx, dw, None, None


class Conv1x1SkipFunction(torch.autograd.Function):
    """(y, skip) = (conv1x1(x), x): the 1x1 GEMM convolution that also hands its
    input on as the residual branch of a bottleneck block.  Backward receives
    both gradients and forms dx = dskip + dy @ W as ONE GEMM with beta = 1
    (hipBLASLt accumulates into C), replacing conv-dgrad + a separate
    elementwise add over the block input (the residual-gradient sum autograd
    would otherwise launch)."""

    @staticmethod
    def forward(ctx, x, weight, bn=None, src=None):
        ctx.save_for_backward(x, weight)
        ctx.src = src
        if ctx.needs_input_grad[1]:
            _ddp_direct.note_use(weight)
        if src is not None and ctx.needs_input_grad[0] and weight.dtype == torch.bfloat16:
            _register_prep(weight)
        return _conv1x1_fwd(x, weight, bn), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dskip):
        x, weight = ctx.saved_tensors
        n, ci, h, w = x.shape
        co = weight.shape[0]
        dx = dw = None
        if dy is not None:
            dy = dy.contiguous(memory_format=torch.channels_last)
        side = _SideWgrad(weight) if (ctx.needs_input_grad[1] and dy is not None) else None
        src, ctx.src = ctx.src, None
        if ctx.needs_input_grad[0]:
            if dy is None:
                dx = dskip
            elif _bnbwd_ok(dy, weight, src, x.shape, has_add=dskip is not None) and (
                    dskip is None or (dskip.dtype == torch.bfloat16 and dskip.shape == x.shape)):
                # dx = mask * (dskip + dy W^T) with the producing BN's sums (its residual
                # gradient dz is this same tensor)
                add = (dskip.contiguous(memory_format=torch.channels_last)
                       if dskip is not None else None)
                dx = _dgrad_bn(dy, _transpose_1x1(weight), add, src)
            else:
                w2 = weight.reshape(co, ci)
                if dskip is not None:
                    # accumulate in place into the residual gradient (a fresh buffer
                    # from the BN backward): C += dy @ W, no copy of C first
                    dskip = dskip.contiguous(memory_format=torch.channels_last)
                    dx2 = _as_rows(dskip).addmm_(_as_rows(dy), w2)
                else:
                    dx2 = torch.mm(_as_rows(dy), w2)
                dx = dx2.view(n, h, w, ci).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1] and dy is not None:
            direct = None if side.on else _ddp_direct.slots(weight)
            tgt, acc = _ddp_direct.grad_target(weight) if direct is not None else (None, True)
            if direct is not None and tgt.is_contiguous():
                wgrad_1x1(_as_rows(dy), _as_rows(x), weight.dtype, out=tgt, accumulate=acc)
                _ddp_direct.mark_ready(direct)
            else:
                so, sa = _side_out(side, weight)
                dw = side.run(lambda: _wgrad_1x1_w(dy, x, weight, so, sa), dy, x)
        return dx, dw, None, None


class Conv1x1Stride2Function(torch.autograd.Function):
    """Stride-2 1x1 convolution (the ResNet downsample projection) on the MFMA
    implicit-GEMM kernel: forward reads every other pixel in place (no subsample
    copy), the data gradient is one launch over the 4 input-parity classes (the
    even-even class is the GEMM dY @ W, the other three a zero store), the weight
    gradient is the per-tap split-K kernel with one tap."""

    @staticmethod
    def forward(ctx, x, weight, bn=None):
        ctx.save_for_backward(x, weight)
        if ctx.needs_input_grad[1]:
            _ddp_direct.note_use(weight)
        if ctx.needs_input_grad[0]:
            _register_prep(weight)
        return _conv_fwd(x, weight, 2, bn)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        cv = _native.require().conv
        dy = dy.contiguous(memory_format=torch.channels_last)
        co, ci = weight.shape[0], weight.shape[1]
        dx = dw = None
        side = _SideWgrad(weight) if ctx.needs_input_grad[1] else None
        if ctx.needs_input_grad[0]:
            dx = cv.conv_dgrad_s2(dy, _transpose_1x1(weight), x.size(2), x.size(3))
        if ctx.needs_input_grad[1]:
            direct = None if side.on else _ddp_direct.slots(weight)
            tgt, acc = _ddp_direct.grad_target(weight) if direct is not None else (None, True)
            if direct is not None and tgt.is_contiguous(memory_format=torch.channels_last):
                cv.conv_wgrad(dy, x, weight.dtype, 0, 2, 1, out=tgt, accumulate=acc)
                _ddp_direct.mark_ready(direct)
            else:
                so, sa = _side_out(side, weight, cl=True)
                dw = side.run(lambda: cv.conv_wgrad(dy, x, weight.dtype, 0, 2, 1, out=so,
                                                    accumulate=sa), dy, x)
        return dx, dw, None


# A bottleneck's first block in layers 2-4: the block input feeds conv1 (1x1, stride 1)
# and the stride-2 1x1 downsample projection.  As two Functions, the downsample's input
# gradient is a full-size tensor that is zero on 3 of 4 pixels (its data-gradient kernel
# writes all of them) and conv1's data gradient reads it back as the residual term.  One
# Function for both convs keeps that gradient COMPACT - the plain 1x1 GEMM dY_d W_d on the
# strided pixels - and conv1's dgrad epilogue adds it onto the even pixels only
# (ConvBnEpi.add_s2).
_PAIR_S2 = True
PAIR_S2_CALLS = [0]  # backward passes that took the compact path (tests)


class Conv1x1PairS2Function(torch.autograd.Function):
    """(conv1x1(x, w1), conv1x1_stride2(x, wd)) over one input."""

    @staticmethod
    def forward(ctx, x, w1, wd, bn1=None, bnd=None, src=None):
        ctx.save_for_backward(x, w1, wd)
        ctx.src = src
        for w, k in ((w1, 1), (wd, 2)):
            if ctx.needs_input_grad[k]:
                _ddp_direct.note_use(w)
        if ctx.needs_input_grad[0]:
            _register_prep(w1)
            _register_prep(wd)
        y1 = _conv1x1_fwd(x, w1, bn1)
        ent1 = getattr(_TLS, "slab", None)
        _TLS.slab = None
        yd = _conv_fwd(x, wd, 2, bnd)
        ent2 = getattr(_TLS, "slab", None)
        _TLS.slab = None
        _TLS.pair = (ent1, ent2)
        return y1, yd

    @staticmethod
    def backward(ctx, dy1, dyd):
        x, w1, wd = ctx.saved_tensors
        n, ci, h, w = x.shape
        cv = _native.require().conv
        src, ctx.src = ctx.src, None
        dx = dw1 = dwd = None
        if dy1 is not None:
            dy1 = dy1.contiguous(memory_format=torch.channels_last)
        if dyd is not None:
            dyd = dyd.contiguous(memory_format=torch.channels_last)
        side1 = _SideWgrad(w1) if (ctx.needs_input_grad[1] and dy1 is not None) else None
        sided = _SideWgrad(wd) if (ctx.needs_input_grad[2] and dyd is not None) else None
        if ctx.needs_input_grad[0]:
            # the downsample's input gradient on the strided pixels only: dY_d W_d
            cd = (_conv1x1_dgrad(dyd, wd, (n, ci, h // 2, w // 2)).contiguous(
                memory_format=torch.channels_last) if dyd is not None else None)
            if dy1 is None:
                dx = torch.zeros_like(x)
                if cd is not None:
                    dx[:, :, ::2, ::2] = cd
            elif cd is not None and _bnbwd_ok(dy1, w1, src, x.shape, has_add=True):
                PAIR_S2_CALLS[0] += 1
                dx = _dgrad_bn(dy1, _transpose_1x1(w1), cd, src, add_stride2=True)
            else:
                dx = _conv1x1_dgrad(dy1, w1, x.shape).contiguous(
                    memory_format=torch.channels_last)
                if cd is not None:
                    dx[:, :, ::2, ::2] += cd
        if side1 is not None:
            direct = None if side1.on else _ddp_direct.slots(w1)
            tgt, acc = _ddp_direct.grad_target(w1) if direct is not None else (None, True)
            if direct is not None and tgt.is_contiguous():
                wgrad_1x1(_as_rows(dy1), _as_rows(x), w1.dtype, out=tgt, accumulate=acc)
                _ddp_direct.mark_ready(direct)
            else:
                so, sa = _side_out(side1, w1)
                dw1 = side1.run(lambda: _wgrad_1x1_w(dy1, x, w1, so, sa), dy1, x)
        if sided is not None:
            direct = None if sided.on else _ddp_direct.slots(wd)
            tgt, acc = _ddp_direct.grad_target(wd) if direct is not None else (None, True)
            if direct is not None and tgt.is_contiguous(memory_format=torch.channels_last):
                cv.conv_wgrad(dyd, x, wd.dtype, 0, 2, 1, out=tgt, accumulate=acc)
                _ddp_direct.mark_ready(direct)
            else:
                so, sa = _side_out(sided, wd, cl=True)
                dwd = sided.run(lambda: cv.conv_wgrad(dyd, x, wd.dtype, 0, 2, 1, out=so,
                                                      accumulate=sa), dyd, x)
        return dx, dw1, dwd, None, None, None


def conv1x1_pair_s2(conv1, convd, x):
    """(conv1(x), convd(x)) for a stride-1 ``Conv2d1x1`` and a stride-2 ``Conv2d1x1`` over
    the same input - one Function with a compact downsample gradient where the own
    kernels apply, else the two convs as usual."""
    if (_PAIR_S2 and isinstance(conv1, Conv2d1x1) and isinstance(convd, Conv2d1x1)
            and conv1._gemm_ok(x) and convd._strided_ok(x) and x.dtype == torch.bfloat16
            and conv1.weight.dtype == torch.bfloat16 and _native.available()):
        y1, yd = Conv1x1PairS2Function.apply(x, conv1.weight, convd.weight,
                                             _stats_bn(conv1, x), _stats_bn(convd, x),
                                             bn_src_of(x))
        ent1, ent2 = getattr(_TLS, "pair", (None, None))
        _TLS.pair = (None, None)
        if ent1 is not None:
            y1._amd_bn_stats = ent1
        if ent2 is not None:
            yd._amd_bn_stats = ent2
        return y1, yd
    return conv1(x), convd(x)


class Conv2d1x1(nn.Conv2d):
    """nn.Conv2d(kernel_size=1) whose stride-1 channels-last GPU path runs as a
    GEMM; every other case falls back to the regular convolution."""

    def __init__(self, in_planes, out_planes, stride=1, bias=False):
        super().__init__(in_planes, out_planes, kernel_size=1, stride=stride, bias=bias)

    def forward(self, x):
        if self._gemm_ok(x):
            return _tag_stats(Conv1x1GemmFunction.apply(x, self.weight, _stats_bn(self, x),
                                                        bn_src_of(x)))
        if self._strided_ok(x):
            return _tag_stats(Conv1x1Stride2Function.apply(x, self.weight, _stats_bn(self, x)))
        return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation,
                        self.groups)

    def forward_with_skip(self, x):
        """(conv(x), x) with the residual-gradient add fused into the dgrad GEMM."""
        if self._gemm_ok(x):
            y, skip = Conv1x1SkipFunction.apply(x, self.weight, _stats_bn(self, x),
                                                bn_src_of(x))
            return _tag_stats(y), skip
        return self.forward(x), x

    def _strided_ok(self, x):
        return (self.stride == (2, 2) and self.bias is None and x.is_cuda and x.dim() == 4
                and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16
                and x.is_contiguous(memory_format=torch.channels_last) and self.groups == 1
                and x.size(2) % 2 == 0 and x.size(3) % 2 == 0
                and x.size(0) * x.size(2) * x.size(3) < (1 << 22)
                and self.in_channels % 64 == 0 and self.out_channels % 64 == 0)

    def _gemm_ok(self, x):
        return (self.stride == (1, 1) and self.bias is None and x.is_cuda and x.dim() == 4
                and x.is_contiguous(memory_format=torch.channels_last)
                and x.dtype == self.weight.dtype and self.groups == 1)


# 3x3 weight gradient: "tap" = per-tap MFMA kernel (default), "nine" = the all-taps
# strip kernel (W <= 56), "miopen" = MIOpen's convolution_backward
_WGRAD3 = "tap"
# 3x3 stride-1 weight gradients on the strip-ring kernel (csrc/hip/conv_igemm.hip
# conv3x3_wgrad_c64_k, algo 4: all nine taps per workgroup from one padded-row strip):
# 64 -> 64 (ResNet layer 1, 93.8 us / 631 TF vs 175 us for the per-tap kernel, docs/PERF.md
# round 4); round 6 generalised it to 64 x 64 channel tiles: bs 256, incl. the split
# reduction, 128@28 113 -> 85 us, 256@14 104 -> 93 us; at 7 x 7 every K-tile is a new
# image (a full strip load each), 110 -> 123 us, so W < 14 keeps the per-tap kernel
# (profiles/r6/wgrad9_bench.md).  In the model it measured neutral (ResNet-50 same box
# 11,956 / 11,948 vs 11,982 / 11,906 img/s: the kernel holds a whole CU, 147 KB LDS, so
# the main-stream kernels it overlapped lose residency), so the wider routing is opt-in
# (APEX_AMD_WGRAD9=1); the 64 -> 64 shapes always take it
_WGRAD64 = True
_WGRAD9_ALL = os.environ.get("APEX_AMD_WGRAD9", "0") == "1"


def _wgrad3_algo(x, weight, stride):
    """conv_wgrad algo for a 3x3 weight gradient under _WGRAD3 == "tap"."""
    cin, cout = x.size(1), weight.size(0)
    if not (_WGRAD64 and stride == 1 and x.size(3) <= 56 and cin % 64 == 0
            and cout % 64 == 0):
        return 0
    if cin == 64 and cout == 64:
        return 4
    return 4 if _WGRAD9_ALL and x.size(3) >= 14 else 0
# the own reduction / rotation kernels (tests turn them off to compare with ATen)
_USE_SPLITK_REDUCE = True
_USE_ROT_KERNEL = True


def _rot_weight(weight):
    """W'[ci, co, r, s] = W[co, ci, 2-r, 2-s]: the data gradient of a 3x3 stride-1
    pad-1 conv is the same conv applied to dY with W' (one tiled-transpose kernel)."""
    if _USE_ROT_KERNEL and weight.is_cuda and weight.element_size() == 2:
        got = _prepared(weight)
        if got is not None:
            return got
        return _native.require().conv.rot_weight(weight)
    return weight.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)


# Backward weight layouts (rotated 3x3 filters, transposed 1x1 filters) of every conv
# whose data gradient runs on the own kernels, made in ONE launch per backward pass
# (conv.prep_weights) instead of one ~10 us launch per filter (27 per ResNet-50 step).
# Forward registers the filter; the first backward request prepares every registered
# filter; the next forward of a filter drops its prepared copy (the optimizer may
# have rewritten the weights in place since).
_USE_PREP = True
_PREP_PENDING = {}   # id(weight) -> weight
_PREP_READY = {}     # id(weight) -> (weight, prepared layout)


def _register_prep(weight):
    if not (_USE_PREP and weight.is_cuda and weight.element_size() == 2):
        return
    k = id(weight)
    _PREP_READY.pop(k, None)
    _PREP_PENDING[k] = weight


def _prepared(weight):
    k = id(weight)
    ent = _PREP_READY.get(k)
    if ent is not None and ent[0] is weight:
        return ent[1]
    if k not in _PREP_PENDING:
        return None
    ws = list(_PREP_PENDING.values())
    _PREP_PENDING.clear()
    _PREP_READY.clear()  # only the latest batch is kept (bounded memory)
    outs = _native.require().conv.prep_weights(ws)
    for w, o in zip(ws, outs):
        _PREP_READY[id(w)] = (w, o)
    return _PREP_READY[k][1]


class Conv3x3Function(torch.autograd.Function):
    """3x3 / pad 1 / stride 1 or 2 NHWC bf16 conv on the MFMA implicit-GEMM
    kernels (csrc/hip/conv_igemm.hip): forward, data gradient (stride 1: the same
    kernel with rotated weights; stride 2: one launch over the 4 input-parity
    classes, each with only its matching filter taps) and weight gradient
    (per-tap split-K kernel)."""

    @staticmethod
    def forward(ctx, x, weight, stride, bn=None, src=None):
        ctx.save_for_backward(x, weight)
        ctx.stride = stride
        ctx.src = src if stride == 1 else None
        if ctx.needs_input_grad[1]:
            _ddp_direct.note_use(weight)
        if ctx.needs_input_grad[0] and _USE_ROT_KERNEL:
            _register_prep(weight)
        return _conv_fwd(x, weight, stride, bn)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride = ctx.stride
        cv = _native.require().conv
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        n_pix = x.size(0) * x.size(2) * x.size(3)
        own_wgrad = n_pix < (1 << 22) and (
            _WGRAD3 == "tap" or (_WGRAD3 == "nine" and stride == 1 and x.size(3) <= 56))
        side = _SideWgrad(weight) if (ctx.needs_input_grad[1] and own_wgrad) else None
        src, ctx.src = ctx.src, None
        if ctx.needs_input_grad[0]:
            if stride == 1 and _bnbwd_ok(dy, weight, src, x.shape):
                dx = _dgrad_bn(dy, _rot_weight(weight), None, src)
            elif stride == 1:
                dx = cv.conv_fwd(dy, _rot_weight(weight), 1)
            elif _BNBWD_S2 and _bnbwd_ok(dy, weight, src, x.shape):
                # stride-2 3x3 dgrad with the BN-backward epilogue (no reduction pass for
                # the BN whose output this conv read)
                dx, slab = cv.conv_dgrad_s2_bnbwd(
                    dy, _rot_weight(weight), x.size(2), x.size(3), src.x, src.mask, src.mean,
                    src.invstd, src.weight, src.bias, src.relu_mode)
                src.result = (dx.data_ptr(), slab, dx._version)
            else:
                dx = cv.conv_dgrad_s2(dy, _rot_weight(weight), x.size(2), x.size(3))
        direct = None
        if ctx.needs_input_grad[1] and own_wgrad and not side.on:
            direct = _ddp_direct.slots(weight)
            if direct is not None:
                tgt, acc = _ddp_direct.grad_target(weight)
                if not tgt.is_contiguous(memory_format=torch.channels_last):
                    direct = None
        if direct is not None:
            # accumulate straight into the DDP bucket view, no autograd add kernel
            cv.conv_wgrad(dy, x, weight.dtype,
                          _wgrad3_algo(x, weight, stride) if _WGRAD3 == "tap" else 1,
                          stride if _WGRAD3 == "tap" else 1, out=tgt, accumulate=acc)
            _ddp_direct.mark_ready(direct)
        elif ctx.needs_input_grad[1]:
            so, sa = _side_out(side, weight, cl=True)
            if _WGRAD3 == "tap" and n_pix < (1 << 22):
                algo = _wgrad3_algo(x, weight, stride)
                dw = side.run(lambda: cv.conv_wgrad(dy, x, weight.dtype, algo, stride, out=so,
                                                    accumulate=sa), dy, x)
            elif _WGRAD3 == "nine" and stride == 1 and x.size(3) <= 56 and n_pix < (1 << 22):
                dw = side.run(lambda: cv.conv_wgrad(dy, x, weight.dtype, 1, 1, out=so,
                                                    accumulate=sa), dy, x)
            else:
                dw = torch.ops.aten.convolution_backward(
                    dy, x, weight, None, (stride, stride), (1, 1), (1, 1), False, (0, 0), 1,
                    (False, True, False))[1]
        return dx, dw, None, None, None


class Conv2d3x3(nn.Conv2d):
    """nn.Conv2d(k=3, padding=1) whose stride-1 channels-last bf16 GPU path runs
    the MFMA implicit-GEMM kernel; everything else uses the regular conv."""

    def __init__(self, in_planes, out_planes, stride=1, bias=False):
        super().__init__(in_planes, out_planes, kernel_size=3, stride=stride, padding=1,
                         bias=bias)

    def forward(self, x):
        st = self.stride[0]
        if (self.stride in ((1, 1), (2, 2)) and self.bias is None and x.is_cuda and x.dim() == 4
                and (st == 1 or (x.size(2) % 2 == 0 and x.size(3) % 2 == 0))
                and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16
                and x.is_contiguous(memory_format=torch.channels_last) and self.groups == 1
                and self.in_channels % 64 == 0 and self.out_channels % 64 == 0
                and self.dilation == (1, 1) and self.padding == (1, 1)):
            return _tag_stats(Conv3x3Function.apply(x, self.weight, st, _stats_bn(self, x),
                                                    bn_src_of(x)))
        return F.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation,
                        self.groups)


def _pack_stem_weight(weight):
    """[64, 3, 7, 7] -> [64, 7 (r), 32 (4 s + c)] bf16, zeros at c = 3 and s = 7."""
    wk = torch.zeros(64, 7, 8, 4, device=weight.device, dtype=torch.bfloat16)
    wk[:, :, :7, :3] = weight.permute(0, 2, 3, 1)
    return wk.view(64, 224)


class StemConvFunction(torch.autograd.Function):
    """ResNet stem 7x7/2 conv (3 -> 64 channels) on the gfx950 stem kernels
    (csrc/hip/stem_conv.hip): the image is zero-padded once to 4 channels, a wave
    computes whole output rows from an LDS ring of input rows; the weight
    gradient reads the same padded image.  The image gradient (not needed for
    training from data) falls back to MIOpen."""

    @staticmethod
    def forward(ctx, x, weight, bn=None):
        cv = _native.require().conv
        xp = cv.stem_pad(x)
        ctx.save_for_backward(x, xp, weight)
        if bn is None:
            return cv.stem_fwd(xp, _pack_stem_weight(weight))
        # the stem BN's statistics from the kernel's epilogue (handed to the module, which
        # tags the output; ops/pool.py bn_relu_maxpool or the BN consume it)
        shift = _shift_of(bn)
        y, slab = cv.stem_fwd_stats(xp, _pack_stem_weight(weight), shift)
        _TLS.slab = (slab, shift, bn)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, xp, weight = ctx.saved_tensors
        dx = dw = None
        if ctx.needs_input_grad[1]:
            part = _native.require().conv.stem_wgrad(xp, dy)  # [64, 256] fp32
            dw = part.view(64, 8, 8, 4)[:, :7, :7, :3].permute(0, 3, 1, 2).to(weight.dtype)
            dw = dw.contiguous(memory_format=torch.channels_last) \
                if weight.is_contiguous(memory_format=torch.channels_last) else dw.contiguous()
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(
                dy, x, weight, None, (2, 2), (3, 3), (1, 1), False, (0, 0), 1,
                (True, False, False))[0]
        return dx, dw, None


class StemConv2d(nn.Conv2d):
    """nn.Conv2d(3, 64, 7, stride=2, padding=3) whose bf16 GPU path runs the MFMA
    stem kernels; other dtypes / sizes use the regular convolution."""

    def __init__(self, in_planes=3, out_planes=64):
        super().__init__(in_planes, out_planes, kernel_size=7, stride=2, padding=3, bias=False)

    def forward(self, x):
        if (x.is_cuda and x.dim() == 4 and x.size(1) == 3 and self.out_channels == 64
                and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16
                and x.size(2) % 2 == 0 and x.size(3) % 2 == 0 and x.size(3) <= 250
                and self.in_channels == 3):
            return _tag_stats(StemConvFunction.apply(x, self.weight, _stats_bn(self, x)))
        return F.conv2d(x, self.weight, None, self.stride, self.padding)
