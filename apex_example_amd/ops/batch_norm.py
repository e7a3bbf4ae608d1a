"""Fused BatchNorm(+residual)(+ReLU) autograd op on the gfx950 kernels
(csrc/hip/batch_norm.hip), shared by ``SyncBatchNorm`` and the local
``BatchNorm2dReLU`` used by the MI355X ResNet.

Forward (training): split-reduction per-channel stats -> [one packed all_gather
of (mean, var, count) across the process group] -> combine + running-stat
update -> y = relu(x*scale + shift + z) in one elementwise pass.
Backward: one reduction pass (sum dy', sum dy'*(x-mean), dgamma, dbeta) ->
[one packed all_reduce of the two sums] -> one elementwise pass producing dx
(and dz for the residual branch).  The ReLU condition is recomputed from x when
there is no residual; with a residual z (relu(bn(x) + z), every bottleneck's
last BN) the forward writes a 1-bit-per-element ReLU mask instead, so backward
reads 1/16 of z's bytes (twice) and z is not kept alive.

Works for any memory format: NCHW-contiguous runs the NCHW kernels,
channels_last-contiguous 4-D tensors run the NHWC kernels; ``shape_channel_last``
selects apex's channel_last=True convention (C is the LAST dimension of the
shape).
"""
from __future__ import annotations

import os
import threading

import torch
import torch.distributed as dist

from .. import _native
from . import _ddp_direct

# BN backward folded into the consuming conv's data-gradient epilogue (BnBwdSrc below);
# APEX_AMD_CONV_BN_BWD=0 keeps the separate reduction pass
_BWD_EPI = os.environ.get("APEX_AMD_CONV_BN_BWD", "1") == "1"
_TLS = threading.local()
FUSED_BWD_CALLS = [0]  # BN backwards that took the epilogue sums (diagnostics / tests)

# the residual BN's backward sums formed in the consuming BN's elementwise pass
# (bn.backward_elemt_x2; A/B switch), and a count of the BN backwards that used them
_X2_BWD = os.environ.get("APEX_AMD_BN_X2", "1") == "1"
X2_BWD_CALLS = [0]


def _x2_target_ok(zc, ctx, weight):
    """zc (the residual BN's autograd node) can take its sums from ctx's elementwise pass:
    a local, ReLU-free, residual-free BN over the same rows, weights of one dtype."""
    return (getattr(zc, "world", 0) == 1 and not getattr(zc, "fuse_relu", True)
            and not getattr(zc, "has_z", True) and getattr(zc, "count", -1) == ctx.count
            and not getattr(zc, "shape_channel_last", True) and not ctx.shape_channel_last
            and (zc.saved_tensors[2] is None) == (weight is None)
            and (weight is None or zc.saved_tensors[2].dtype == weight.dtype)
            and zc.saved_tensors[6] is None)


class BnBwdSrc:
    """What a stride-1 data-gradient conv that consumes this BN's output needs to do the
    BN's backward reduction in its epilogue (ops/conv.py, csrc/hip/conv_igemm.hip
    ConvBnEpi): the BN input x, the batch mean / invstd, the affine parameters and how
    to rebuild the ReLU mask (0 none, 1 the forward's bitmask, 2 recompute from x).
    The conv stores g = mask * dL/dy instead of dL/dy and leaves (g's address, the
    per-tile sums slab) in ``result``; this BN's backward then skips its reduction
    pass - and, with a residual, its dz store (dz is g).  The output tensor carries
    the record as ``_amd_bn_src``."""
    __slots__ = ("x", "mean", "invstd", "weight", "bias", "mask", "relu_mode", "result")

    def __init__(self, x, mean, invstd, weight, bias, mask, relu_mode):
        self.x, self.mean, self.invstd = x, mean, invstd
        self.weight, self.bias, self.mask, self.relu_mode = weight, bias, mask, relu_mode
        self.result = None


def _bwd_src(x, xl, mean, invstd, weight, bias, mask, fuse_relu, has_z):
    if not (_BWD_EPI and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and x is xl and x.size(1) % 64 == 0
            and x.is_contiguous(memory_format=torch.channels_last)):
        return None
    if fuse_relu and has_z:
        if mask is None:
            return None
        mode = 1
    elif fuse_relu:
        if any(t is not None and t.dtype != torch.float32 for t in (weight, bias)):
            return None
        mode = 2
    else:
        mode = 0
    return BnBwdSrc(x, mean, invstd, weight, bias, mask, mode)


# SyncBN collectives on the compute stream through the dedicated SyncBN group's RCCL
# communicator (csrc/torch/reducer.cpp syncbn_*_raw); APEX_AMD_SYNCBN_RAW_RCCL=0 keeps the
# process group's own stream (c10d calls from C++).
#
# Failure detection: the raw calls are invisible to ProcessGroupNCCL's work tracking, so
# its watchdog never times out a SyncBN collective itself.  A dead or diverged peer is
# still caught: the raw collective stalls the COMPUTE stream (the host does not block on
# it), the host goes on to enqueue the step's DDP bucket collectives - c10d works on the
# DDP communicator, stream-ordered behind the stalled compute stream - and those time out
# after the process group's timeout (bench.py --pg-timeout, 300 s) and the watchdog aborts
# the process (TORCH_NCCL_ASYNC_ERROR_HANDLING).  Without DDP in the step (SyncBN alone),
# set APEX_AMD_SYNCBN_RAW_RCCL=0 to keep every collective under the watchdog.
#
# Two communicators in flight (SyncBN on the compute stream, DDP buckets on their own
# high-priority stream) cannot deadlock each other: each communicator's collectives are
# issued in the same order on every rank (SyncBN: layer order of one program; DDP: the
# rank-0-synchronised bucket order), the two never wait on each other's kernels, and an
# RCCL collective occupies one workgroup per channel (<= RCCL's channel count, see
# bench.py --rccl-channels), so both kernels fit on the 256 CUs at once whatever their
# relative order on a rank; the compute kernels around them are finite, never spinning.
_RAW_RCCL = os.environ.get("APEX_AMD_SYNCBN_RAW_RCCL", "1") == "1"
_COMMS = {}


def _raw_comm(pg):
    """The RCCL communicator pointer of ``pg`` when the raw path may drive it, else 0."""
    return _raw_comm_rank(pg)[0]


def _raw_comm_rank(pg):
    """(communicator pointer or 0, this process's rank in ``pg``)."""
    if not _RAW_RCCL:
        return 0, -1
    c = _COMMS.get(id(pg))
    if c is not None and c[0] is pg:
        return c[1], c[2]
    from ..parallel.sync_batchnorm import is_syncbn_comm_group

    ptr = 0
    if is_syncbn_comm_group(pg) and _native.require().reducer.syncbn_raw_available():
        try:
            ptr = int(pg._get_backend(torch.device("cuda"))._comm_ptr())
        except Exception:  # not an RCCL group / older torch
            ptr = 0
    rank = dist.get_rank(pg)
    if ptr:  # (the communicator exists after the group's first c10d collective)
        _COMMS[id(pg)] = (pg, ptr, rank)
    return ptr, rank


# SyncBN collective timing (bench.py's timing steps at N > 1 / --force-collectives): HIP
# events on the compute stream around every SyncBN collective, so the record shows what
# the 2 latency-bound collectives per BN layer cost the step (including waiting for the
# slowest peer).  None = off; else a list of (kind, start event, end event).
_SBN_EVENTS = None


def syncbn_timing(on=True):
    """Start (clear) or stop recording SyncBN collective timing events."""
    global _SBN_EVENTS
    _SBN_EVENTS = [] if on else None


def syncbn_timing_result():
    """{"calls", "ms", "allgather_ms", "allreduce_ms"} summed over the recorded
    collectives (synchronizes on the last event); None if nothing was recorded."""
    ev = _SBN_EVENTS
    if not ev:
        return None
    ev[-1][2].synchronize()
    out = {"calls": len(ev), "ms": 0.0, "allgather_ms": 0.0, "allreduce_ms": 0.0}
    for kind, a, b in ev:
        ms = a.elapsed_time(b)
        out["ms"] += ms
        out[kind + "_ms"] += ms
    return out


class _SbnTimer:
    def __init__(self, kind):
        self.kind = kind

    def __enter__(self):
        if _SBN_EVENTS is not None:
            self.a = torch.cuda.Event(enable_timing=True)
            self.a.record()
        return self

    def __exit__(self, *exc):
        if _SBN_EVENTS is not None and hasattr(self, "a"):
            b = torch.cuda.Event(enable_timing=True)
            b.record()
            _SBN_EVENTS.append((self.kind, self.a, b))
        return False


def _allreduce(t, pg):
    """In-place SUM all-reduce of a SyncBN packed buffer."""
    if t.is_cuda and _SBN_EVENTS is not None:
        with _SbnTimer("allreduce"):
            return _allreduce_body(t, pg)
    return _allreduce_body(t, pg)


def _allreduce_body(t, pg):
    if dist.get_backend(pg) == "nccl":
        comm = _raw_comm(pg)
        if comm:
            _native.require().reducer.syncbn_allreduce_raw(t, comm)
        else:
            _native.require().reducer.syncbn_allreduce(t, pg)
    else:
        dist.all_reduce(t, group=pg)


# calls that gathered SyncBN statistics through a rank slot of the gather buffer
# (tests/test_ddp_gpu.py checks the rank > 0 slot arithmetic ran)
SLOT_GATHER_CALLS = [0]


def _gather_slot(C, world, rank, device):
    """The [world * (2C + 1)] gather destination and this rank's [2C + 1] slot of it
    (mean | var | count, the layout of local_stats_packed / slab_packed_stats)."""
    n = 2 * C + 1
    assert 0 <= rank < world, (rank, world)
    gathered = torch.empty(world * n, dtype=torch.float32, device=device)
    SLOT_GATHER_CALLS[0] += 1
    return gathered, gathered[rank * n:(rank + 1) * n]


def _direct_targets(params, need_w):
    """(slots, dgamma target, dbeta target, accumulate) of the DDP direct path for a BN's
    affine pair, or (None, None, None, True): both targets must be bucket views in the
    same state (accumulated or lazily zeroed)."""
    direct = _ddp_direct.slots(*params) if need_w else None
    if direct is None:
        return None, None, None, True
    tw, aw = _ddp_direct.grad_target(params[0])
    tb, ab = _ddp_direct.grad_target(params[1])
    if aw != ab:
        return None, None, None, True
    return direct, tw, tb, aw


def bn_src_of(x):
    """The BnBwdSrc of ``x`` when x is a fused BN's output (else None)."""
    return getattr(x, "_amd_bn_src", None)


def _C():
    # (grid sizing of the NHWC kernels: bn.set_tuning, used by tools/microbench.py bn-tune)
    return _native.require().bn


def _to_logical(x, shape_channel_last):
    if shape_channel_last:
        C = x.size(-1)
        return x.reshape(-1, C)
    return x


class BatchNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, z, weight, bias, running_mean, running_var, eps, momentum, process_group,
                fuse_relu, shape_channel_last, num_batches_tracked=None, force_collectives=False,
                slab=None, slab_shift=None):
        C = _C()
        ctx.params = (weight, bias)   # the Parameter objects (DDP bucket slots live on them)
        if ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            _ddp_direct.note_use(weight, bias)
        orig_shape = x.shape
        xl = _to_logical(x, shape_channel_last)
        zl = _to_logical(z, shape_channel_last) if z is not None else None
        count = xl.numel() // xl.size(1)
        if process_group is False or not (dist.is_available() and dist.is_initialized()):
            world = 1  # local statistics
            force_collectives = False
        else:
            world = dist.get_world_size(process_group)
        # force_collectives: take the cross-rank path (packed all_gather / all_reduce)
        # even on a 1-rank group - the test / bench hook that runs SyncBN's RCCL code
        # on a single GPU (DistributedDataParallel has the same switch)
        collective = world > 1 or bool(force_collectives)
        want_mask = bool(fuse_relu) and zl is not None and xl.is_cuda
        if not collective and xl.is_cuda:
            if slab is not None:
                # statistics already summed by the producing conv's epilogue
                # (ops/conv.py): one finalize launch + the apply launch
                mean_g, invstd = C.slab_train_stats(slab, count, slab_shift, running_mean,
                                                    running_var, num_batches_tracked,
                                                    float(eps), float(momentum))
                if want_mask:
                    y, mask = C.apply_mask(xl, mean_g, invstd, weight, bias, zl, bool(fuse_relu))
                else:
                    y, mask = C.apply(xl, mean_g, invstd, weight, bias, zl, bool(fuse_relu)), None
            else:
                # one stats launch + one finalize (mean, invstd, running stats and
                # num_batches_tracked in the same kernel) + one apply launch
                y, mean_g, invstd, mask = C.forward_local(xl, weight, bias, running_mean,
                                                          running_var, num_batches_tracked,
                                                          float(eps), float(momentum), zl,
                                                          bool(fuse_relu), want_mask)
            ctx.save_for_backward(xl, zl if mask is None else None, weight, bias, mean_g, invstd,
                                  mask)
            ctx.src = _TLS.src = _bwd_src(x, xl, mean_g, invstd, weight, bias, mask,
                                          bool(fuse_relu), zl is not None)
            ctx.pg, ctx.world, ctx.fuse_relu, ctx.total, ctx.count = None, 1, bool(fuse_relu), \
                None, count
            # a residual input produced by another local BN (ResNet's downsample BN): this
            # BN's backward may form that BN's sums in its own elementwise pass (_X2_BWD)
            zg = getattr(z, "grad_fn", None) if z is not None else None
            ctx.zctx = zg if isinstance(zg, BatchNormFunction._backward_cls) else None
            ctx.pre = None
            ctx.orig_shape, ctx.has_z, ctx.shape_channel_last = orig_shape, z is not None, \
                shape_channel_last
            return y.view(orig_shape) if shape_channel_last else y
        if collective and xl.is_cuda:
            # SyncBN: the stats kernels write [mean | var | count] into one buffer -> ONE
            # all_gather -> one combine kernel (global mean / invstd, running stats,
            # num_batches_tracked, 1/global count) -> apply.  No host sync, no cat.
            pg = process_group if process_group is not None else dist.group.WORLD
            nccl = dist.get_backend(pg) == "nccl"
            comm, rank = _raw_comm_rank(pg) if nccl else (0, dist.get_rank(pg))
            gathered = slot = None
            if comm or not nccl:
                # the stats kernels write straight into this rank's slot of the gather
                # destination: the RCCL all_gather runs in place (no send-buffer copy).
                # gloo (the multi-process GPU tests) takes the same slot arithmetic.
                gathered, slot = _gather_slot(xl.size(1), world, rank, x.device)
            packed = (C.slab_packed_stats(slab, count, slab_shift, out=slot) if slab is not None
                      else C.local_stats_packed(xl, out=slot))
            if nccl:
                # all_gather + combine in one C++ call (csrc/torch/reducer.cpp): the Python
                # c10d wrapper cost ~20 us of host time per layer; on the compute stream
                # through the group's communicator when it is the dedicated SyncBN group
                R = _native.require().reducer
                with _SbnTimer("allgather"):
                    if comm:
                        mean_g, invstd, inv_total = R.syncbn_allgather_combine_raw(
                            packed, comm, world, float(eps), float(momentum), running_mean,
                            running_var, num_batches_tracked, gathered=gathered, rank=rank)
                    else:
                        mean_g, invstd, inv_total = R.syncbn_allgather_combine(
                            packed, pg, float(eps), float(momentum), running_mean,
                            running_var, num_batches_tracked)
            else:  # gloo with GPU tensors (tests): list form into views of `gathered`
                # (send a copy: gloo does not take a send buffer inside the output)
                with _SbnTimer("allgather"):
                    dist.all_gather(list(gathered.chunk(world)), packed.clone(), group=pg)
                mean_g, invstd, inv_total = C.combine_stats_sync(
                    gathered.view(world, -1), float(eps), float(momentum), running_mean,
                    running_var, num_batches_tracked)
            if want_mask:
                y, mask = C.apply_mask(xl, mean_g, invstd, weight, bias, zl, bool(fuse_relu))
            else:
                y, mask = C.apply(xl, mean_g, invstd, weight, bias, zl, bool(fuse_relu)), None
            ctx.save_for_backward(xl, zl if mask is None else None, weight, bias, mean_g, invstd,
                                  mask)
            ctx.src = _TLS.src = _bwd_src(x, xl, mean_g, invstd, weight, bias, mask,
                                          bool(fuse_relu), zl is not None)
            ctx.pg, ctx.world, ctx.fuse_relu, ctx.total, ctx.count = pg, max(world, 2), \
                bool(fuse_relu), inv_total, count
            ctx.orig_shape, ctx.has_z, ctx.shape_channel_last = orig_shape, z is not None, \
                shape_channel_last
            return y.view(orig_shape) if shape_channel_last else y
        if num_batches_tracked is not None:
            num_batches_tracked.add_(1)
        mean, var = C.local_stats(xl)
        if collective:
            pg = process_group if process_group is not None else dist.group.WORLD
            cnt = torch.full((1,), float(count), dtype=torch.float32, device=x.device)
            packed = torch.cat([mean, var, cnt])
            gathered = torch.empty(world * packed.numel(), dtype=packed.dtype, device=x.device)
            dist.all_gather_into_tensor(gathered, packed, group=pg)
            g = gathered.view(world, -1)
            Cn = mean.numel()
            means, vars_, counts = g[:, :Cn], g[:, Cn:2 * Cn], g[:, 2 * Cn]
            total = counts.sum()
        else:
            pg = None
            means, vars_ = mean.view(1, -1), var.view(1, -1)
            counts = torch.full((1,), float(count), dtype=torch.float32, device=x.device)
            total = None
        mean_g, invstd, _ = C.combine_stats(means, vars_, counts, float(eps), float(momentum),
                                            running_mean, running_var)
        if want_mask:
            y, mask = C.apply_mask(xl, mean_g, invstd, weight, bias, zl, bool(fuse_relu))
        else:
            y, mask = C.apply(xl, mean_g, invstd, weight, bias, zl, bool(fuse_relu)), None
        ctx.save_for_backward(xl, zl if mask is None else None, weight, bias, mean_g, invstd, mask)
        ctx.src = None
        ctx.pg = pg
        ctx.world = max(world, 2) if collective else world  # > 1: collective backward
        ctx.fuse_relu = bool(fuse_relu)
        ctx.total = total
        ctx.count = count
        ctx.orig_shape = orig_shape
        ctx.has_z = z is not None
        ctx.shape_channel_last = shape_channel_last
        return y.view(orig_shape) if shape_channel_last else y

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        xl, zl, weight, bias, mean, invstd, mask = ctx.saved_tensors
        dyl = _to_logical(dy, ctx.shape_channel_last)
        need_w = weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        src = ctx.src
        res = src.result if src is not None else None
        if res is not None:
            src.result = None
        # the epilogue's g, untouched since: an in-place accumulation by another consumer
        # of this BN's output (autograd's InputBuffer adds into g) bumps its version, and
        # the slab sums would then miss that contribution -> the reduce pass below
        if res is not None and res[0] == dyl.data_ptr() and res[2] == dyl._version and (
                dyl.is_contiguous(memory_format=torch.channels_last)):
            # the consuming conv's dgrad epilogue already applied the ReLU mask (dy is
            # g) and summed (g, g*(x-mean)) per tile: no reduction pass, no dz store
            FUSED_BWD_CALLS[0] += 1
            if ctx.world > 1:
                direct, tw, tb, acc = _direct_targets(ctx.params, need_w)
                sum_dy, sum_dy_xmu, gw, gb = C.slab_reduce_grad(res[1], invstd, weight, need_w,
                                                               sum_scale=ctx.total,
                                                               grad_weight=tw, grad_bias=tb,
                                                               accumulate=acc)
                if direct:
                    # dgamma / dbeta accumulated into the DDP bucket views by the finalize
                    _ddp_direct.mark_ready(direct)
                    need_w = False
                n = sum_dy.numel()
                _allreduce(sum_dy.as_strided((2 * n,), (1,)), ctx.pg)
                total = 1.0
            else:
                sum_dy, sum_dy_xmu, gw, gb = C.slab_reduce_grad(res[1], invstd, weight, need_w)
                total = float(ctx.count)
            zc = getattr(ctx, "zctx", None) if ctx.has_z else None
            if _X2_BWD and zc is not None and ctx.world == 1 and _x2_target_ok(zc, ctx, weight):
                # dy (= dz) is the residual BN's gradient too: its backward sums ride on
                # this elementwise pass (reads its input once; no second pass over dy)
                xd, _, wd, _, md, isd, _ = zc.saved_tensors
                if C.backward_x2_ok(dyl, xl, xd):
                    need_wd = wd is not None and (zc.needs_input_grad[2] or zc.needs_input_grad[3])
                    dx, s1, s2, gw2, gb2 = C.backward_elemt_x2(
                        dyl, xl, mean, invstd, weight, bias, sum_dy, sum_dy_xmu, total, xd, md,
                        isd, wd, need_wd)
                    zc.pre = (dyl.data_ptr(), dyl._version, s1, s2, gw2, gb2)
                    return (dx, dyl, gw if need_w else None, gb if need_w else None, None, None,
                            None, None, None, None, None, None, None, None, None)
            dx, _ = C.backward_elemt(dyl, xl, mean, invstd, weight, bias, sum_dy, sum_dy_xmu,
                                     total, None, False, False)
            return (dx, dyl if ctx.has_z else None, gw if need_w else None,
                    gb if need_w else None, None, None, None, None, None, None, None, None, None,
                    None, None)
        pre = getattr(ctx, "pre", None)
        if pre is not None:
            ctx.pre = None
            if pre[0] == dyl.data_ptr() and pre[1] == dyl._version:
                # sums formed by the consuming BN's elementwise pass (backward_elemt_x2)
                _, _, sum_dy, sum_dy_xmu, gw, gb = pre
                X2_BWD_CALLS[0] += 1
                dx, _ = C.backward_elemt(dyl, xl, mean, invstd, weight, bias, sum_dy, sum_dy_xmu,
                                         float(ctx.count), None, False, False)
                if ctx.shape_channel_last:
                    dx = dx.view(ctx.orig_shape)
                return (dx, None, gw if need_w else None, gb if need_w else None, None, None,
                        None, None, None, None, None, None, None, None, None)
        if ctx.world > 1 and xl.is_cuda:
            # SyncBN: the reduce writes (sum_dy | sum_dy_xmu) / global_count into one [2C]
            # buffer (the scale is a device scalar from the forward's combine) -> ONE
            # in-place all_reduce yields the global means -> elementwise pass
            direct, tw, tb, acc = _direct_targets(ctx.params, need_w)
            sum_dy, sum_dy_xmu, gw, gb = C.reduce_grad(dyl, xl, mean, invstd, weight, bias, zl,
                                                       ctx.fuse_relu, need_w, mask=mask,
                                                       sum_scale=ctx.total, grad_weight=tw,
                                                       grad_bias=tb, accumulate=acc)
            if direct:
                _ddp_direct.mark_ready(direct)
                need_w = False
            n = sum_dy.numel()
            packed = sum_dy.as_strided((2 * n,), (1,))  # sum_dy_xmu follows sum_dy in memory
            _allreduce(packed, ctx.pg)
            dx, dz = C.backward_elemt(dyl, xl, mean, invstd, weight, bias, sum_dy, sum_dy_xmu,
                                      1.0, zl, ctx.fuse_relu, ctx.has_z, mask=mask)
            if ctx.shape_channel_last:
                dx = dx.view(ctx.orig_shape)
                if dz is not None:
                    dz = dz.view(ctx.orig_shape)
            return (dx, dz if ctx.has_z else None, gw if need_w else None,
                    gb if need_w else None, None, None, None, None, None, None, None, None, None, None, None)
        if ctx.world == 1 and xl.is_cuda:
            # reduce + elementwise, one native call
            dx, dz, gw, gb = C.backward_local(dyl, xl, mean, invstd, weight, bias, zl,
                                              ctx.fuse_relu, need_w, ctx.has_z, mask=mask)
            if ctx.shape_channel_last:
                dx = dx.view(ctx.orig_shape)
                if dz is not None:
                    dz = dz.view(ctx.orig_shape)
            return (dx, dz if ctx.has_z else None, gw if need_w else None,
                    gb if need_w else None, None, None, None, None, None, None, None, None, None, None, None)
        sum_dy, sum_dy_xmu, gw, gb = C.reduce_grad(dyl, xl, mean, invstd, weight, bias, zl,
                                                   ctx.fuse_relu, need_w, mask=mask)
        if ctx.world > 1:
            packed = torch.cat([sum_dy, sum_dy_xmu])
            dist.all_reduce(packed, group=ctx.pg)
            n = sum_dy.numel()
            # normalise by the global count on the device (no host sync)
            packed = packed / ctx.total
            sum_dy, sum_dy_xmu = packed[:n], packed[n:]
            total = 1.0
        else:
            total = float(ctx.count)
        dx, dz = C.backward_elemt(dyl, xl, mean, invstd, weight, bias, sum_dy, sum_dy_xmu, total,
                                  zl, ctx.fuse_relu, ctx.has_z, mask=mask)
        if ctx.shape_channel_last:
            dx = dx.view(ctx.orig_shape)
            if dz is not None:
                dz = dz.view(ctx.orig_shape)
        return (dx, dz if ctx.has_z else None, gw if need_w else None, gb if need_w else None,
                None, None, None, None, None, None, None, None, None, None, None)


def take_slab(x, bn):
    """(slab, shift) when ``x`` carries the epilogue statistics a conv computed for
    ``bn`` (ops/conv.py) - consumed once - else (None, None)."""
    ent = getattr(x, "_amd_bn_stats", None)
    if ent is None:
        return None, None
    del x._amd_bn_stats
    slab, shift, owner = ent
    if owner is not bn or slab.size(1) != x.size(1):
        return None, None
    return slab, shift


def batch_norm_act(x, weight, bias, running_mean, running_var, training, momentum, eps,
                   z=None, fuse_relu=False, process_group=False, shape_channel_last=False,
                   num_batches_tracked=None, force_collectives=False, slab=None, slab_shift=None):
    """Functional fused BN(+z)(+ReLU).  ``process_group=False`` -> local statistics.
    ``num_batches_tracked`` (int64 tensor) is incremented on the device.  ``slab``:
    per-tile statistics a producing conv already summed ([C][2][S], ops/conv.py)."""
    if training:
        _TLS.src = None
        y = BatchNormFunction.apply(x, z, weight, bias, running_mean, running_var, eps, momentum,
                                    process_group, fuse_relu, shape_channel_last,
                                    num_batches_tracked, force_collectives, slab, slab_shift)
        src = _TLS.src
        if src is not None:
            _TLS.src = None
            y._amd_bn_src = src
        return y
    # inference: running statistics (autograd through plain torch ops)
    if shape_channel_last:
        xs = x.movedim(-1, 1)
        zs = z.movedim(-1, 1) if z is not None else None
    else:
        xs, zs = x, z
    y = torch.nn.functional.batch_norm(xs, running_mean, running_var, weight, bias, False, 0.0, eps)
    if zs is not None:
        y = y + zs
    if fuse_relu:
        y = torch.relu(y)
    return y.movedim(1, -1) if shape_channel_last else y


class BatchNorm2dReLU(torch.nn.BatchNorm2d):
    """BatchNorm2d with optional fused residual add and ReLU on the gfx950 kernels
    (local, per-GPU statistics).  ``forward(x, z=None)`` = relu(bn(x) + z)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True, fuse_relu=True, **kw):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, **kw)
        self.fuse_relu = fuse_relu

    def _amd_accepts_slab(self):
        """Can take statistics from the producing conv's epilogue (ops/conv.py)."""
        return self.training and (self.momentum is not None or not self.track_running_stats)

    def forward(self, x, z=None):
        slab, shift = take_slab(x, self)
        if not x.is_cuda and not _native.available():
            y = super().forward(x)
            if z is not None:
                y = y + z
            return torch.relu(y) if self.fuse_relu else y
        momentum = 0.0 if self.momentum is None else self.momentum
        nbt = None
        if self.training and self.track_running_stats:
            if self.momentum is None:  # cumulative average needs the count on the host
                self.num_batches_tracked.add_(1)
                momentum = 1.0 / float(self.num_batches_tracked)
            else:
                nbt = self.num_batches_tracked  # incremented inside the stats kernel
        use_batch = self.training or not self.track_running_stats
        return batch_norm_act(x, self.weight, self.bias,
                              self.running_mean if self.track_running_stats else None,
                              self.running_var if self.track_running_stats else None,
                              use_batch, momentum, self.eps, z=z, fuse_relu=self.fuse_relu,
                              process_group=False, num_batches_tracked=nbt,
                              slab=slab if use_batch else None, slab_shift=shift)


# ---------------------------------------------------------------- relu(bn3(x) + bn_d(xd))
# ResNet's downsample block output in ONE apply pass (csrc/hip/bn_nhwc.hip apply_k ZA): the
# downsample BN's output is formed on load (rounded as its own apply pass would store it, so
# y and the ReLU mask are bitwise the unfused result) and never written - its apply pass (a
# read and a write of the tensor) goes; the backward runs bn3's elementwise pass with the
# downsample BN's sums (backward_elemt_x2) and that BN's elementwise pass.
_FUSE_DS = os.environ.get("APEX_AMD_BN_DS_FUSE", "1") == "1"
FUSED_DS_CALLS = [0]


class BatchNormAddBNReLUFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, xd, w, b, wd, bd, rm, rv, nbt, rmd, rvd, nbtd, eps, mom, epsd, momd,
                slab, shift, slabd, shiftd):
        C = _C()
        ctx.params = (w, b, wd, bd)
        if ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            _ddp_direct.note_use(w, b)
        if ctx.needs_input_grad[4] or ctx.needs_input_grad[5]:
            _ddp_direct.note_use(wd, bd)
        count = x.numel() // x.size(1)

        def stats(t, sl, sh, rm_, rv_, nbt_, eps_, mom_):
            if sl is not None:
                return C.slab_train_stats(sl, count, sh, rm_, rv_, nbt_, float(eps_), float(mom_))
            return C.train_stats(t, rm_, rv_, nbt_, float(eps_), float(mom_))

        mean, invstd = stats(x, slab, shift, rm, rv, nbt, eps, mom)
        meand, invstdd = stats(xd, slabd, shiftd, rmd, rvd, nbtd, epsd, momd)
        y, mask = C.apply2_mask(x, mean, invstd, w, b, xd, meand, invstdd, wd, bd)
        ctx.save_for_backward(x, xd, w, b, wd, bd, mean, invstd, meand, invstdd, mask)
        ctx.src = _TLS.src = _bwd_src(x, x, mean, invstd, w, b, mask, True, True)
        ctx.count = count
        FUSED_DS_CALLS[0] += 1
        return y

    @staticmethod
    def backward(ctx, dy):
        C = _C()
        x, xd, w, b, wd, bd, mean, invstd, meand, invstdd, mask = ctx.saved_tensors
        need = w is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        needd = wd is not None and (ctx.needs_input_grad[4] or ctx.needs_input_grad[5])
        cnt = float(ctx.count)
        src = ctx.src
        res = src.result if src is not None else None
        if res is not None:
            src.result = None
        if (res is not None and res[0] == dy.data_ptr() and res[2] == dy._version
                and dy.is_contiguous(memory_format=torch.channels_last)):
            # dy is the consuming conv's g (ReLU mask applied) with its sums in a slab
            FUSED_BWD_CALLS[0] += 1
            s1, s2, gw, gb = C.slab_reduce_grad(res[1], invstd, w, need)
            dx, t1, t2, gwd, gbd = C.backward_elemt_x2(dy, x, mean, invstd, w, b, s1, s2, cnt,
                                                       xd, meand, invstdd, wd, needd)
            dxd, _ = C.backward_elemt(dy, xd, meand, invstdd, wd, bd, t1, t2, cnt, None, False,
                                      False)
        else:
            dyc = dy.contiguous(memory_format=torch.channels_last)
            s1, s2, gw, gb = C.reduce_grad(dyc, x, mean, invstd, w, b, None, True, need,
                                           mask=mask)
            dx, d = C.backward_elemt(dyc, x, mean, invstd, w, b, s1, s2, cnt, None, True, True,
                                     mask=mask)
            dxd, _, gwd, gbd = C.backward_local(d, xd, meand, invstdd, wd, bd, None, False,
                                                needd, False)
        return (dx, dxd, gw if need else None, gb if need else None, gwd if needd else None,
                gbd if needd else None) + (None,) * 14


def _ds_fusable(bn, x, bnd, xd):
    return (_FUSE_DS and type(bn) is BatchNorm2dReLU and type(bnd) is BatchNorm2dReLU
            and bn.training and bnd.training and bn.fuse_relu and not bnd.fuse_relu
            and bn.track_running_stats and bnd.track_running_stats
            and bn.momentum is not None and bnd.momentum is not None
            and bn.affine == bnd.affine and x.is_cuda and xd.is_cuda and x.dim() == 4
            and x.shape == xd.shape and x.dtype == xd.dtype
            and x.dtype in (torch.bfloat16, torch.float16)
            and (not bn.affine or bn.weight.dtype == bnd.weight.dtype)
            and _native.available() and _C().backward_x2_ok(x, x, xd))


def bn_add_bn_relu(bn, x, bnd, xd):
    """relu(bn(x) + bnd(xd)) - one fused pass where both are local BatchNorm2dReLU modules in
    training mode (bn with ReLU, bnd without), else the two module calls."""
    if not _ds_fusable(bn, x, bnd, xd):
        return bn(x, bnd(xd))
    slab, shift = take_slab(x, bn)
    slabd, shiftd = take_slab(xd, bnd)
    _TLS.src = None
    y = BatchNormAddBNReLUFunction.apply(
        x, xd, bn.weight, bn.bias, bnd.weight, bnd.bias, bn.running_mean, bn.running_var,
        bn.num_batches_tracked, bnd.running_mean, bnd.running_var, bnd.num_batches_tracked,
        bn.eps, bn.momentum, bnd.eps, bnd.momentum, slab, shift, slabd, shiftd)
    src = _TLS.src
    if src is not None:
        _TLS.src = None
        y._amd_bn_src = src
    return y
