"""Channels-last max pooling on the gfx950 kernels (csrc/hip/pool.hip).

The forward keeps a one-byte tap index per output element; the backward is a
gather over the windows covering each input pixel (no atomics, every dx
element written once), replacing ATen's NHWC max_pool2d kernels, which cost
~0.9 ms per ResNet-50 step at bs 256 on MI355X (profiles/).
"""
from __future__ import annotations


import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native

# A/B switch for the fused stem (tools, docs/PERF.md)
_FUSE_STEM = True
# its backward: the BN-backward sums inside the max-pool gather (csrc/hip/pool.hip BNR)
_FUSE_STEM_BWD = True
_GAP_KERNEL = True


class MaxPool2dNHWCFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = _native.require().pool.max_fwd(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.geom = (x.size(2), x.size(3), k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, p = ctx.geom
        return _native.require().pool.max_bwd(dy, idx, H, W, k, s, p), None, None, None


class BNReLUMaxPoolFunction(torch.autograd.Function):
    """maxpool(relu(batchnorm(x))) in training mode without materialising the
    BatchNorm output (the ResNet stem: conv 7x7 -> BN -> ReLU -> max-pool 3x3/2).

    Forward: the BN statistics pass (running stats and num_batches_tracked
    updated on the device), then ONE pooling pass that applies the BN affine +
    ReLU to x as it loads the window (csrc/hip/pool.hip) - the separate BN
    apply (read x, write y: 2 x 411 MB per step at ResNet-50 bs 256) disappears.
    Backward: the pooling gather yields the gradient of the BN+ReLU output, then
    the BN reduce + elementwise kernels (ReLU condition recomputed from x)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, eps, momentum, k, s, p,
                pg=None, slab=None, shift=None):
        C = _native.require()
        inv_total = None
        count = x.numel() // x.size(1)
        if pg is None and slab is not None:
            # statistics from the stem conv's epilogue slab (no pass over x)
            mean, invstd = C.bn.slab_train_stats(slab, count, shift, running_mean, running_var,
                                                 nbt, float(eps), float(momentum))
        elif pg is None:
            mean, invstd = C.bn.train_stats(x, running_mean, running_var, nbt, float(eps),
                                            float(momentum))
        else:
            # SyncBatchNorm stem: the same packed stats exchange as ops/batch_norm.py
            # (one all_gather of [mean | var | count]), then the fused pool pass
            import torch.distributed as dist
            world = dist.get_world_size(pg)
            packed = (C.bn.slab_packed_stats(slab, count, shift) if slab is not None
                      else C.bn.local_stats_packed(x))
            gathered = torch.empty(world * packed.numel(), dtype=packed.dtype, device=x.device)
            if dist.get_backend(pg) == "nccl":
                dist.all_gather_into_tensor(gathered, packed, group=pg)
            else:
                dist.all_gather(list(gathered.chunk(world)), packed, group=pg)
            mean, invstd, inv_total = C.bn.combine_stats_sync(
                gathered.view(world, -1), float(eps), float(momentum), running_mean,
                running_var, nbt)
        y, idx = C.pool.max_fwd_bn(x, mean, invstd, weight, bias, k, s, p)
        ctx.save_for_backward(x, weight, bias, mean, invstd, idx)
        ctx.geom = (x.size(2), x.size(3), k, s, p)
        ctx.pg, ctx.inv_total = pg, inv_total
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, bias, mean, invstd, idx = ctx.saved_tensors
        H, W, k, s, p = ctx.geom
        C = _native.require()
        need_w = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        if (ctx.pg is None and _FUSE_STEM_BWD and (k, s, p) == (3, 2, 1) and x.size(1) == 64
                and x.element_size() == 2 and dy.dtype == x.dtype):
            # the BN-backward sums formed inside the pooling gather (one pass over x instead
            # of a reduction pass over dbn and x)
            dbn, slab = C.pool.max_bwd_bn(dy, idx, H, W, x, mean, invstd, weight, bias)
            sum_dy, sum_dy_xmu, gw, gb = C.bn.slab_reduce_grad(slab, invstd, weight, need_w)
            count = float(x.numel() // x.size(1))
        elif ctx.pg is None:
            dbn = C.pool.max_bwd(dy, idx, H, W, k, s, p)
            sum_dy, sum_dy_xmu, gw, gb = C.bn.reduce_grad(dbn, x, mean, invstd, weight, bias,
                                                          None, True, need_w)
            count = float(x.numel() // x.size(1))
        else:
            import torch.distributed as dist
            dbn = C.pool.max_bwd(dy, idx, H, W, k, s, p)
            sum_dy, sum_dy_xmu, gw, gb = C.bn.reduce_grad(dbn, x, mean, invstd, weight, bias,
                                                          None, True, need_w,
                                                          sum_scale=ctx.inv_total)
            n = sum_dy.numel()
            dist.all_reduce(sum_dy.as_strided((2 * n,), (1,)), group=ctx.pg)
            count = 1.0
        dx, _ = C.bn.backward_elemt(dbn, x, mean, invstd, weight, bias, sum_dy, sum_dy_xmu,
                                    count, None, True, False)
        return (dx, gw if need_w else None, gb if need_w else None,
                None, None, None, None, None, None, None, None, None, None, None)


def _stem_pg(bn):
    """None: local statistics (BatchNorm2dReLU); a process group: SyncBatchNorm whose
    cross-rank statistics the fused stem exchanges itself; False: not fusable."""
    from .batch_norm import BatchNorm2dReLU

    if type(bn) is BatchNorm2dReLU:
        return None
    from ..parallel.sync_batchnorm import SyncBatchNorm, syncbn_comm_group
    import torch.distributed as dist

    if type(bn) is not SyncBatchNorm or bn.channel_last:
        return False
    if not (dist.is_available() and dist.is_initialized()):
        return None
    if bn.process_group is not None:
        return bn.process_group
    if dist.get_world_size() > 1 or getattr(bn, "force_collectives", False):
        return syncbn_comm_group()
    return None


def bn_relu_maxpool_fusable(x, bn, pool):
    """True when ``pool(relu(bn(x)))`` can run as BNReLUMaxPoolFunction: a local
    BatchNorm2dReLU, or a SyncBatchNorm (the statistics are exchanged first)."""
    k, s, p = pool.kernel_size, pool.stride, pool.padding
    return (_FUSE_STEM and getattr(bn, "fuse_relu", False) and _stem_pg(bn) is not False
            and bn.training and bn.track_running_stats and bn.momentum is not None
            and x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
            and x.size(1) % 8 == 0 and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and bn.weight is not None and bn.weight.dtype == torch.float32
            and bn.bias.dtype == torch.float32 and bn.running_mean.dtype == torch.float32
            and isinstance(k, int) and isinstance(s, int) and isinstance(p, int)
            and pool.dilation == 1 and not pool.ceil_mode and not pool.return_indices
            and p <= k // 2 and k <= 15 and _native.available())


def bn_relu_maxpool(x, bn, pool):
    from .batch_norm import take_slab

    slab, shift = take_slab(x, bn)  # the stem conv's epilogue statistics, if it wrote them
    return BNReLUMaxPoolFunction.apply(x, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                       bn.num_batches_tracked, bn.eps, bn.momentum,
                                       pool.kernel_size, pool.stride, pool.padding,
                                       _stem_pg(bn), slab, shift)


class MaxPool2dNHWC(nn.MaxPool2d):
    """nn.MaxPool2d whose channels-last GPU path runs the gfx950 kernels."""

    def forward(self, x):
        k, s, p = self.kernel_size, self.stride, self.padding
        if (x.is_cuda and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)
                and isinstance(k, int) and isinstance(s, int) and isinstance(p, int)
                and self.dilation == 1 and not self.ceil_mode and not self.return_indices
                and p <= k // 2 and k <= 15):
            return MaxPool2dNHWCFunction.apply(x, k, s, p)
        return F.max_pool2d(x, self.kernel_size, self.stride, self.padding, self.dilation,
                            self.ceil_mode, self.return_indices)


class GlobalAvgPoolNHWCFunction(torch.autograd.Function):
    """x.mean((2, 3), keepdim=True) whose gradient is written channels-last by one
    vectorized kernel (csrc/hip/pool.hip gap_bwd_k).  ATen's gradient is an expanded
    [N, C, H, W] view; the fused BN backward behind it needs a dense channels-last
    tensor, and the resulting .contiguous() ran as strided 2-byte copies (~80 us per
    copy for ResNet-50's [256, 2048, 7, 7] at bs 256, twice per step)."""

    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.size(2), x.size(3))
        return x.mean((2, 3), keepdim=True)

    @staticmethod
    def backward(ctx, dy):
        H, W = ctx.hw
        return _native.require().pool.gap_bwd(dy, H, W)


class GlobalAvgPool2dNHWC(nn.AdaptiveAvgPool2d):
    """nn.AdaptiveAvgPool2d((1, 1)) with the channels-last gradient kernel on the GPU."""

    def __init__(self):
        super().__init__((1, 1))

    def forward(self, x):
        if (_GAP_KERNEL and x.is_cuda and x.dim() == 4
                and x.is_contiguous(memory_format=torch.channels_last)
                and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
                and _native.available()):
            return GlobalAvgPoolNHWCFunction.apply(x)
        return super().forward(x)
