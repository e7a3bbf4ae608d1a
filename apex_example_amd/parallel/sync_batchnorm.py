"""SyncBatchNorm (apex@f3a960f8 apex/parallel/optimized_sync_batchnorm.py and the
Python fallback apex/parallel/sync_batchnorm.py).

Forward: local Welford-equivalent stats on the gfx950 split-reduction kernels,
ONE packed all_gather of [mean, biased var, count] per layer (apex older
revisions used three), Chan combine (exact for uneven per-rank batches),
running-stat momentum update with the unbiased global variance, fused
normalise (+z)(+ReLU).  Backward: local reduction, ONE packed all_reduce of
[sum_dy, sum_dy_xmu], fused elementwise dx (+dz).  Collectives run over RCCL
(nccl backend) on MI355X or gloo on CPU.

Communicator: with ``process_group=None`` the layers share ONE dedicated
process group over all ranks (created on first use - every rank reaches its
first SyncBN forward in the same order, so the collective creation lines up),
with high-priority HIP streams under RCCL.  These per-layer collectives are
latency-bound and sit on the critical path (the compute stream waits on them at
once), so they must not queue behind DDP's multi-MB bucket all-reduces, which
run on their own communicator (``parallel.distributed``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch.nn.modules.batchnorm import _BatchNorm

from .. import _native
from ..ops.batch_norm import BatchNormFunction  # noqa: F401  (re-exported)


_COMM_GROUPS = {}


def is_syncbn_comm_group(pg):
    """True for the dedicated SyncBN group made by ``syncbn_comm_group`` (only SyncBN
    collectives ever run on its communicator)."""
    return any(g is pg for g in _COMM_GROUPS.values())


def syncbn_comm_group():
    """The dedicated SyncBN process group for the current world (see module doc)."""
    key = id(dist.group.WORLD)
    g = _COMM_GROUPS.get(key)
    if g is not None:
        try:  # destroyed by destroy_process_group() (a new world may reuse the id)
            alive = g in dist.distributed_c10d._world.pg_map
        except AttributeError:
            alive = True
        if not alive:
            g = None
    if g is None:
        if dist.get_backend() == "nccl":
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            g = dist.new_group(ranks=list(range(dist.get_world_size())), pg_options=opts)
        else:
            g = dist.new_group(ranks=list(range(dist.get_world_size())))
        _COMM_GROUPS.clear()
        _COMM_GROUPS[key] = g
    return g


class SyncBatchNorm(_BatchNorm):
    """Synchronized batch norm over ``process_group`` (default: the world).

    ``channel_last=True`` follows apex: the input's LAST dimension is C (e.g. an
    [N, H, W, C] tensor).  A PyTorch channels_last-format [N, C, H, W] tensor
    needs no flag - its memory layout is detected and the NHWC kernels run.
    ``fuse_relu=True`` applies ReLU after the (optional) residual ``z``.
    ``force_collectives=True`` runs the cross-rank path (packed all_gather of the
    statistics, packed all_reduce of the gradient sums) even when the group has
    one rank: the 1-GPU test / bench hook for SyncBN's RCCL code
    (``set_syncbn_force_collectives``).
    """

    warned = False

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True, process_group=None, channel_last=False,
                 fuse_relu=False, force_collectives=False):
        super(SyncBatchNorm, self).__init__(num_features, eps=eps, momentum=momentum,
                                            affine=affine,
                                            track_running_stats=track_running_stats)
        self.process_group = process_group
        self.channel_last = channel_last
        self.fuse_relu = fuse_relu
        self.force_collectives = force_collectives

    def _specify_process_group(self, process_group):
        self.process_group = process_group

    def _specify_channel_last(self, channel_last):
        self.channel_last = channel_last

    def _check_input_dim(self, input):
        if input.dim() < 2:
            raise ValueError("expected at least 2D input (got {}D input)".format(input.dim()))

    def _amd_accepts_slab(self):
        """Can take statistics from the producing conv's epilogue (ops/conv.py): the
        fused path (native kernels, NCHW-shaped input) in training mode."""
        return (self.training and not self.channel_last and _native.available()
                and (self.momentum is not None or not self.track_running_stats))

    def forward(self, input, z=None):
        self._check_input_dim(input)
        from ..ops.batch_norm import take_slab
        slab, shift = take_slab(input, self)
        channel_last = self.channel_last if input.dim() != 2 else False
        if (not self.training and self.track_running_stats and not channel_last
                and not self.fuse_relu and z is None):
            # fall back to pytorch implementation for inference
            return F.batch_norm(input, self.running_mean, self.running_var, self.weight,
                                self.bias, False, 0.0, self.eps)
        exponential_average_factor = 0.0
        nbt = None
        if self.training and self.track_running_stats:
            if self.momentum is None:
                self.num_batches_tracked += 1
                exponential_average_factor = 1.0 / float(self.num_batches_tracked)
            else:
                exponential_average_factor = self.momentum
                if _native.available():
                    nbt = self.num_batches_tracked  # incremented by the BN op on the device
                else:
                    self.num_batches_tracked += 1
        use_batch = self.training or not self.track_running_stats
        if not use_batch:
            from ..ops.batch_norm import batch_norm_act

            return batch_norm_act(input, self.weight, self.bias, self.running_mean,
                                  self.running_var, False, 0.0, self.eps, z=z,
                                  fuse_relu=self.fuse_relu, shape_channel_last=channel_last)
        if not _native.available():
            return _python_sync_bn(self, input, z, exponential_average_factor, channel_last)
        pg = self.process_group
        force = bool(getattr(self, "force_collectives", False))
        if not (dist.is_available() and dist.is_initialized()):
            pg = False
        elif pg is None and (dist.get_world_size() > 1 or force):
            pg = syncbn_comm_group()
        from ..ops.batch_norm import batch_norm_act

        # (batch_norm_act tags the output for the consuming conv's BN-backward epilogue)
        return batch_norm_act(input, self.weight, self.bias,
                              self.running_mean if self.track_running_stats else None,
                              self.running_var if self.track_running_stats else None,
                              True, exponential_average_factor, self.eps, z=z,
                              fuse_relu=self.fuse_relu, process_group=pg,
                              shape_channel_last=channel_last, num_batches_tracked=nbt,
                              force_collectives=force, slab=slab, slab_shift=shift)


def set_syncbn_force_collectives(module, on=True):
    """Turn the 1-rank collective path of every SyncBatchNorm in ``module`` on/off;
    returns the number of layers changed."""
    n = 0
    for m in module.modules():
        if isinstance(m, SyncBatchNorm):
            m.force_collectives = bool(on)
            n += 1
    return n


class _PySyncBNFunction(torch.autograd.Function):
    """Reference implementation in torch ops (apex sync_batchnorm_kernel.py)."""

    @staticmethod
    def forward(ctx, input, weight, bias, running_mean, running_variance, eps, process_group,
                world_size, momentum):
        input = input.contiguous()
        C = input.size(1)
        xf = input.float().transpose(0, 1).reshape(C, -1)
        local_count = xf.size(1)
        local_sum = xf.sum(1)
        local_sqsum = (xf * xf).sum(1)
        cnt = torch.tensor([float(local_count)], device=input.device)
        packed = torch.cat([local_sum, local_sqsum, cnt])
        if world_size > 1:
            dist.all_reduce(packed, group=process_group)
        n = packed[-1]
        mean = packed[:C] / n
        var = packed[C:2 * C] / n - mean * mean
        if running_mean is not None:
            with torch.no_grad():
                running_mean.mul_(1 - momentum).add_(momentum * mean.to(running_mean.dtype))
                unb = var * n / (n - 1).clamp_min(1)
                running_variance.mul_(1 - momentum).add_(momentum * unb.to(running_variance.dtype))
        invstd = (var + eps).rsqrt()
        shape = [1, C] + [1] * (input.dim() - 2)
        xhat = (input.float() - mean.view(shape)) * invstd.view(shape)
        out = xhat
        if weight is not None:
            out = out * weight.float().view(shape) + bias.float().view(shape)
        ctx.save_for_backward(xhat, weight, invstd)
        ctx.pg, ctx.world, ctx.n = process_group, world_size, n
        return out.to(input.dtype)

    @staticmethod
    def backward(ctx, grad_output):
        xhat, weight, invstd = ctx.saved_tensors
        C = xhat.size(1)
        shape = [1, C] + [1] * (xhat.dim() - 2)
        go = grad_output.float().contiguous()
        dims = [0] + list(range(2, xhat.dim()))
        grad_bias = go.sum(dims)
        grad_weight = (go * xhat).sum(dims)
        packed = torch.cat([grad_bias, grad_weight])
        if ctx.world > 1:
            dist.all_reduce(packed, group=ctx.pg)
        mdy = packed[:C] / ctx.n
        mdyx = packed[C:] / ctx.n
        w = weight.float().view(shape) if weight is not None else 1.0
        gi = (go - mdy.view(shape) - xhat * mdyx.view(shape)) * invstd.view(shape) * w
        gw = grad_weight.to(weight.dtype) if weight is not None else None
        gb = grad_bias.to(weight.dtype) if weight is not None else None
        return gi.to(grad_output.dtype), gw, gb, None, None, None, None, None, None


def _python_sync_bn(mod, input, z, momentum, channel_last):
    if channel_last:
        input = input.movedim(-1, 1)
        z = z.movedim(-1, 1) if z is not None else None
    pg = mod.process_group or (dist.group.WORLD if dist.is_initialized() else None)
    world = dist.get_world_size(pg) if dist.is_initialized() else 1
    out = _PySyncBNFunction.apply(input, mod.weight, mod.bias,
                                  mod.running_mean if mod.track_running_stats else None,
                                  mod.running_var if mod.track_running_stats else None,
                                  mod.eps, pg, world, momentum)
    if z is not None:
        out = out + z
    if mod.fuse_relu:
        out = torch.relu(out)
    return out.movedim(1, -1) if channel_last else out


class SyncBatchNormPython(SyncBatchNorm):
    """Apex's pure-Python SyncBatchNorm (used when the extension is absent); kept
    as the numerical reference for the fused kernels."""

    def forward(self, input, z=None):
        if not self.training and self.track_running_stats and z is None and not self.fuse_relu:
            return F.batch_norm(input, self.running_mean, self.running_var, self.weight,
                                self.bias, False, 0.0, self.eps)
        momentum = self.momentum if self.momentum is not None else 0.0
        if self.training and self.track_running_stats:
            self.num_batches_tracked += 1
        return _python_sync_bn(self, input, z, momentum, self.channel_last and input.dim() != 2)
