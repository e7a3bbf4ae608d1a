"""apex.parallel for MI355X: DDP over RCCL/xGMI, SyncBatchNorm, LARC."""
from __future__ import annotations

import torch
import torch.distributed as dist

from .distributed import DistributedDataParallel, Reducer  # noqa: F401
from .LARC import LARC  # noqa: F401
from .sync_batchnorm import (SyncBatchNorm, SyncBatchNormPython,  # noqa: F401
                             set_syncbn_force_collectives)

ReduceOp = dist.ReduceOp


def convert_syncbn_model(module, process_group=None, channel_last=False):
    """Recursively replace every ``_BatchNorm`` (not InstanceNorm) with
    ``SyncBatchNorm``, sharing running buffers and cloning affine params
    (apex.parallel.convert_syncbn_model)."""
    mod = module
    if isinstance(module, torch.nn.modules.instancenorm._InstanceNorm):
        return module
    if isinstance(module, torch.nn.modules.batchnorm._BatchNorm):
        fuse_relu = getattr(module, "fuse_relu", False)
        mod = SyncBatchNorm(module.num_features, module.eps, module.momentum, module.affine,
                            module.track_running_stats, process_group, channel_last=channel_last,
                            fuse_relu=fuse_relu)
        mod.running_mean = module.running_mean
        mod.running_var = module.running_var
        mod.num_batches_tracked = module.num_batches_tracked
        if module.affine:
            mod.weight.data = module.weight.data.clone().detach()
            mod.bias.data = module.bias.data.clone().detach()
    for name, child in module.named_children():
        mod.add_module(name, convert_syncbn_model(child, process_group=process_group,
                                                  channel_last=channel_last))
    del module
    return mod


def create_syncbn_process_group(group_size):
    """Create process groups of ``group_size`` contiguous ranks for SyncBatchNorm
    (every rank creates every group, as torch.distributed requires) and return
    the group this rank belongs to.  group_size 0 -> None (whole world)."""
    if group_size == 0:
        return None
    world_size = dist.get_world_size()
    assert world_size >= group_size
    assert world_size % group_size == 0
    group = None
    for group_num in range(world_size // group_size):
        group_ids = range(group_num * group_size, (group_num + 1) * group_size)
        cur_group = dist.new_group(ranks=group_ids)
        if dist.get_rank() // group_size == group_num:
            group = cur_group
    assert group is not None
    return group
