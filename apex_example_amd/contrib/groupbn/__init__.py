"""NHWC group BatchNorm (apex@f3a960f8 apex/contrib/groupbn/batch_norm.py,
SURVEY.md A-24): ``BatchNorm2d_NHWC(num_features, fuse_relu=False, bn_group=1,
...)`` on channels-last activations with the fused add + ReLU of
``forward(x, z=None)``.

Apex builds this on peer-memory exchanges between ``bn_group`` GPUs; here the
statistics of a group are combined with the same single packed RCCL
all_gather / all_reduce per layer as SyncBatchNorm (ranks grouped in
consecutive blocks of ``bn_group``), and the elementwise / reduction passes are
the gfx950 NHWC kernels of ops/batch_norm.py (1-bit ReLU mask for the residual
form).  Input: an [N, C, H, W] tensor in channels_last memory format, or an
[N, H, W, C] tensor (apex's layout) - the trailing-C view is detected.
"""
from __future__ import annotations

import torch.distributed as dist
from torch.nn.modules.batchnorm import _BatchNorm

from ...ops.batch_norm import BatchNormFunction, batch_norm_act

_GROUPS = {}


def _bn_group(bn_group):
    if bn_group <= 1 or not (dist.is_available() and dist.is_initialized()):
        return False  # local statistics
    world = dist.get_world_size()
    assert world % bn_group == 0, "world size must be a multiple of bn_group"
    if bn_group not in _GROUPS:
        from ...parallel import create_syncbn_process_group

        _GROUPS[bn_group] = create_syncbn_process_group(bn_group)
    return _GROUPS[bn_group]


class BatchNorm2d_NHWC(_BatchNorm):  # noqa: N801 (apex name)
    def __init__(self, num_features, fuse_relu=False, bn_group=1, max_cta_per_sm=2,
                 cta_launch_margin=12, multi_stream=False, eps=1e-5, momentum=0.1):
        super().__init__(num_features, eps=eps, momentum=momentum, affine=True,
                         track_running_stats=True)
        self.fuse_relu = fuse_relu
        self.bn_group = bn_group
        # occupancy knobs of apex's CUDA kernels; grid sizing here is automatic
        self.max_cta_per_sm = max_cta_per_sm
        self.cta_launch_margin = cta_launch_margin
        self.multi_stream = multi_stream

    def _check_input_dim(self, input):
        if input.dim() != 4:
            raise ValueError("expected 4D input (got {}D input)".format(input.dim()))

    def forward(self, x, z=None):
        self._check_input_dim(x)
        if z is not None:
            assert self.fuse_relu, "the residual add is fused together with ReLU only (apex)"
        # apex layout: [N, H, W, C] contiguous -> C is the last dim of the shape
        shape_cl = (x.size(-1) == self.num_features and x.size(1) != self.num_features)
        if self.training:
            self.num_batches_tracked.add_(1)
            return BatchNormFunction.apply(x, z, self.weight, self.bias, self.running_mean,
                                           self.running_var, self.eps, self.momentum,
                                           _bn_group(self.bn_group), self.fuse_relu, shape_cl,
                                           None)
        return batch_norm_act(x, self.weight, self.bias, self.running_mean, self.running_var,
                              False, 0.0, self.eps, z=z, fuse_relu=self.fuse_relu,
                              shape_channel_last=shape_cl)
