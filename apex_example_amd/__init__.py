"""apex_example_amd - an MI355X-native (gfx950 / CDNA4) mixed-precision and
data-parallel training framework with NVIDIA Apex's capabilities and API:

* ``amp``            - O0-O3 opt levels, fp16/bf16 casting, fp32 master weights,
                       dynamic loss scaling (device-resident, sync-free), Apex
                       checkpoint format;
* ``optimizers``     - FusedSGD / FusedAdam / FusedLAMB / FusedNovoGrad /
                       FusedAdagrad on a multi-tensor-apply engine;
* ``normalization``  - FusedLayerNorm / FusedRMSNorm;
* ``parallel``       - DistributedDataParallel (flat-bucket all-reduce over RCCL,
                       overlapped with backward), SyncBatchNorm, LARC;
* ``fp16_utils``     - convert_network, FP16_Optimizer, ...;
* ``multi_tensor_apply``, ``amp_C``, ``apex_C`` - Apex's low-level surfaces;
* ``contrib``        - fused softmax cross entropy, fast multi-head attention,
                       NHWC group BN, ZeRO-style DistributedFusedAdam;
* ``reparameterization`` (weight norm), ``RNN``, ``mlp``, ``pyprof``.

All kernels are hand-written HIP for gfx950 (csrc/hip), built in-tree by
``python tools/build_ext.py``.
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401
from . import amp, fp16_utils, multi_tensor_apply, normalization, optimizers, parallel  # noqa: F401
from . import contrib, fused_dense, reparameterization  # noqa: F401
