"""apex.parallel.DistributedDataParallel / Reducer for MI355X
(apex@f3a960f8 apex/parallel/distributed.py).

One process per GPU; collectives go through ``torch.distributed`` (backend
"nccl" = RCCL over xGMI on MI355X, "gloo" on CPU).  The bucketing / overlap core
is the C++ ``_C.reducer.Reducer``:

* gradients are views into persistent flat bucket buffers (no flatten /
  unflatten copies per step);
* buckets are filled in gradient-arrival order (recorded on the first backward,
  synchronised from rank 0, then fixed) and all-reduced as soon as they are
  complete, in the same order on every rank, overlapping the rest of backward;
* the end-of-backward epilogue makes the compute stream wait on every bucket
  and raises if a bucket was never reduced.

Bucket size (``message_size``, elements): Apex's default 1e7, or ``"auto"``: a
bucket of XGMI_BUCKET_BYTES (32 MiB) ON THE WIRE - elements = 32 MiB / the size
of the dtype the collective actually moves (fp32 for bf16 buckets under the fp32
accumulation default).  The sizing model (docs/DDP_TUNING.md): an 8-rank RCCL
all-reduce over the fully connected xGMI mesh (7 links x ~153 GB/s per GPU)
costs t(S) = a + 2(n-1)/n * S / B with a ~ 30 us per call and B ~ 300 GB/s
of bus bandwidth for multi-channel rings; a bucket must be >= ~16 MB to keep a
under 20 % of t (link-rate), and the LAST bucket's t is exposed after backward,
so buckets much above ~64 MB lengthen the tail.  32 MiB sits in that window for
1..8 ranks; see tools/allreduce_sweep.py to refit a and B on a node.

Calibration (``"auto"`` at world size > 1, env ``APEX_AMD_DDP_CALIBRATE=0`` to skip):
at construction DDP times fp32 all-reduces of 1, 8 and 32 MiB on its own bucket
communicator, takes the slowest rank's median per size (one MAX all-reduce, so every
rank derives the same number), fits ``a`` and ``B`` by least squares and sizes the
bucket from the link-rate rule - the smallest power-of-two MiB with a <= 20 % of t(S),
clamped to [8, 64] MiB - instead of the model's assumed constants.  The fit and the
choice are kept in ``ddp.calibration`` (bench.py writes them to its JSON), so the
driver's multi-GPU runs record the node's own a and B.  A fit that is not physical
(a <= 0 or B <= 0: noise) keeps the 32 MiB default.

Tapered tail (``tapered_buckets``, default on; env ``APEX_AMD_DDP_TAPER=0`` for Apex's
plain size cut): buckets are cut from the END of the gradient-arrival order with limits
message_size/16, /8, /4, /2, then message_size - the buckets that can only launch when
backward ends (the first layers' gradients arrive last) are small, so the exposed
all-reduce tail is short, and the early gradients still travel in full buckets.

Communicators (RCCL): the buckets go to a DEDICATED process group whose HIP
streams are created high-priority (``ProcessGroupNCCL.Options
(is_high_priority_stream=True)``), not to the default group: bucket
all-reduces are then scheduled ahead of the backward kernels they overlap, and
they never queue behind (or interleave with) collectives other code issues on
the default group - SyncBatchNorm uses its own communicator as well
(``parallel.sync_batchnorm``).

Precision: bf16 buckets are reduced in fp32 by default (RCCL rounds the running
sum to the wire dtype at every ring hop; with an 8-bit mantissa that costs ~3 bits
over 8 ranks) - ``allreduce_always_fp32=None`` means "fp32 sums for bf16 buckets,
native for fp16" (Apex's fp16 behaviour); True / False force an fp32 / native
all-reduce for every 16-bit bucket.  How the fp32 sum of a bf16 bucket travels
(``bf16_wire``, env ``APEX_AMD_DDP_BF16_WIRE``):

* ``"rsag"`` (default): fp32 reduce-scatter + in-place bf16 all-gather - each rank's
  shard is summed in fp32 and rounded to bf16 once (one rounding of an fp32 sum, as
  the fp32 all-reduce; bitwise equal to it on gloo, while on RCCL the two may sum in
  different orders), at (n-1)/n x 6 bytes per element on the wire instead of 2 (n-1)/n x 4;
* ``"fp32"``: one fp32 all-reduce of an up-cast copy (8 bytes per element);
* ``"native"``: bf16 all-reduce (4 bytes per element, rounded at every hop).

docs/DDP_TUNING.md records the measurements behind the default.
"""
from __future__ import annotations

import contextlib
import os
import warnings

import torch
import torch.distributed as dist
from torch.nn.modules import Module

from .. import _native
from ..ops import _ddp_direct


XGMI_BUCKET_BYTES = 32 << 20
_CAL_SIZES_MIB = (1, 8, 32)
_CAL_MIN_MIB, _CAL_MAX_MIB = 8, 64


def _group_world(pg):
    return dist.get_world_size(pg) if pg is not None else dist.get_world_size()


def flat_dist_call(tensors, call, extra_args=None, group=None):
    """apex flat_dist_call: coalesce per dtype, run a collective, copy back.
    all_reduce results are averaged over the world size (apex semantics)."""
    buckets = {}
    for t in tensors:
        buckets.setdefault((t.dtype, t.device), []).append(t)
    for (dtype, device), ts in buckets.items():
        flat = torch.cat([t.contiguous().view(-1) for t in ts])
        kwargs = {}
        if group is not None:
            kwargs["group"] = group
        if extra_args is not None:
            call(flat, *extra_args, **kwargs)
        else:
            call(flat, **kwargs)
        if call is dist.all_reduce:
            flat.div_(_group_world(group))
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


def split_half_float_double(tensors):
    dtypes = [torch.float16, torch.bfloat16, torch.float32, torch.float64]
    buckets = []
    for dtype in dtypes:
        bucket = [t for t in tensors if t.dtype == dtype]
        if bucket:
            buckets.append(bucket)
    return buckets


def split_by_type(tensors):
    buckets = {}
    for t in tensors:
        buckets.setdefault(t.dtype, []).append(t)
    return buckets


def extract_tensors(maybe_tensor, tensor_list):
    if torch.is_tensor(maybe_tensor):
        tensor_list.append(maybe_tensor)
    else:
        try:
            for item in maybe_tensor:
                extract_tensors(item, tensor_list)
        except TypeError:
            return


class Reducer(object):
    """Manual all-reduce helper (apex.parallel.Reducer): broadcast params at
    construction, ``reduce()`` averages gradients across ranks when called."""

    def __init__(self, module_or_grads_list, process_group=None):
        self.process_group = process_group
        if isinstance(module_or_grads_list, Module):
            self.module = module_or_grads_list
            flat_dist_call([p.data for p in self.module.parameters()], dist.broadcast, (0,),
                           group=process_group)
        else:
            self.module = None
            self.grads = []
            extract_tensors(module_or_grads_list, self.grads)

    def reduce(self):
        if self.module:
            grads = [p.grad.data for p in self.module.parameters() if p.grad is not None]
            flat_dist_call(grads, dist.all_reduce, group=self.process_group)
        else:
            flat_dist_call(self.grads, dist.all_reduce, group=self.process_group)


class DistributedDataParallel(Module):
    """Data parallel wrapper with flat-bucket, overlapped gradient all-reduce.

    Apex-compatible constructor::

        DistributedDataParallel(module, message_size=10000000, delay_allreduce=False,
            shared_param=None, allreduce_trigger_params=None, retain_allreduce_buffers=False,
            allreduce_always_fp32=False, num_allreduce_streams=1,
            allreduce_communicators=None, gradient_average=True,
            gradient_predivide_factor=1.0, gradient_average_split_factor=None, prof=False)

    Extensions: ``process_group``, ``allow_unused`` (tolerate params without
    grads), ``bucket_align`` (elements; views 16-B aligned for vector kernels),
    ``use_avg_op`` (ReduceOp.AVG instead of SUM + scale; default on for RCCL),
    ``high_priority_streams`` (RCCL: a dedicated bucket communicator on
    high-priority streams; default on), ``force_collectives`` (issue the bucket
    all-reduces even at world size 1 - test hook for 1-GPU boxes),
    ``allreduce_always_fp32=None`` (auto: fp32 accumulation for bf16 buckets).

    ``retain_allreduce_buffers``: in Apex it keeps the flat all-reduced buffers alive
    after the backward (they are otherwise freed once unflattened into ``.grad``) and
    exposes them as ``allreduce_buffers``.  Here every parameter's ``.grad`` is a view
    into its persistent flat bucket, so the buffers are always retained and
    ``allreduce_buffers`` always returns them; the flag is accepted for API parity and
    changes nothing (``tests/test_parallel_gloo.py`` checks the buffers alias the grads).
    ``prof=True``: roctx ranges around the forward and, in the C++ reducer, around each
    bucket's launch and the post-backward finalize (Apex ranges its hook and
    ``comm_ready_buckets``).
    """

    def __init__(self, module, message_size=10000000, delay_allreduce=False, shared_param=None,
                 allreduce_trigger_params=None, retain_allreduce_buffers=False,
                 allreduce_always_fp32=None, num_allreduce_streams=1,
                 allreduce_communicators=None, gradient_average=True,
                 gradient_predivide_factor=1.0, gradient_average_split_factor=None, prof=False,
                 process_group=None, allow_unused=False, bucket_align=64, use_avg_op=None,
                 high_priority_streams=True, force_collectives=False, bf16_wire=None,
                 tapered_buckets=None):
        super().__init__()
        if not dist.is_initialized():
            raise RuntimeError("DistributedDataParallel requires torch.distributed to be "
                               "initialized (init_process_group)")
        if shared_param is not None:
            raise ValueError("shared_param is no longer supported as an option.  It was "
                             "misleadingly named from the start.  It turns out overlapping "
                             "communication with computation should work fine with shared "
                             "parameters.  If you still wish to delay communication to the end "
                             "of the backward pass, use delay_allreduce=True|False instead.")
        if gradient_average_split_factor is not None:
            print("Warning:  gradient_average_split_factor has been renamed to "
                  "gradient_predivide_factor.  For now, gradient_average_split_factor will also "
                  "work, but please update to gradient_predivide_factor instead.")
            gradient_predivide_factor = gradient_average_split_factor

        self.module = module
        self.process_group = process_group
        self.backend = dist.get_backend(process_group)
        self.world_size = _group_world(process_group)
        self._message_size_arg = message_size
        self.delay_allreduce = delay_allreduce
        self.retain_allreduce_buffers = retain_allreduce_buffers
        self.allreduce_always_fp32 = allreduce_always_fp32
        self.gradient_average = gradient_average
        self.gradient_predivide_factor = gradient_predivide_factor
        self.num_allreduce_streams = num_allreduce_streams
        self.prof = prof
        self.allow_unused = allow_unused
        self.bucket_align = bucket_align
        if use_avg_op is None:
            use_avg_op = self.backend == "nccl"
        self.use_avg_op = bool(use_avg_op)
        self.force_collectives = bool(force_collectives)
        self.bf16_wire = bf16_wire or os.environ.get("APEX_AMD_DDP_BF16_WIRE", "rsag")
        if self.bf16_wire not in ("rsag", "fp32", "native"):
            raise ValueError("bf16_wire must be 'rsag', 'fp32' or 'native'")
        if tapered_buckets is None:
            tapered_buckets = os.environ.get("APEX_AMD_DDP_TAPER", "1") == "1"
        self.tapered_buckets = bool(tapered_buckets)
        self._trigger_params = allreduce_trigger_params
        self.custom_allreduce_triggers = allreduce_trigger_params is not None

        self.high_priority_streams = bool(high_priority_streams) and self.backend == "nccl"
        self._bucket_pgs = None
        self._comm_pg = process_group
        if allreduce_communicators is not None:
            self._bucket_pgs = list(allreduce_communicators[0] if isinstance(
                allreduce_communicators, tuple) else allreduce_communicators)
            self.num_allreduce_streams = len(self._bucket_pgs)
        elif process_group is not None:
            # new_group() is a collective over the WHOLE world: with a caller-given
            # subgroup only that subgroup's ranks construct this DDP (and disjoint
            # subgroups would pass different rank lists), so no communicator is
            # created here.  The buckets use the caller's group (round-robin over
            # it when num_allreduce_streams > 1); pass allreduce_communicators=
            # [...] built on every rank for dedicated / high-priority ones.
            if num_allreduce_streams > 1:
                self._bucket_pgs = [process_group] * num_allreduce_streams
            self.high_priority_streams = False
        elif num_allreduce_streams > 1:
            self._bucket_pgs = [self._new_comm_group() for _ in range(num_allreduce_streams)]
        elif self.high_priority_streams and (self.world_size > 1 or self.force_collectives):
            # the whole world constructs DDP in the same order, so this collective
            # group creation lines up across ranks
            self._comm_pg = self._new_comm_group()

        self.active_params = self._collect_params()
        self.calibration = None
        self.message_size = self._resolve_message_size(message_size)
        if self.backend == "nccl":
            for p in self.active_params:
                assert p.is_cuda, "NCCL backend only supports model parameters to be on GPU."

        # broadcast parameters from the group's first rank (apex: rank 0; buffers are
        # NOT broadcast).  dist.broadcast takes a GLOBAL source rank.
        if self.world_size > 1:
            src = 0 if process_group is None else dist.get_process_group_ranks(process_group)[0]
            flat_dist_call([p.data for p in self.module.parameters()], dist.broadcast, (src,),
                           group=process_group)
        self._build_reducer()

    # ------------------------------------------------------------------ internals
    def _new_comm_group(self):
        """A communicator over the whole world (called only when process_group is
        None, i.e. when every rank of the world constructs this DDP)."""
        ranks = list(range(dist.get_world_size()))
        if self.backend == "nccl" and self.high_priority_streams:
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            return dist.new_group(ranks=ranks, pg_options=opts)
        return dist.new_group(ranks=ranks)

    def _resolve_message_size(self, message_size):
        """Elements per bucket: an int as given (Apex semantics) or "auto" - 32 MiB of
        wire bytes for the dtype the bucket collective moves (module docstring)."""
        if message_size != "auto":
            return int(message_size)
        dtypes = [p.dtype for p in self.active_params] or [torch.float32]
        dom = max(set(dtypes), key=dtypes.count)
        mode = self._fp32_mode()
        wire = 4 if (dom == torch.float32 or mode == 1
                     or (mode in (2, 3) and dom == torch.bfloat16)) else torch.finfo(dom).bits // 8
        nbytes = XGMI_BUCKET_BYTES
        if self.world_size > 1 and os.environ.get("APEX_AMD_DDP_CALIBRATE", "1") != "0":
            self.calibration = self._calibrate()
            nbytes = self.calibration["bucket_mib"] << 20
        return max(1, nbytes // wire)

    def _calibrate(self, sizes_mib=_CAL_SIZES_MIB, warmup=3, reps=7):
        """Measure t(S) of an fp32 all-reduce on the bucket communicator and size the
        bucket from the fit (module docstring).  Collective: every rank of the group
        runs the same calls in the same order."""
        import time

        pg = self._comm_pg if self._comm_pg is not None else dist.group.WORLD
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" \
            else torch.device("cpu")
        n = self.world_size
        med = []
        for mib in sizes_mib:
            buf = torch.zeros((mib << 20) // 4, dtype=torch.float32, device=dev)
            ts = []
            for i in range(warmup + reps):
                if dev.type == "cuda":
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
                        enable_timing=True)
                    e0.record()
                    dist.all_reduce(buf, group=pg)
                    e1.record()
                    e1.synchronize()
                    dt = e0.elapsed_time(e1) * 1e-3
                else:
                    t0 = time.perf_counter()
                    dist.all_reduce(buf, group=pg)
                    dt = time.perf_counter() - t0
                if i >= warmup:
                    ts.append(dt)
            med.append(sorted(ts)[len(ts) // 2])
            del buf
        # the slowest rank's times: identical inputs to the fit on every rank
        v = torch.tensor(med, dtype=torch.float64, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=pg)
        t = [float(x) for x in v.tolist()]
        S = [float(m << 20) for m in sizes_mib]
        k = len(S)
        sm, tm = sum(S) / k, sum(t) / k
        var = sum((x - sm) ** 2 for x in S)
        slope = sum((x - sm) * (y - tm) for x, y in zip(S, t)) / var if var > 0 else 0.0
        a = tm - slope * sm
        ring = 2.0 * (n - 1) / n
        rec = {"sizes_mib": list(sizes_mib), "t_us": [round(x * 1e6, 1) for x in t],
               "collective": "fp32 all_reduce", "ranks": n}
        if a <= 0 or slope <= 0:
            rec.update({"a_us": round(a * 1e6, 2), "busbw_gbps": None,
                        "bucket_mib": XGMI_BUCKET_BYTES >> 20, "fit": "unphysical: default kept"})
            return rec
        busbw = ring / slope
        need = 4.0 * a * busbw / ring  # a <= 20 % of t(S)
        mib = _CAL_MIN_MIB
        while mib < _CAL_MAX_MIB and (mib << 20) < need:
            mib *= 2
        rec.update({"a_us": round(a * 1e6, 2), "busbw_gbps": round(busbw / 1e9, 1),
                    "link_rate_min_mib": round(need / 2**20, 2), "bucket_mib": mib,
                    "fit": "least squares"})
        return rec

    def _fp32_mode(self):
        """Reducer fp32 mode: 0 native, 1 every 16-bit bucket as an fp32 all-reduce,
        2 bf16 buckets as an fp32 all-reduce, 3 bf16 buckets as an fp32 reduce-scatter
        + bf16 all-gather (fp16 / fp32 buckets native in 2 and 3)."""
        if self.allreduce_always_fp32 is None:
            env = os.environ.get("APEX_AMD_DDP_FP32")  # A/B override of the auto rule
            if env in ("0", "1", "2", "3"):
                return int(env)
            return {"rsag": 3, "fp32": 2, "native": 0}[self.bf16_wire]
        return 1 if self.allreduce_always_fp32 else 0

    def wire_format(self):
        """How each bucket dtype travels: {dtype name: 'fp32 all-reduce' | ...}."""
        mode = self._fp32_mode()
        out = {}
        for p in self.active_params:
            d = p.dtype
            if d in (torch.bfloat16, torch.float16) and (
                    mode == 1 or (mode == 2 and d == torch.bfloat16)):
                out[str(d)] = "fp32 all-reduce"
            elif d == torch.bfloat16 and mode == 3:
                out[str(d)] = "fp32 reduce-scatter + bf16 all-gather"
            else:
                out[str(d)] = "%s all-reduce" % str(d).replace("torch.", "")
        return out

    def _collect_params(self):
        seen = set()
        params = []
        for p in self.module.parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                params.append(p)
        return params

    def _build_reducer(self):
        C = _native.require()
        pg = self._comm_pg if self._comm_pg is not None else dist.group.WORLD
        triggers = []
        if self._trigger_params is not None:
            ids = {id(p) for p in self._trigger_params}
            triggers = [i for i, p in enumerate(self.active_params) if id(p) in ids]
        self.reducer = C.reducer.Reducer(self.active_params, pg, self.message_size,
                                         self._fp32_mode(),
                                         float(self.gradient_predivide_factor),
                                         self.gradient_average, self.delay_allreduce,
                                         self.use_avg_op, triggers, int(self.bucket_align))
        self.reducer.set_allow_unused(self.allow_unused)
        if not self.tapered_buckets:
            self.reducer.set_tapered(False)
        self.reducer.set_force_collectives(self.force_collectives)
        self.reducer.set_prof(bool(self.prof))
        if self._bucket_pgs:
            self.reducer.set_bucket_process_groups(self._bucket_pgs)
        # parameters listed more than once in the module tree (tied weights) get their
        # gradient from several uses: never announced early (ops/_ddp_direct.py)
        uses = {}
        for _, p in self.module.named_parameters(remove_duplicate=False):
            uses[id(p)] = uses.get(id(p), 0) + 1
        shared = [i for i, p in enumerate(self.active_params) if uses.get(id(p), 0) > 1]
        if shared:
            self.reducer.set_no_direct(shared)
        import weakref
        ref = weakref.ref(self.reducer)
        for i, p in enumerate(self.active_params):
            p._amd_grad_is_bucket_view = True
            # side-stream weight gradients (ops/conv.py) announce themselves here
            p._amd_ddp_slot = (ref, i)

    def __setstate__(self, state):
        super().__setstate__(state)
        self._build_reducer()

    def __getstate__(self):
        attrs = self.__dict__.copy()
        attrs.pop("reducer", None)
        return attrs

    # ------------------------------------------------------------------ API
    def enable_allreduce(self):
        self.reducer.set_enabled(True)

    def disable_allreduce(self):
        self.reducer.set_enabled(False)

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (torch.nn.parallel.DDP spelling)."""
        prev = self.reducer.enabled()
        self.reducer.set_enabled(False)
        try:
            yield
        finally:
            self.reducer.set_enabled(prev)

    @property
    def needs_refresh(self):
        return self.reducer.needs_refresh()

    @property
    def allreduce_buffers(self):
        return list(self.reducer.bucket_tensors())

    def bucket_layout(self):
        """List of buckets, each a list of indices into ``active_params``."""
        return [list(b) for b in self.reducer.layout()]

    def enable_bucket_timing(self, on=True):
        """Record HIP events around every bucket (see ``bucket_timing``)."""
        self.reducer.set_timing(bool(on))

    def bucket_timing(self):
        """Timing of the last backward (needs ``enable_bucket_timing()``), in ms
        from the first gradient: ``{"backward_ms", "exposed_tail_ms",
        "launch_ms": [...], "joined_ms": [...], "bucket_numel": [...]}``.
        ``exposed_tail_ms`` is the time between the end of backward and the
        compute stream having joined every bucket's all-reduce - the part of
        the communication that overlap did not hide.  None if nothing timed."""
        t = list(self.reducer.timing())
        if not t:
            return None
        nb = (len(t) - 2) // 2
        return {"backward_ms": t[0], "exposed_tail_ms": t[1], "launch_ms": t[2:2 + nb],
                "joined_ms": t[2 + nb:], "bucket_numel": list(self.reducer.bucket_numels())}

    def zero_grad_buckets(self):
        """Zero every gradient with one memset per bucket (grads stay views)."""
        self.reducer.zero_grads()

    def forward(self, *inputs, **kwargs):
        if not self.delay_allreduce:
            param_list = self._collect_params()
            if (len(param_list) != len(self.active_params)
                    or any(a is not b for a, b in zip(param_list, self.active_params))):
                warnings.warn("DistributedDataParallel: the set of parameters requiring grad "
                              "changed; rebuilding the gradient buckets")
                self.reducer.remove_hooks()
                self.active_params = param_list
                self._build_reducer()
        if self.prof:
            torch.cuda.nvtx.range_push("forward pass DDP logic")
        # own ops count their parameters' forward uses per DDP forward (direct-gradient
        # path eligibility, ops/_ddp_direct.py)
        _ddp_direct.forward_epoch(self.reducer)
        out = self.module(*inputs, **kwargs)
        if self.prof:
            torch.cuda.nvtx.range_pop()
        return out
