"""DistributedFusedAdam: ZeRO-style sharded Adam(W) over RCCL
(apex@f3a960f8 apex/contrib/optimizers/distributed_fused_adam.py, SURVEY.md
A-24 / P-08).

Every rank keeps the full model parameters (16-bit or fp32) for forward and
backward, but the optimizer state - fp32 master weights, exp_avg, exp_avg_sq -
exists only for its 1/world shard.  MI355X-native layout and schedule:

* each param group's parameters and gradients are VIEWS into one flat,
  padded buffer (``p.data`` / ``p.grad`` alias it: no flatten / unflatten copy
  per step);
* the flat buffer is cut into ``dwu_num_blocks`` blocks; block b is
  reduce-scattered (ReduceOp.AVG, one RCCL call: every GPU receives its
  1/world slice of the averaged gradients), updated by ONE multi-tensor Adam
  launch over the local shards (reads the 16-bit grad slice, updates the fp32
  master / moments and writes the 16-bit parameter slice in the same pass,
  csrc/hip/mt_optim.hip), then all-gathered back into the flat parameter
  buffer.  Blocks pipeline: the update of block b overlaps the collectives of
  its neighbours.  Large, few collectives - the right shape for xGMI's
  point-to-point links;
* optional global gradient clipping (``max_grad_norm``) and loss-scale
  overflow checking run on the device (one tiny all_reduce each, no host
  sync); an overflow turns the Adam launch into a no-op on every rank.

Use it INSTEAD of a DDP wrapper (it reduces the gradients itself).  Loss
scaling: ``set_global_scale(scale)`` (float or device tensor) before ``step``;
the kernel multiplies the gradients by 1 / scale.  With gloo (CPU tests) the
reduce-scatter is emulated by all_reduce + slice.
"""
from __future__ import annotations

import types

import torch
import torch.distributed as dist

from ... import _native, amp_C


class DistributedFusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 eps_inside_sqrt=False, weight_decay=0.0, max_grad_norm=0.0, amsgrad=False,
                 adam_w_mode=True, process_group=None, dwu_num_blocks=4, align=128,
                 check_overflow=None, **unused_apex_kwargs):
        if amsgrad:
            raise RuntimeError("DistributedFusedAdam does not support the AMSGrad variant.")
        if eps_inside_sqrt:
            raise RuntimeError("eps_inside_sqrt is not supported (apex deprecates it).")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay, max_grad_norm=max_grad_norm, step=0)
        super().__init__(params, defaults)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self._pg = process_group
        init = dist.is_available() and dist.is_initialized()
        self._world = dist.get_world_size(process_group) if init else 1
        self._rank = dist.get_rank(process_group) if init else 0
        self._nccl = self._world > 1 and dist.get_backend(process_group) == "nccl"
        self._nb = max(1, int(dwu_num_blocks))
        self._align = int(align)
        self._grad_scale = 1.0
        self._check_overflow = check_overflow
        self._noop = None
        self._groups = [self._build(g) for g in self.param_groups]

    # ------------------------------------------------------------------ layout
    def _build(self, group):
        params = [p for p in group["params"] if p.requires_grad]
        if not params:
            return None
        dtype, dev = params[0].dtype, params[0].device
        for p in params:
            if p.dtype != dtype or p.device != dev:
                raise TypeError("DistributedFusedAdam: a param group must share one dtype and "
                                "device (split mixed groups into several param groups)")
        a, W, nb = self._align, self._world, self._nb
        offs, n = [], 0
        for p in params:
            offs.append(n)
            n += (p.numel() + a - 1) // a * a
        unit = W * nb * a
        total = max(unit, (n + unit - 1) // unit * unit)
        flat_p = torch.zeros(total, dtype=dtype, device=dev)
        flat_g = torch.zeros(total, dtype=dtype, device=dev)
        with torch.no_grad():
            for p, o in zip(params, offs):
                flat_p[o:o + p.numel()].copy_(p.detach().reshape(-1))
        if W > 1:  # replicas start from rank 0's parameters
            dist.broadcast(flat_p, src=self._global(0), group=self._pg)
        for p, o in zip(params, offs):
            p.data = flat_p[o:o + p.numel()].view_as(p)
            p.grad = flat_g[o:o + p.numel()].view_as(p)
        blk = total // nb
        sh = blk // W
        r = self._rank
        G = types.SimpleNamespace(params=params, dtype=dtype, device=dev, flat_p=flat_p,
                                  flat_g=flat_g, blk=blk, sh=sh)
        G.p_blocks = [flat_p[b * blk:(b + 1) * blk] for b in range(nb)]
        G.g_blocks = [flat_g[b * blk:(b + 1) * blk] for b in range(nb)]
        G.p_shards = [pb[r * sh:(r + 1) * sh] for pb in G.p_blocks]
        if W == 1:
            G.g_shards = list(G.g_blocks)
        else:
            G.g_shard_buf = torch.empty(nb * sh, dtype=dtype, device=dev)
            G.g_shards = [G.g_shard_buf[b * sh:(b + 1) * sh] for b in range(nb)]
        fopt = dict(dtype=torch.float32, device=dev)
        if dtype == torch.float32:
            G.master = None
            G.masters = G.p_shards  # updated in place, then all-gathered
        else:
            G.master = torch.cat([s.float() for s in G.p_shards])
            G.masters = [G.master[b * sh:(b + 1) * sh] for b in range(nb)]
        G.exp_avg = torch.zeros(nb * sh, **fopt)
        G.exp_avg_sq = torch.zeros(nb * sh, **fopt)
        G.ms = [G.exp_avg[b * sh:(b + 1) * sh] for b in range(nb)]
        G.vs = [G.exp_avg_sq[b * sh:(b + 1) * sh] for b in range(nb)]
        G.step_t = None
        return G

    def _global(self, group_rank):
        if self._pg is None:
            return group_rank
        return dist.get_global_rank(self._pg, group_rank)

    # ------------------------------------------------------------------ API
    def set_global_scale(self, global_scale):
        """Loss scale the gradients carry (float or 1-element fp32 device tensor)."""
        self._grad_scale = global_scale

    @property
    def global_scale(self):
        return self._grad_scale

    def zero_grad(self, set_to_none=False):
        """Gradients are views into the flat buffers: always zeroed in place."""
        for G in self._groups:
            if G is not None:
                G.flat_g.zero_()

    def _reduce_scatter(self, G, b):
        gin, out = G.g_blocks[b], G.g_shards[b]
        if self._world == 1:
            return None
        if self._nccl:
            return dist.reduce_scatter_tensor(out, gin, op=dist.ReduceOp.AVG, group=self._pg,
                                              async_op=True)
        dist.all_reduce(gin, group=self._pg)  # gloo: no reduce_scatter
        out.copy_(gin[self._rank * G.sh:(self._rank + 1) * G.sh]).div_(self._world)
        return None

    def _all_gather(self, G, b):
        if self._world == 1:
            return None
        if self._nccl:
            return dist.all_gather_into_tensor(G.p_blocks[b], G.p_shards[b], group=self._pg,
                                               async_op=True)
        dist.all_gather(list(G.p_blocks[b].chunk(self._world)), G.p_shards[b].clone(),
                        group=self._pg)
        return None

    @torch.no_grad()
    def step(self, closure=None, skip_overflow_check=False):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        scaled = not (isinstance(self._grad_scale, (int, float)) and self._grad_scale == 1.0)
        check = self._check_overflow if self._check_overflow is not None else scaled
        check = check and not skip_overflow_check
        for group, G in zip(self.param_groups, self._groups):
            if G is None:
                continue
            if self._noop is None or self._noop.device != G.device:
                self._noop = torch.zeros(1, dtype=torch.int32, device=G.device)
            noop = self._noop
            noop.zero_()
            needs_global = check or group["max_grad_norm"] > 0
            works = [self._reduce_scatter(G, b) for b in range(self._nb)]
            if needs_global:
                for w in works:
                    if w is not None:
                        w.wait()
                works = [None] * self._nb
            # gradient multiplier: 1 / loss_scale [* clip coefficient], on the device
            if isinstance(self._grad_scale, torch.Tensor):
                mult = 1.0 / self._grad_scale.float().reshape(1)
            else:
                mult = 1.0 / float(self._grad_scale)
            if check:
                amp_C.multi_tensor_check_finite(65536, noop, [G.g_shards])
                if self._world > 1:
                    dist.all_reduce(noop, op=dist.ReduceOp.MAX, group=self._pg)
            if group["max_grad_norm"] > 0:
                norm, _ = amp_C.multi_tensor_l2norm(65536, noop, [G.g_shards])
                sq = (norm * norm).reshape(1)
                if self._world > 1:
                    dist.all_reduce(sq, group=self._pg)
                gnorm = sq.sqrt() * mult
                clip = torch.clamp(group["max_grad_norm"] / (gnorm + 1e-6), max=1.0)
                mult = clip * mult
            if check and G.device.type == "cuda":
                if G.step_t is None:
                    G.step_t = torch.tensor([int(group["step"])], dtype=torch.int32,
                                            device=G.device)
                step = G.step_t
            else:
                group["step"] += 1
                step = group["step"]
            beta1, beta2 = group["betas"]
            gathers = []
            for b in range(self._nb):
                if works[b] is not None:
                    works[b].wait()
                lists = [[G.g_shards[b]], [G.masters[b]], [G.ms[b]], [G.vs[b]]]
                if G.master is not None:
                    lists.append([G.p_shards[b]])
                amp_C.multi_tensor_adam(65536, noop, lists, group["lr"], beta1, beta2,
                                        group["eps"], step, self.adam_w_mode,
                                        1 if group["bias_correction"] else 0,
                                        group["weight_decay"], scale=mult)
                gathers.append(self._all_gather(G, b))
            if isinstance(step, torch.Tensor):
                _native.require().mt.advance_step(step, noop)
            for w in gathers:
                if w is not None:
                    w.wait()
        return loss

    # ------------------------------------------------------------------ checkpoint
    def _materialize_steps(self):
        for group, G in zip(self.param_groups, self._groups):
            if G is not None and G.step_t is not None:
                group["step"] = int(G.step_t.item())

    def state_dict(self):
        """This rank's shard of the optimizer state (apex DistributedFusedAdam
        checkpoints are per rank as well)."""
        self._materialize_steps()
        groups = [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]
        shards = []
        for G in self._groups:
            if G is None:
                shards.append(None)
                continue
            shards.append({"master": torch.cat([m.float() for m in G.masters]),
                           "exp_avg": G.exp_avg.clone(), "exp_avg_sq": G.exp_avg_sq.clone()})
        return {"world_size": self._world, "rank": self._rank, "num_blocks": self._nb,
                "param_groups": groups, "shards": shards}

    def load_state_dict(self, state_dict):
        if (state_dict["world_size"] != self._world or state_dict["rank"] != self._rank
                or state_dict["num_blocks"] != self._nb):
            raise ValueError("DistributedFusedAdam state was saved with a different world size / "
                             "rank / dwu_num_blocks")
        for g, sg in zip(self.param_groups, state_dict["param_groups"]):
            g.update(sg)
        with torch.no_grad():
            for G, sh in zip(self._groups, state_dict["shards"]):
                if G is None:
                    continue
                m = sh["master"].to(G.device)
                for b in range(self._nb):
                    G.masters[b].copy_(m[b * G.sh:(b + 1) * G.sh])
                    if G.master is not None:
                        G.p_shards[b].copy_(G.masters[b])
                G.exp_avg.copy_(sh["exp_avg"])
                G.exp_avg_sq.copy_(sh["exp_avg_sq"])
                G.step_t = None
                for w in [self._all_gather(G, b) for b in range(self._nb)]:
                    if w is not None:
                        w.wait()
