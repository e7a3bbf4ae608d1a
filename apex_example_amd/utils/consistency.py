"""Cross-rank correctness signals for multi-GPU runs (bench.py at N > 1).

Data-parallel training keeps every rank's parameters BITWISE identical: the DDP
all-reduce (or the rsag wire's reduce-scatter + all-gather) hands every rank the same
reduced bytes, and the optimizer is deterministic per element.  A rank whose weights
drift - a missed bucket, a stream race on one rank, a collective that reduced
different buckets on different ranks - is caught here after the timed region:

* ``tensor_digest``: two int64 checksums of the raw bits of a list of tensors (a plain
  sum of the words and a position-weighted sum; integer wrap-around is associative, so
  the result does not depend on the reduction order of the device);
* ``cross_rank_match``: every rank's digest per named group, all-reduced with MAX and
  MIN - the group matches on every rank iff MAX == MIN;
* ``comm_info``: the rank count and rank that the RCCL communicator of a process group
  itself reports (``ncclCommCount`` / ``ncclCommUserRank``), i.e. what the collectives
  really span - not just what the launcher said.

Reference: the reference trains one replica per GPU with apex DDP
(/root/reference/test_apex_distributed_spawn.py:57,109,122) and never checks that the
replicas stayed in sync; this is the self-check its first multi-GPU run would need.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional

import torch
import torch.distributed as dist

_INT_OF_SIZE = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def _words(t: torch.Tensor) -> torch.Tensor:
    t = t.detach()
    if t.is_complex():
        t = torch.view_as_real(t)
    t = t.contiguous().view(-1)
    return t.view(_INT_OF_SIZE[t.element_size()]).to(torch.int64)


def tensor_digest(tensors: Iterable[torch.Tensor], device=None) -> torch.Tensor:
    """int64 [2]: (sum of words, sum of words * position weight) over the raw bits of
    every tensor, in order.  Bitwise-equal inputs give equal digests on any device."""
    acc = None
    for i, t in enumerate(tensors):
        if t is None or t.numel() == 0:
            continue
        w = _words(t)
        pos = torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 65521
        pos += (i * 7919) % 65521 + 1
        d = torch.stack([w.sum(), (w * pos).sum()])
        acc = d if acc is None else acc + d.to(acc.device)
    if acc is None:
        acc = torch.zeros(2, dtype=torch.int64)
    return acc.to(device) if device is not None else acc


def _group_device(group) -> torch.device:
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def cross_rank_match(groups: Dict[str, List[torch.Tensor]], group=None) -> Dict[str, dict]:
    """{name: {"match": bool, "digest": hex of the MIN digest over ranks (every rank's
    digest when they match)}} for each named tensor list, identical on every rank.  A
    collective: call on every rank, same names in the same order."""
    names = list(groups)
    dev = _group_device(group)
    d = torch.stack([tensor_digest(groups[n], device=dev) for n in names]) if names else \
        torch.zeros(0, 2, dtype=torch.int64, device=dev)
    hi, lo = d.clone(), d.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    hi, lo = hi.cpu(), lo.cpu()
    out = {}
    for i, n in enumerate(names):
        out[n] = {"match": bool(torch.equal(hi[i], lo[i])),
                  "digest": "%016x%016x" % tuple(int(v) & (2 ** 64 - 1) for v in lo[i].tolist())}
    return out


def comm_info(pg) -> Optional[dict]:
    """{"backend", "size", "rank"} of ``pg``; for RCCL the size and rank come from the
    communicator itself (``ncclCommCount`` / ``ncclCommUserRank``) once it exists."""
    if pg is None or not dist.is_initialized():
        return None
    backend = dist.get_backend(pg)
    rec = {"backend": backend, "size": dist.get_world_size(pg), "rank": dist.get_rank(pg),
           "source": "process group"}
    if backend == "nccl":
        try:
            from .. import _native

            ptr = int(pg._get_backend(torch.device("cuda"))._comm_ptr())
            if ptr:
                n, r = _native.require().reducer.rccl_comm_info(ptr)
                rec.update(size=int(n), rank=int(r), source="rccl communicator")
        except Exception as e:  # communicator not created yet / older torch
            rec["source"] = "process group (%s)" % type(e).__name__
    return rec


def model_state_groups(model: torch.nn.Module, optimizer=None) -> Dict[str, List[torch.Tensor]]:
    """The tensors replicas must agree on: parameters, buffers, and the optimizer's own
    parameters (amp O2's fp32 masters) plus its state tensors (momentum, Adam moments)."""
    params = [p for p in model.parameters()]
    buffers = [b for b in model.buffers()]
    groups = {"params": params, "buffers": buffers}
    if optimizer is not None:
        seen = {id(p) for p in params}
        masters, state = [], []
        for g in optimizer.param_groups:
            for p in g["params"]:
                if id(p) not in seen:
                    seen.add(id(p))
                    masters.append(p)
                st = optimizer.state.get(p, {}) if hasattr(optimizer, "state") else {}
                for k in sorted(st):
                    v = st[k]
                    if torch.is_tensor(v) and v.numel() > 1:
                        state.append(v)
        groups["optimizer_params"] = masters
        groups["optimizer_state"] = state
    return groups
