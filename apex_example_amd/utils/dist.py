"""Process-group setup: one process per GPU, torchrun / mp.spawn compatible.

Backend "nccl" (= RCCL over xGMI on MI355X) when GPUs are present, "gloo" on
CPU.  MASTER_ADDR / MASTER_PORT come from the environment (defaulting to
127.0.0.1:29500) - fixing the reference's hard-coded localhost:8888, which made
``--nodes > 1`` unusable (test_apex_distributed_spawn.py:55-56).
The device is bound BEFORE the process group is created (the reference did it
after, relying on lazy NCCL init).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def get_rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else int(
        os.environ.get("RANK", "0"))


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else int(
        os.environ.get("WORLD_SIZE", "1"))


def is_main_process() -> bool:
    return get_rank() == 0


def init_distributed(backend=None, rank=None, world_size=None, local=None, timeout_s=1800,
                     device_id_binding=True):
    """Initialise torch.distributed from env:// (torchrun) or explicit args.

    Returns (rank, world_size, device)."""
    rank = int(os.environ.get("RANK", "0")) if rank is None else rank
    world_size = int(os.environ.get("WORLD_SIZE", "1")) if world_size is None else world_size
    local = local_rank() if local is None else local
    # test hooks: run every rank on one device / force the collective backend
    # (rehearsing the multi-process path on a single-GPU box)
    if os.environ.get("APEX_AMD_SINGLE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("APEX_AMD_DIST_BACKEND", backend)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    # dmabuf IPC is the only mode the MI355X host driver supports
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    use_gpu = torch.cuda.is_available() and os.environ.get("APEX_AMD_FORCE_CPU") != "1"
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if use_gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world_size > 1 and not dist.is_initialized():
        kw = dict(backend=backend, init_method="env://", world_size=world_size, rank=rank,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if use_gpu and device_id_binding and backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return rank, world_size, device


def barrier():
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def cleanup():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
