#!/usr/bin/env python3
"""Reference-parity driver: the MNIST ConvNet trained with amp + apex-style DDP,
one process per GPU via ``mp.spawn`` (test_apex_distributed_spawn.py:35-174,
SURVEY.md R-01..R-19), on this framework.

    python examples/spawn_train.py --gpus 8 --apex_opt_level O2 --epochs 10
    python examples/spawn_train.py --gpus 2 --apex_enabled false   # torch DDP path

Same CLI (``--nodes --gpus --nr --apex_enabled --apex_opt_level --epochs
--batch_size``), same model, optimizer (SGD lr 1e-4), sampler, logging lines
("Epoch [e/E], Step [s/S], Loss: x" every 100 steps, "Training complete in:").
Fixed quirks of the original, each noted where it happens:
  * ``--apex_enabled`` parses booleans properly (R-04: ``type=bool``);
  * MASTER_ADDR / MASTER_PORT come from the environment when set (P-04),
    defaulting to 127.0.0.1:8888;
  * the device is bound before the process group is created (R-06);
  * ``DistributedSampler.set_epoch`` is called every epoch (R-15);
  * logging happens on global rank 0, not every node's local GPU 0 (R-19).
Data: :class:`SyntheticMNIST` (no network for torchvision downloads) unless
``--data mnist`` points at an existing torchvision MNIST directory.
Without GPUs the workers run on the CPU with the gloo backend (O0/O2 bf16 on
the C++ CPU kernels), so the whole flow is testable anywhere.
"""
from __future__ import annotations

import argparse
import os
import sys
from datetime import datetime

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from apex_example_amd import amp  # noqa: E402
from apex_example_amd.models import ConvNet  # noqa: E402
from apex_example_amd.parallel import DistributedDataParallel  # noqa: E402
from apex_example_amd.utils import set_cuda, set_seed  # noqa: E402
from apex_example_amd.utils.data import SyntheticMNIST, str2bool  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--nodes", default=1, type=int, metavar="N", help="number of nodes")
    p.add_argument("--gpus", default=4, type=int, help="processes (GPUs) per node")
    p.add_argument("--nr", default=0, type=int, help="rank of this node among the nodes")
    p.add_argument("--apex_enabled", default=True, type=str2bool, help="use amp + apex DDP")
    p.add_argument("--apex_opt_level", default="O2", type=str,
                   help="amp optimization level (O0, O1, O2, O3)")
    p.add_argument("--half_dtype", default=None, choices=[None, "fp16", "bf16"],
                   help="16-bit type for O1-O3 (default fp16 on GPU, bf16 on CPU)")
    p.add_argument("--epochs", default=10, type=int, metavar="N")
    p.add_argument("--batch_size", default=100, type=int, metavar="N")
    p.add_argument("--lr", default=1e-4, type=float)
    p.add_argument("--data", default="synthetic", help="'synthetic' or a torchvision MNIST root")
    p.add_argument("--dataset_size", default=60000, type=int, help="synthetic dataset length")
    p.add_argument("--log_every", default=100, type=int)
    p.add_argument("--deterministic", default=True, type=str2bool)
    p.add_argument("--cpu", action="store_true", help="force CPU workers (gloo)")
    p.add_argument("--result_file", default=None, help="rank 0 writes final loss/time here")
    return p.parse_args(argv)


def spawn_workers(args):
    args.world_size = args.gpus * args.nodes
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "8888")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    mp.spawn(train, nprocs=args.gpus, args=(args,))


def _dataset(args):
    if args.data == "synthetic":
        return SyntheticMNIST(n=args.dataset_size)
    import torchvision  # only when real data was requested
    import torchvision.transforms as transforms

    return torchvision.datasets.MNIST(root=args.data, train=True,
                                      transform=transforms.ToTensor(), download=False)


def train(gpu, args):
    use_gpu = torch.cuda.is_available() and not args.cpu
    rank = args.nr * args.gpus + gpu
    if use_gpu:
        torch.cuda.set_device(gpu)
        device = torch.device("cuda", gpu)
        backend = "nccl"
    else:
        device = torch.device("cpu")
        backend = "gloo"
        torch.set_num_threads(max(1, (os.cpu_count() or 2) // max(args.gpus, 1)))
    dist.init_process_group(backend=backend, init_method="env://", world_size=args.world_size,
                            rank=rank)
    set_cuda(deterministic=args.deterministic)
    set_seed(0)

    model = ConvNet().to(device)
    optimizer = torch.optim.SGD(model.parameters(), args.lr)
    if args.apex_enabled:
        half = args.half_dtype or ("fp16" if use_gpu else "bf16")
        model, optimizer = amp.initialize(
            model, optimizer, opt_level=args.apex_opt_level,
            half_dtype=torch.float16 if half == "fp16" else torch.bfloat16,
            verbosity=1 if rank == 0 else 0)
        model = DistributedDataParallel(model)
    else:
        model = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[gpu] if use_gpu else None)

    dataset = _dataset(args)
    sampler = torch.utils.data.distributed.DistributedSampler(dataset,
                                                              num_replicas=args.world_size,
                                                              rank=rank)
    loader = torch.utils.data.DataLoader(dataset, batch_size=args.batch_size, shuffle=False,
                                         num_workers=0, pin_memory=use_gpu, sampler=sampler)

    criterion = nn.CrossEntropyLoss().to(device)
    start = datetime.now()
    total_step = len(loader)
    loss = None
    first_loss = None
    for epoch in range(args.epochs):
        sampler.set_epoch(epoch)
        for i, (images, labels) in enumerate(loader):
            images = images.to(device, non_blocking=True)
            labels = labels.to(device, non_blocking=True)
            outputs = model(images)
            loss = criterion(outputs.float(), labels)
            optimizer.zero_grad()
            if args.apex_enabled:
                with amp.scale_loss(loss, optimizer) as scaled_loss:
                    scaled_loss.backward()
            else:
                loss.backward()
            optimizer.step()
            if first_loss is None:
                first_loss = loss.item()
            if (i + 1) % args.log_every == 0 and rank == 0:
                print(f"Epoch [{epoch + 1}/{args.epochs}], Step [{i + 1}/{total_step}], "
                      f"Loss: {loss.item():.4f}", flush=True)
    if rank == 0:
        elapsed = datetime.now() - start
        print(f"Training complete in: {elapsed}", flush=True)
        if args.result_file:
            import json

            with open(args.result_file, "w") as f:
                json.dump({"first_loss": first_loss, "final_loss": loss.item(),
                           "seconds": elapsed.total_seconds(), "world_size": args.world_size,
                           "steps_per_epoch": total_step}, f)
    dist.barrier()
    dist.destroy_process_group()


def main(argv=None):
    spawn_workers(parse_args(argv))


if __name__ == "__main__":
    main()
