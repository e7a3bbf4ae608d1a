#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 amp O2 (bf16) training throughput, images/sec
for the whole job (BASELINE.json metric), 1..8 MI355X, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [...]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Without torchrun (WORLD_SIZE unset) and --gpus N > 1, bench.py starts the N
rank processes itself (one per GPU, child processes started BEFORE anything
touches the GPU in the parent, 127.0.0.1 rendezvous) and exits with the worst
child status.  Every rank checks that the world it joined has exactly --gpus
ranks and exits non-zero otherwise (the reference derives its process count
from --gpus the same way: test_apex_distributed_spawn.py:42,53-57).

Step = forward + loss + amp.scale_loss backward (+ bucketed RCCL all-reduce
overlapped with backward when N > 1) + FusedSGD step (momentum 0.9, wd 5e-5,
fp32 master weights, bf16 model copy written in-kernel).  Synthetic ImageNet
shaped data (224x224, 1000 classes) generated on the device per rank;
random-init weights.  W untimed warmup steps, then exactly K timed steps
bracketed by barrier + synchronize; the slowest rank's time is reported.

Other BASELINE.json configs (same harness):
  --model bert_large   BERT-large pretraining, amp O2 + FusedLAMB + FusedLayerNorm
                       (sequences/sec; seq 512, 80 masked predictions / sequence)
  --model gpt2_medium  GPT-2-medium LM, amp O1 fp16 + FusedAdam, dynamic loss
                       scaling (tokens/sec; seq 1024)

``--impl stock`` runs the same model / data / schedule on the stock
PyTorch-ROCm path (torch.autocast + torch.optim fused + torch DDP, plain
BatchNorm / LayerNorm) - the comparator of BASELINE.md section 2.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# vs_baseline: BASELINE.md publishes no number for the reference; the comparator is the
# stock PyTorch-ROCm path (bench.py --impl stock: torch.optim.SGD(fused), PyTorch
# BatchNorm, MIOpen convs, torch.autocast bf16) measured on MI355X with this same harness,
# per GPU, bs 256, at its BEST setting: round 6 re-measured it with MIOpen find mode
# (--cudnn-benchmark) - 6,540.2 img/s, and 6,538.9 with TunableOp online tuning on top -
# against 5,983-5,986 in immediate mode (rounds 1-5); this path on the same box 11,510-11,540
# (profiles/r6/stock/).
STOCK_BASELINE_PER_GPU = {"resnet50": 6540.2}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=15)
    ap.add_argument("--model", default="resnet50",
                    choices=["resnet50", "resnet18", "bert_large", "gpt2_medium", "convnet"])
    ap.add_argument("--batch-size", type=int, default=None, help="per GPU")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--impl", choices=["amd", "stock"], default="amd")
    ap.add_argument("--opt-level", default=None)
    ap.add_argument("--dtype", choices=["bf16", "fp16"], default=None)
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--no-fused-bn", action="store_true")
    ap.add_argument("--no-fused-loss", action="store_true",
                    help="transformers: torch cross entropy on fp32 logits instead of the fused kernel")
    ap.add_argument("--no-fused-attn", action="store_true",
                    help="transformers: PyTorch SDPA instead of the gfx950 attention kernels")
    ap.add_argument("--no-fused-residual-ln", action="store_true",
                    help="GPT-2: unfused residual add / dropout / LayerNorm sublayer joins")
    ap.add_argument("--syncbn", action="store_true",
                    help="SyncBatchNorm across ranks (the default for ResNet at N > 1)")
    ap.add_argument("--no-syncbn", action="store_true",
                    help="per-GPU BatchNorm statistics at N > 1 (not the BASELINE config)")
    ap.add_argument("--message-size", default="auto",
                    help="DDP bucket elements, or 'auto': at N > 1 calibrated from timed "
                         "all-reduces on the bucket communicator (power of two in [8, 64] MiB, "
                         "parallel/distributed.py, docs/DDP_TUNING.md); 32 MiB at N = 1")
    ap.add_argument("--force-collectives", action="store_true",
                    help="1 GPU: run the N>1 code path anyway - apex DDP (+ SyncBN for ResNet) "
                         "with every bucket all-reduce and SyncBN all_gather / all_reduce "
                         "issued on a 1-rank RCCL communicator (the per-GPU cost of the "
                         "multi-GPU step, measured on one GPU)")
    ap.add_argument("--materialize-master-grads", action="store_true")
    ap.add_argument("--no-gemm-1x1", action="store_true",
                    help="keep MIOpen for the stride-1 1x1 convs (default: hipBLASLt GEMM)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole training step in a hipGraph and replay it")
    ap.add_argument("--gemm-tuning", choices=["auto", "off"], default="auto",
                    help="auto: library GEMMs use the TunableOp selections in tuning/<model>.csv "
                         "(read-only, validator-checked; tools/tune_gemms.sh makes them)")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--convnet-optimizer", choices=["sgd", "fused"], default="sgd",
                    help="convnet: torch.optim.SGD as the reference program uses, or FusedSGD "
                         "(sync-free amp)")
    ap.add_argument("--deterministic", action="store_true")
    # MIOpen immediate mode measured as fast as exhaustive find for ResNet-50 on
    # MI355X (docs/PERF.md) and avoids ~200 s of solver search on a fresh box.
    ap.add_argument("--cudnn-benchmark", action="store_true",
                    help="MIOpen find (solver search) instead of immediate mode")
    ap.add_argument("--opt-step-iters", type=int, default=20)
    ap.add_argument("--pg-timeout", type=int, default=300,
                    help="process-group timeout, seconds: a collective hang at N ranks fails "
                         "within this instead of the 30-minute default")
    ap.add_argument("--rccl-channels", type=int, default=0,
                    help="cap RCCL at this many channels (NCCL_MIN/MAX_NCHANNELS; one workgroup "
                         "per channel) so bucket all-reduces leave the backward kernels their CUs; "
                         "0 = RCCL's own choice")
    ap.add_argument("--ddp-bf16-wire", choices=["rsag", "fp32", "native"], default=None,
                    help="how a bf16 DDP bucket travels: fp32 reduce-scatter + bf16 all-gather "
                         "(default), fp32 all-reduce, or native bf16 all-reduce")
    ap.add_argument("--main-stream-priority", choices=["default", "high"],
                    default=os.environ.get("APEX_AMD_MAIN_STREAM_PRIO", "default"),
                    help="high: run the training step on a high-priority HIP stream, so its "
                         "critical-path kernels win the CUs over the side-stream weight "
                         "gradients")
    ap.add_argument("--bucket-timing-steps", type=int, default=5,
                    help="N > 1: extra untimed steps with per-bucket DDP timing (0 = off)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--loss-trace", action="store_true",
                    help="keep every step's loss (device scalars, read after timing) in the JSON")
    ap.add_argument("--allow-skipped-steps", action="store_true",
                    help="do not fail when the loss scaler skipped a timed step (fp16 runs "
                         "whose dynamic scale is still settling)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch + rendezvous + world-size check only (launcher tests)")
    return ap.parse_args()


def _free_port():
    """Rendezvous port for self-spawned ranks, drawn below Linux's ephemeral range
    (32768-60999) so an outgoing connection cannot take it between this check and the
    store's bind; an ephemeral port is the fallback."""
    import random
    import socket

    rng = random.Random(os.getpid() ^ int.from_bytes(os.urandom(4), "little"))
    for _ in range(200):
        port = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", port))
            return port
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """Start ranks 0..n-1 of this same command as child processes and wait.

    Runs before any GPU call in this (parent) process: counting devices does not
    initialise HIP.  A child that fails takes the others down (they would block
    in a collective otherwise).  Returns the exit code for the parent."""
    import subprocess

    ndev = torch.cuda.device_count()
    if (ndev < n and os.environ.get("APEX_AMD_SINGLE_DEVICE") != "1"
            and os.environ.get("APEX_AMD_FORCE_CPU") != "1"):
        print("bench.py: --gpus %d but only %d GPU(s) visible" % (n, ndev), file=sys.stderr)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                   APEX_AMD_BENCH_LAUNCHER="self-spawn")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0:
                rc = rc or (code if code > 0 else 128 - code)
                for q in alive:
                    q.terminate()
        if alive:
            time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


class Workload:
    """step(batch) -> loss, opt_only(), batch, units/step/GPU, metric, unit, config."""


def build_resnet(args, device, world):
    from apex_example_amd import amp
    from apex_example_amd.models import resnet18, resnet50
    from apex_example_amd.optimizers import FusedSGD
    from apex_example_amd.parallel import DistributedDataParallel, convert_syncbn_model

    half = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    bs = args.batch_size or 256
    # lr 0.02: the synthetic task re-presents ONE random batch, on which lr 0.1 (+
    # momentum 0.9) is unstable for the stock and the fused path alike (loss 7.1 ->
    # 6.9 / 9.2 by step 25, chaotic divergence after ~12 steps); at 0.02 the two agree
    # to +-0.02 over 25 steps and fall monotonically (profiles/r2/r50_*_trace*.json).
    # Throughput does not depend on the value.
    lr = args.lr or 0.02
    opt_level = args.opt_level or "O2"
    ctor = {"resnet50": resnet50, "resnet18": resnet18}[args.model]
    fused_bn = args.impl == "amd" and not args.no_fused_bn
    gemm_1x1 = args.impl == "amd" and not args.no_gemm_1x1
    model = ctor(fused_bn=fused_bn, gemm_1x1=gemm_1x1).to(device)
    # BASELINE.json's multi-GPU ResNet-50 config is DDP + SyncBN: on by default at N > 1
    multi = world > 1 or args.force_collectives
    args.syncbn = multi and not args.no_syncbn
    if args.syncbn:
        if args.impl == "amd":
            model = convert_syncbn_model(model)
            if args.force_collectives:
                from apex_example_amd.parallel import set_syncbn_force_collectives
                set_syncbn_force_collectives(model, True)
        else:
            model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
    mf = torch.channels_last if not args.no_channels_last else torch.contiguous_format
    model = model.to(memory_format=mf)
    x = torch.randn(bs, 3, args.image_size, args.image_size, device=device).to(memory_format=mf)
    y = torch.randint(0, 1000, (bs,), device=device)
    w = Workload()
    if args.impl == "amd":
        opt = FusedSGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5,
                       materialize_master_grads=args.materialize_master_grads)
        model, opt = amp.initialize(model, opt, opt_level=opt_level, half_dtype=half,
                                    verbosity=0)
        if multi:
            model = DistributedDataParallel(model, message_size=args.message_size,
                                            force_collectives=args.force_collectives,
                                            bf16_wire=args.ddp_bf16_wire)
            w.ddp = model

        def step(b):
            out = model(b[0])
            loss = F.cross_entropy(out, b[1])
            opt.zero_grad()
            with amp.scale_loss(loss, opt) as scaled:
                scaled.backward()
            opt.step()
            return loss
    else:
        opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5,
                              fused=True)
        scaler = torch.amp.GradScaler("cuda", enabled=(half == torch.float16))
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[device.index], bucket_cap_mb=25, gradient_as_bucket_view=True)

        def step(b):
            with torch.autocast("cuda", dtype=half):
                loss = F.cross_entropy(model(b[0]), b[1])
            opt.zero_grad(set_to_none=True)
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
            return loss
    w.model, w.opt = model, opt
    w.step, w.opt_only, w.batch = step, opt.step, (x, y)
    w.units = bs
    w.metric = "images/sec (whole node) ResNet-50 amp O2" if args.model == "resnet50" else \
        "images/sec (whole node) %s amp %s" % (args.model, opt_level)
    w.unit = "images/s"
    w.dtype = "bf16" if half == torch.bfloat16 else "fp16"
    w.data = ("synthetic (on-device random 3x%dx%d images, random labels; random-init "
              "weights)" % (args.image_size, args.image_size))
    w.config = {
        "model": args.model, "global_batch": bs * world, "per_gpu_batch": bs, "seq_len": None,
        "image_size": args.image_size, "parallelism": "dp%d" % world, "impl": args.impl,
        "opt_level": opt_level,
        "optimizer": "FusedSGD(momentum=0.9, wd=5e-5)" if args.impl == "amd"
                     else "torch.optim.SGD(fused)",
        "channels_last": not args.no_channels_last, "fused_bn": fused_bn,
        "syncbn": bool(args.syncbn and multi),
        "ddp_message_size": args.message_size if multi else None,
        "force_collectives": bool(args.force_collectives),
        "gemm_1x1": gemm_1x1, "hip_graph": bool(args.graph),
    }
    return w


def build_convnet(args, device, world):
    """The reference program's own workload (test_apex_distributed_spawn.py:83-164): the
    MNIST ConvNet, batch 100 per process, SGD lr 1e-4, amp O2 with Apex's fp16 default,
    apex DDP; synthetic 1x28x28 batches on the device.  Besides images/s the record
    carries the reference's own metric, the wall time of one 60,000-image epoch."""
    from apex_example_amd import amp
    from apex_example_amd.models import ConvNet
    from apex_example_amd.optimizers import FusedSGD
    from apex_example_amd.parallel import DistributedDataParallel

    half = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    bs = args.batch_size or 100
    lr = args.lr or 1e-4
    opt_level = args.opt_level or "O2"
    multi = world > 1 or args.force_collectives
    model = ConvNet().to(device)
    x = torch.rand(bs, 1, 28, 28, device=device)
    y = torch.randint(0, 10, (bs,), device=device)
    crit = torch.nn.CrossEntropyLoss().to(device)
    w = Workload()
    if args.impl == "amd":
        if args.convnet_optimizer == "fused":
            opt = FusedSGD(model.parameters(), lr=lr, materialize_master_grads=False)
        else:
            opt = torch.optim.SGD(model.parameters(), lr)
        model, opt = amp.initialize(model, opt, opt_level=opt_level, half_dtype=half, verbosity=0)
        if multi:
            model = DistributedDataParallel(model, force_collectives=args.force_collectives)
            w.ddp = model

        def step(b):
            loss = crit(model(b[0]).float(), b[1])
            opt.zero_grad()
            with amp.scale_loss(loss, opt) as scaled:
                scaled.backward()
            opt.step()
            return loss
        optname = ("FusedSGD(lr=%g)" % lr) if args.convnet_optimizer == "fused" else \
            "torch.optim.SGD(lr=%g) (reference)" % lr
    else:
        opt = torch.optim.SGD(model.parameters(), lr)
        scaler = torch.amp.GradScaler("cuda", enabled=(half == torch.float16))
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[device.index])

        def step(b):
            with torch.autocast("cuda", dtype=half):
                loss = crit(model(b[0]).float(), b[1])
            opt.zero_grad(set_to_none=True)
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
            return loss
        optname = "torch.optim.SGD(lr=%g)" % lr
    w.model, w.opt = model, opt
    w.step, w.opt_only, w.batch = step, opt.step, (x, y)
    w.units = bs
    w.metric = "images/sec (whole node) MNIST ConvNet amp %s" % opt_level
    w.unit = "images/s"
    w.dtype = "bf16" if half == torch.bfloat16 else "fp16"
    w.data = "synthetic (on-device random 1x28x28 images, random labels; random-init weights)"
    w.steps_per_epoch = -(-60000 // (world * bs))
    w.config = {"model": "convnet", "global_batch": bs * world, "per_gpu_batch": bs,
                "seq_len": None, "image_size": 28, "parallelism": "dp%d" % world,
                "impl": args.impl, "opt_level": opt_level, "optimizer": optname,
                "force_collectives": bool(args.force_collectives)}
    return w


def build_bert(args, device, world):
    from apex_example_amd import amp
    from apex_example_amd.models.bert import (BertConfig, BertForPreTraining, pretraining_loss,
                                              synthetic_batch)
    from apex_example_amd.optimizers import FusedLAMB
    from apex_example_amd.parallel import DistributedDataParallel

    half = torch.float16 if args.dtype == "fp16" else torch.bfloat16
    bs = args.batch_size or 32
    seq = args.seq_len or 512
    max_pred = 80 if seq >= 512 else 20
    opt_level = args.opt_level or "O2"
    cfg = BertConfig(fused_layer_norm=(args.impl == "amd"),
                     fused_attention=(args.impl == "amd" and not args.no_fused_attn))
    model = BertForPreTraining(cfg).to(device)
    batch = synthetic_batch(cfg, bs, seq, max_pred, device, seed=17 + (
        dist.get_rank() if world > 1 else 0))
    w = Workload()
    if args.impl == "amd":
        opt = FusedLAMB(model.parameters(), lr=args.lr or 6e-3, weight_decay=0.01,
                        max_grad_norm=1.0, materialize_master_grads=args.materialize_master_grads)
        model, opt = amp.initialize(model, opt, opt_level=opt_level, half_dtype=half, verbosity=0)
        if world > 1 or args.force_collectives:
            model = DistributedDataParallel(model, message_size=args.message_size,
                                            force_collectives=args.force_collectives,
                                            bf16_wire=args.ddp_bf16_wire)
            w.ddp = model

        def step(b):
            mlm, nsp = model(b[0], b[1], b[2])
            loss = pretraining_loss(mlm, nsp, b[3], b[4], fused=not args.no_fused_loss)
            opt.zero_grad()
            with amp.scale_loss(loss, opt) as scaled:
                scaled.backward()
            opt.step()
            return loss
        optname = "FusedLAMB(wd=0.01, max_grad_norm=1.0)"
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=args.lr or 1e-4, weight_decay=0.01,
                                fused=True)
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[device.index])

        def step(b):
            with torch.autocast("cuda", dtype=half):
                mlm, nsp = model(b[0], b[1], b[2])
                loss = pretraining_loss(mlm, nsp, b[3], b[4], fused=False)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            return loss
        optname = "torch.optim.AdamW(fused) (torch has no LAMB)"
    w.model, w.opt = model, opt
    w.step, w.opt_only, w.batch = step, opt.step, batch
    w.units = bs
    w.metric = "sequences/sec (whole node) BERT-large pretrain amp %s" % opt_level
    w.unit = "sequences/s"
    w.dtype = "bf16" if half == torch.bfloat16 else "fp16"
    w.data = "synthetic token ids / segment ids / masked positions; random-init weights"
    w.config = {"model": "bert_large", "global_batch": bs * world, "per_gpu_batch": bs,
                "seq_len": seq, "max_predictions": max_pred, "parallelism": "dp%d" % world,
                "impl": args.impl, "opt_level": opt_level, "optimizer": optname,
                "fused_layer_norm": args.impl == "amd",
                "fused_attention": cfg.fused_attention}
    return w


def build_gpt2(args, device, world):
    from apex_example_amd import amp
    from apex_example_amd.models.gpt2 import GPT2Config, GPT2LMHeadModel, lm_loss
    from apex_example_amd.optimizers import FusedAdam
    from apex_example_amd.parallel import DistributedDataParallel

    half = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    bs = args.batch_size or 8
    seq = args.seq_len or 1024
    opt_level = args.opt_level or "O1"
    cfg = GPT2Config(fused_layer_norm=(args.impl == "amd"),
                     fused_attention=(args.impl == "amd" and not args.no_fused_attn),
                     fused_residual_ln=(args.impl == "amd" and not args.no_fused_residual_ln))
    model = GPT2LMHeadModel(cfg).to(device)
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, cfg.vocab_size, (bs, seq), generator=g).to(device)
    w = Workload()
    if args.impl == "amd":
        # materialize_master_grads=False: the O1 unscale is folded into FusedAdam
        # (read-only overflow check instead of an in-place pass over every grad)
        opt = FusedAdam(model.parameters(), lr=args.lr or 1.5e-4, weight_decay=0.01,
                        materialize_master_grads=args.materialize_master_grads)
        model, opt = amp.initialize(model, opt, opt_level=opt_level, half_dtype=half, verbosity=0)
        if world > 1 or args.force_collectives:
            model = DistributedDataParallel(model, message_size=args.message_size,
                                            force_collectives=args.force_collectives,
                                            bf16_wire=args.ddp_bf16_wire)
            w.ddp = model

        def step(b):
            loss = lm_loss(model(b[0]), b[0], fused=not args.no_fused_loss)
            opt.zero_grad()
            with amp.scale_loss(loss, opt) as scaled:
                scaled.backward()
            opt.step()
            return loss
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=args.lr or 1.5e-4, weight_decay=0.01,
                                fused=True)
        scaler = torch.amp.GradScaler("cuda", enabled=(half == torch.float16))
        if world > 1:
            model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[device.index])

        def step(b):
            with torch.autocast("cuda", dtype=half):
                loss = lm_loss(model(b[0]), b[0], fused=False)
            opt.zero_grad(set_to_none=True)
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
            return loss
    w.model, w.opt = model, opt
    w.step, w.opt_only, w.batch = step, opt.step, (ids,)
    w.units = bs * seq
    w.metric = "tokens/sec (whole node) GPT-2-medium amp %s" % opt_level
    w.unit = "tokens/s"
    w.dtype = "bf16" if half == torch.bfloat16 else "fp16"
    w.data = "synthetic token ids; random-init weights"
    w.config = {"model": "gpt2_medium", "global_batch": bs * world, "per_gpu_batch": bs,
                "seq_len": seq, "parallelism": "dp%d" % world, "impl": args.impl,
                "opt_level": opt_level,
                "optimizer": "FusedAdam(wd=0.01)" if args.impl == "amd"
                             else "torch.optim.AdamW(fused)",
                "fused_layer_norm": args.impl == "amd",
                "fused_attention": cfg.fused_attention}
    return w


def _bucket_comm(ddp, b, pg):
    """One bucket's collective(s) in the DDP's wire format (comm-only timing)."""
    mode = ddp._fp32_mode()
    if b.dtype == torch.bfloat16 and mode == 3:
        cb = b.float()
        n = dist.get_world_size(pg)
        shard = torch.empty(cb.numel() // n, dtype=torch.float32, device=cb.device)
        dist.reduce_scatter_tensor(shard, cb, group=pg)
        mine = b.view(n, -1)[dist.get_rank(pg)]
        mine.copy_(shard)
        dist.all_gather_into_tensor(b, mine, group=pg)
        return
    up = b.dtype != torch.float32 and (mode == 1 or (mode == 2 and b.dtype == torch.bfloat16))
    dist.all_reduce(b.float() if up else b, group=pg)


def ddp_timing(ddp, step, batch, steps, device):
    """Per-bucket DDP timing over a few extra (untimed) steps: when each bucket's
    collective was launched during backward, the exposed post-backward tail
    (end of backward -> every collective joined), the same buckets reduced back to
    back with nothing else running (the comm-only cost the overlap has to hide), and
    what the SyncBN collectives cost the compute stream.  Max over ranks."""
    from apex_example_amd.ops import batch_norm as bnmod

    ddp.enable_bucket_timing(True)
    tails, bwd, launches = [], [], None
    sbn_ms, sbn_calls = [], []
    for _ in range(steps):
        bnmod.syncbn_timing(True)
        step(batch)
        sb = bnmod.syncbn_timing_result()
        bnmod.syncbn_timing(False)
        if sb is not None:
            sbn_ms.append(sb["ms"])
            sbn_calls.append(sb["calls"])
        t = ddp.bucket_timing()
        if t is None:
            continue
        tails.append(t["exposed_tail_ms"])
        bwd.append(t["backward_ms"])
        launches = t["launch_ms"]
        numels = t["bucket_numel"]
    ddp.enable_bucket_timing(False)
    if not tails:
        return None
    bufs = ddp.allreduce_buffers
    pg = ddp._comm_pg
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    for i in range(reps + 1):
        if i == 1:
            e0.record()
        for b in bufs:
            _bucket_comm(ddp, b, pg)
    e1.record()
    torch.cuda.synchronize()
    comm_ms = e0.elapsed_time(e1) / reps
    ddp.zero_grad_buckets()  # the buckets above were summed, not averaged
    sbn = sum(sbn_ms) / len(sbn_ms) if sbn_ms else 0.0
    v = torch.tensor([sum(tails) / len(tails), sum(bwd) / len(bwd), comm_ms, sbn],
                     dtype=torch.float64, device=device)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    tail, bw, comm, sbn = [float(x) for x in v.tolist()]
    rec = {
        "buckets": len(numels),
        "bucket_mb": [round(n * bufs[i].element_size() / 2**20, 2) for i, n in enumerate(numels)],
        "message_size": ddp.message_size,
        "calibration": ddp.calibration,
        "wire": ddp.wire_format(),
        "allreduce_fp32_accumulate_bf16": ddp._fp32_mode() in (2, 3),
        "high_priority_streams": ddp.high_priority_streams,
        "rccl_channels": os.environ.get("NCCL_MAX_NCHANNELS", "rccl default"),
        "backward_ms": round(bw, 3),
        "exposed_tail_ms": round(tail, 3),
        "comm_only_ms": round(comm, 3),
        "launch_ms": [round(x, 3) for x in launches],
        "timing_steps": len(tails),
    }
    if sbn_ms:
        # HIP-event time of the SyncBN all_gather (+ combine) / all_reduce calls on the
        # compute stream per step, including waiting for the slowest peer
        rec["syncbn_ms_per_step"] = round(sbn, 3)
        rec["syncbn_calls"] = int(max(sbn_calls))
    return rec


def main():
    args = parse()
    if args.message_size != "auto":
        args.message_size = int(args.message_size)
    from apex_example_amd.utils.dist import barrier, init_distributed

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if args.rccl_channels > 0:
        # read by RCCL when a communicator is created (before any process group exists)
        os.environ["NCCL_MIN_NCHANNELS"] = str(args.rccl_channels)
        os.environ["NCCL_MAX_NCHANNELS"] = str(args.rccl_channels)
    rank, world, device = init_distributed(timeout_s=args.pg_timeout)
    if args.force_collectives and world == 1 and args.impl == "amd":
        # a 1-rank process group (RCCL on the GPU) for the forced collectives
        import datetime
        os.environ["MASTER_PORT"] = str(_free_port())
        kw = {"device_id": device} if device.type == "cuda" else {}
        dist.init_process_group("nccl" if device.type == "cuda" else "gloo", rank=0,
                                world_size=1, timeout=datetime.timedelta(seconds=args.pg_timeout),
                                **kw)
    if world != args.gpus:
        print("bench.py: --gpus %d but the job has %d rank(s) (WORLD_SIZE=%s); refusing to "
              "report a number for the wrong world size" % (args.gpus, world,
                                                           os.environ.get("WORLD_SIZE")),
              file=sys.stderr)
        sys.exit(3)
    if args.dry_run:
        if world > 1:
            barrier()
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "backend":
                              dist.get_backend() if world > 1 else None,
                              "launcher": os.environ.get("APEX_AMD_BENCH_LAUNCHER", "single")}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    torch.backends.cudnn.benchmark = (not args.deterministic) and args.cudnn_benchmark
    torch.backends.cudnn.deterministic = args.deterministic
    if args.deterministic:
        from apex_example_amd.utils import set_deterministic
        set_deterministic(True)
    torch.manual_seed(1234 + rank)
    gemm_table = None
    if args.gemm_tuning == "auto" and not os.environ.get("PYTORCH_TUNABLEOP_ENABLED"):
        from apex_example_amd.utils.gemm_tuning import use_tuned_gemms
        gemm_table = use_tuned_gemms(args.model)

    if args.model.startswith("resnet"):
        w = build_resnet(args, device, world)
    elif args.model == "convnet":
        w = build_convnet(args, device, world)
    elif args.model == "bert_large":
        w = build_bert(args, device, world)
    else:
        w = build_gpt2(args, device, world)
    step, batch = w.step, w.batch
    if args.main_stream_priority == "high" and device.type == "cuda":
        hp = torch.cuda.Stream(device, priority=torch.cuda.Stream.priority_range()[1])
        hp.wait_stream(torch.cuda.current_stream())
        torch.cuda.set_stream(hp)  # every later launch of this thread goes to it
    w.config["main_stream_priority"] = args.main_stream_priority

    log(rank, "[bench] impl=%s model=%s units/gpu/step=%d world=%d warmup=%d steps=%d" % (
        args.impl, args.model, w.units, world, args.warmup, args.steps))
    t0 = time.time()
    loss = None
    trace = [] if args.loss_trace else None
    for i in range(args.warmup):
        loss = step(batch)
        if trace is not None:
            trace.append(loss.detach())
        if i == 0 or (i + 1) % 5 == 0:
            torch.cuda.synchronize()
            log(rank, "[bench] warmup %d/%d loss %.4f (%.1fs)" % (i + 1, args.warmup, loss.item(),
                                                              time.time() - t0))
    torch.cuda.synchronize()

    if args.graph:
        if world > 1:
            raise SystemExit("--graph is single-GPU only in this version")
        # drop every reference to an eager autograd graph (its AccumulateGrad
        # nodes would pin the default stream), then warm the capture path on a
        # side stream (allocator pools, multi-tensor plan caches)
        del loss
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                step(batch)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static_loss = step(batch)
        torch.cuda.synchronize()
        log(rank, "[bench] captured the training step in a hipGraph")

        def step(b):  # noqa: F811  (replay: same work, one launch)
            graph.replay()
            return static_loss

        step(batch)
        torch.cuda.synchronize()

    def sync_all():
        if world > 1:
            barrier()
        torch.cuda.synchronize()

    sync_all()
    skipped_before = _skipped_steps(args)
    torch.cuda.nvtx.range_push("timed_steps")
    t_start = time.perf_counter()
    for _ in range(args.steps):
        loss = step(batch)
        if trace is not None:
            trace.append(loss.detach().clone())
    sync_all()
    torch.cuda.nvtx.range_pop()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())
    # outside the timed region: how many timed steps did the loss scaler skip?
    # (a step whose grads overflowed trains nothing; the rate would be a lie)
    skipped_after = _skipped_steps(args)
    skipped = (skipped_after - skipped_before) if skipped_before is not None else None
    if world > 1 and skipped is not None:
        t = torch.tensor([skipped], dtype=torch.int64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        skipped = int(t.item())
    scale_now = _loss_scale(args)

    # optimizer step alone (secondary metric of BASELINE.json)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    h0 = time.perf_counter()
    for _ in range(args.opt_step_iters):
        w.opt_only()
    opt_host_ms = (time.perf_counter() - h0) * 1e3 / args.opt_step_iters  # launch side only
    e1.record()
    torch.cuda.synchronize()
    opt_ms = e0.elapsed_time(e1) / args.opt_step_iters

    ddp_stats = None
    ddp = getattr(w, "ddp", None)
    if ((world > 1 or args.force_collectives) and ddp is not None
            and args.bucket_timing_steps > 0):
        ddp_stats = ddp_timing(ddp, step, batch, args.bucket_timing_steps, device)

    consistency = replica_check(w, args, world) if world > 1 else None

    ms_per_step = elapsed / args.steps * 1e3
    value = w.units * world * args.steps / elapsed
    base = STOCK_BASELINE_PER_GPU.get(args.model) if args.impl == "amd" else None
    if args.model.startswith("resnet") and (w.config.get("per_gpu_batch") != 256
                                            or args.image_size != 224):
        base = None
    w.config["deterministic"] = bool(args.deterministic)
    if ddp is not None:
        w.config["ddp_wire"] = ddp.wire_format()
        w.config["rccl_channels"] = args.rccl_channels or "rccl default"
        w.config["pg_timeout_s"] = args.pg_timeout
    w.config["gemm_tuning"] = (os.path.relpath(gemm_table, ROOT) if gemm_table else
                               "env" if os.environ.get("PYTORCH_TUNABLEOP_ENABLED") else None)
    rec = {
        "metric": w.metric,
        "value": round(value, 2),
        "unit": w.unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (base * world), 4) if base else None,
        "dtype": w.dtype,
        "data": w.data,
        "config": w.config,
        "optimizer_step_ms": round(opt_ms, 4),
        "optimizer_step_host_ms": round(opt_host_ms, 4),
        "final_loss": round(final_loss, 4),
        "skipped_steps": skipped,
        "loss_scale": scale_now,
        "launcher": os.environ.get("APEX_AMD_BENCH_LAUNCHER",
                                   "torchrun" if world > 1 else "single"),
    }
    if ddp_stats is not None:
        rec["ddp"] = ddp_stats
    if consistency is not None:
        rec["replicas"] = consistency
    if getattr(w, "steps_per_epoch", None):
        # the reference program's metric: "Training complete in" / epochs
        rec["epoch_seconds"] = round(w.steps_per_epoch * ms_per_step / 1e3, 3)
    if trace is not None:
        rec["loss_trace"] = [round(float(v), 4) for v in trace]
    if rank == 0:
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        barrier()
    if dist.is_initialized():
        dist.destroy_process_group()
    if consistency is not None and not consistency["in_sync"]:
        print("bench.py: the %d replicas are NOT bitwise in sync after the timed steps: %s; "
              "the throughput above does not measure data-parallel training" % (
                  world, {k: v["match"] for k, v in consistency["digests"].items()}),
              file=sys.stderr)
        sys.exit(5)
    if skipped and not args.allow_skipped_steps:
        print("bench.py: %d of the %d timed steps were skipped by the loss scaler (gradient "
              "overflow); the throughput above does not measure training steps" % (
                  skipped, args.steps), file=sys.stderr)
        sys.exit(4)


def replica_check(w, args, world):
    """N > 1, after the timed region: what the collectives really span (the rank count
    each RCCL communicator reports) and whether the replicas are still bitwise equal
    (cross-rank MAX / MIN of per-rank digests of parameters, amp master weights,
    optimizer state and buffers; apex_example_amd/utils/consistency.py).  BatchNorm
    running statistics differ legitimately without SyncBN, so buffers only count when
    SyncBN is on or the model has no BatchNorm."""
    from apex_example_amd.utils.consistency import (comm_info, cross_rank_match,
                                                    model_state_groups)

    if os.environ.get("APEX_AMD_TEST_DESYNC_RANK") == str(dist.get_rank()):
        # test hook (tests/test_ddp_gpu.py): flip the lowest bit of one weight on one rank
        with torch.no_grad():
            p = next(iter(w.model.parameters())).detach()
            p = p.as_strided((1,), (1,), p.storage_offset())
            p.view({2: torch.int16, 4: torch.int32}[p.element_size()]).add_(1)
    comms = {"world": comm_info(dist.group.WORLD)}
    ddp = getattr(w, "ddp", None)
    if ddp is not None:
        comms["ddp"] = comm_info(getattr(ddp, "_comm_pg", None) or dist.group.WORLD)
    if args.impl == "amd" and w.config.get("syncbn"):
        from apex_example_amd.parallel.sync_batchnorm import syncbn_comm_group
        comms["syncbn"] = comm_info(syncbn_comm_group())
    model = w.model.module if hasattr(w.model, "module") else w.model
    groups = model_state_groups(model, w.opt)
    digests = cross_rank_match(groups)
    has_bn = any(isinstance(m, torch.nn.modules.batchnorm._BatchNorm) for m in model.modules())
    required = [k for k in digests if k != "buffers" or w.config.get("syncbn") or not has_bn]
    in_sync = all(digests[k]["match"] for k in required)
    sizes_ok = all(c is None or c["size"] == world for c in comms.values())
    return {"in_sync": bool(in_sync and sizes_ok), "required": required,
            "digests": digests, "comms": comms, "comm_sizes_ok": sizes_ok}


def _amp_scalers(args):
    if args.impl != "amd":
        return []
    from apex_example_amd.amp._amp_state import _amp_state
    return list(getattr(_amp_state, "loss_scalers", None) or [])


def _skipped_steps(args):
    """Total skipped steps of every amp loss scaler (one device read; called
    only outside the timed region).  None for the stock comparator."""
    if args.impl == "amd":
        return sum(sc.skipped_steps() for sc in _amp_scalers(args))
    return None


def _loss_scale(args):
    sc = _amp_scalers(args)
    return float(sc[0].loss_scale()) if sc else None


if __name__ == "__main__":
    main()
