"""Worker functions for the multi-process (gloo, CPU) distributed tests.

Each worker initialises torch.distributed on 127.0.0.1, runs one scenario and
writes its results with torch.save to <out>/rank<r>.pt (files this test suite
writes itself)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F


def free_port():
    """A port for a child process's TCP rendezvous, drawn below Linux's ephemeral range
    (32768-60999): a port the kernel hands out as ephemeral (bind to 0) can be taken by
    any outgoing connection on a shared box between this check and the child's bind
    (EADDRINUSE seen on a GPU box)."""
    import random

    rng = random.Random(os.getpid() ^ int.from_bytes(os.urandom(4), "little"))
    for _ in range(200):
        p = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, rdzv, fn_name, out, kw):
    # file rendezvous: a port picked by free_port() can be taken by another process on a
    # shared box between the pick and the child's bind (EADDRINUSE seen on a GPU box)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method="file://" + rdzv, rank=rank, world_size=world)
    try:
        res = globals()[fn_name](rank, world, **kw)
        torch.save(res, os.path.join(out, "rank%d.pt" % rank))
        dist.barrier()  # only on success: a failing rank exits and mp.spawn stops the rest
    finally:
        dist.destroy_process_group()


def run(fn_name, world, out, **kw):
    rdzv = os.path.join(out, "rdzv_%s_%d" % (fn_name, os.getpid()))
    if os.path.exists(rdzv):
        os.remove(rdzv)
    mp.spawn(_entry, args=(world, rdzv, fn_name, out, kw), nprocs=world, join=True)
    return [torch.load(os.path.join(out, "rank%d.pt" % r), weights_only=False)
            for r in range(world)]


def _mlp():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 32), nn.ReLU(),
                         nn.Linear(32, 4))


def _data(n=8, seed=123):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 16, generator=g), torch.randint(0, 4, (n,), generator=g)


# ---------------------------------------------------------------------- DDP
def ddp_grads(rank, world, message_size=10_000_000, delay=False, predivide=1.0, average=True,
              fp32=False, iters=2, streams=1):
    from apex_example_amd.parallel import DistributedDataParallel

    model = _mlp()
    if rank == 1:  # different init on rank 1: DDP must broadcast rank 0's params
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    ddp = DistributedDataParallel(model, message_size=message_size, delay_allreduce=delay,
                                  gradient_predivide_factor=predivide, gradient_average=average,
                                  allreduce_always_fp32=fp32, num_allreduce_streams=streams)
    x, y = _data(8 * world)
    xs, ys = x.chunk(world)[rank], y.chunk(world)[rank]
    out = {}
    for it in range(iters):
        for p in model.parameters():
            if p.grad is not None:
                p.grad.zero_()
        loss = F.cross_entropy(ddp(xs), ys)
        loss.backward()
        out["grads%d" % it] = [p.grad.detach().clone() for p in model.parameters()]
    out["params"] = [p.detach().clone() for p in model.parameters()]
    out["layout"] = ddp.bucket_layout()
    out["views"] = all(getattr(p, "_amd_grad_is_bucket_view", False) for p in model.parameters())
    return out


def ddp_subgroups(rank, world, streams=1, message_size=300):
    """Two disjoint data-parallel subgroups {0,1} and {2,3}: every rank creates both
    groups (in the same order), then only the members of a group construct the DDP
    over it.  Each subgroup averages over its own 2 ranks' data."""
    from apex_example_amd.parallel import DistributedDataParallel

    groups = [dist.new_group(ranks=[0, 1]), dist.new_group(ranks=[2, 3])]
    mine = groups[rank // 2]
    model = _mlp()
    ddp = DistributedDataParallel(model, message_size=message_size, process_group=mine,
                                  num_allreduce_streams=streams)
    x, y = _data(16, seed=200 + rank // 2)   # subgroup-specific batch
    xs, ys = x.chunk(2)[rank % 2], y.chunk(2)[rank % 2]
    out = {}
    for it in range(2):
        for p in model.parameters():
            p.grad = None if it == 0 else p.grad.zero_()
        F.cross_entropy(ddp(xs), ys).backward()
        out["grads%d" % it] = [p.grad.detach().clone() for p in model.parameters()]
    return out


def ddp_auto_size(rank, world):
    """message_size='auto': 32 MiB on the wire for the dtype the collective moves
    (the sizing rule alone: calibration off)."""
    from apex_example_amd.parallel import DistributedDataParallel

    os.environ["APEX_AMD_DDP_CALIBRATE"] = "0"
    out = {}
    for name, dt, fp32 in (("bf16", torch.bfloat16, None), ("bf16_native", torch.bfloat16, False),
                           ("fp16", torch.float16, None), ("fp32", torch.float32, None)):
        m = nn.Linear(64, 64).to(dt)
        ddp = DistributedDataParallel(m, message_size="auto", allreduce_always_fp32=fp32)
        out[name] = ddp.message_size
    return out


def ddp_calibrate(rank, world):
    """message_size='auto' at world > 1: the bucket size comes from a measured
    all-reduce fit, identical on every rank."""
    from apex_example_amd.parallel import DistributedDataParallel

    os.environ.pop("APEX_AMD_DDP_CALIBRATE", None)
    m = nn.Linear(64, 64)
    ddp = DistributedDataParallel(m, message_size="auto")
    x = torch.randn(4, 64)
    ddp(x).sum().backward()  # the reducer still works after the calibration collectives
    return {"cal": ddp.calibration, "message_size": ddp.message_size,
            "grad": m.weight.grad.clone()}


def ddp_retain_buffers(rank, world):
    """retain_allreduce_buffers=True (Apex): the all-reduced flat buffers stay
    accessible as ``allreduce_buffers`` after backward - here every .grad is a view
    into them."""
    from apex_example_amd.parallel import DistributedDataParallel

    model = _mlp()
    ddp = DistributedDataParallel(model, message_size=700, retain_allreduce_buffers=True)
    x, y = _data(8 * world)
    xs, ys = x.chunk(world)[rank], y.chunk(world)[rank]
    F.cross_entropy(ddp(xs), ys).backward()
    bufs = ddp.allreduce_buffers
    spans = [(b.data_ptr(), b.data_ptr() + b.numel() * b.element_size()) for b in bufs]
    inside = [any(lo <= p.grad.data_ptr() < hi for lo, hi in spans) for p in model.parameters()]
    total = sum(b.numel() for b in bufs)
    return {"n_bufs": len(bufs), "inside": inside, "total": total,
            "n_params": sum(p.numel() for p in model.parameters()),
            "buf_sum": float(sum(b.double().sum() for b in bufs)),
            "grad_sum": float(sum(p.grad.double().sum() for p in model.parameters()))}


def ddp_bf16_precision(rank, world, fp32=None, n=4096):
    """bf16 gradient buckets averaged over ``world`` ranks; returns the reduced
    bf16 gradient and the exact fp32 average of the per-rank bf16 gradients."""
    from apex_example_amd.parallel import DistributedDataParallel

    p = nn.Parameter(torch.ones(n, dtype=torch.bfloat16))
    mod = nn.Module()
    mod.p = p
    mod.forward = lambda c: (mod.p.float() * c).sum()
    ddp = DistributedDataParallel(mod, allreduce_always_fp32=fp32)
    cs = [torch.randn(n, generator=torch.Generator().manual_seed(100 + r)) *
          (1.0 + 0.37 * r) for r in range(world)]
    bf = [c.to(torch.bfloat16).float() for c in cs]
    ddp(cs[rank]).backward()
    exact = sum(bf) / world
    return {"grad": p.grad.float().clone(), "exact": exact}


def ddp_bf16_wire(rank, world, wire="rsag", n=4099, message_size=1000, iters=2):
    """bf16 buckets (sizes not multiples of world x alignment) reduced through the given
    wire format; returns every iteration's reduced gradients and the exact fp64 average
    of the per-rank bf16 gradients."""
    from apex_example_amd.parallel import DistributedDataParallel

    sizes = [n, n + 13, 2 * n + 7]
    mod = nn.Module()
    mod.ps = nn.ParameterList([nn.Parameter(torch.ones(k, dtype=torch.bfloat16)) for k in sizes])
    mod.forward = lambda cs: sum((p.float() * c).sum() for p, c in zip(mod.ps, cs))
    ddp = DistributedDataParallel(mod, bf16_wire=wire, message_size=message_size)
    out, exact = [], []
    for it in range(iters):
        cs = [[torch.randn(k, generator=torch.Generator().manual_seed(1000 * it + 10 * r + j))
               * (1.0 + 0.37 * r) for j, k in enumerate(sizes)] for r in range(world)]
        for p in mod.ps:
            if p.grad is not None:
                p.grad.zero_()
        ddp(cs[rank]).backward()
        out.append([p.grad.float().clone() for p in mod.ps])
        exact.append([sum(cs[r][j].to(torch.bfloat16).double() for r in range(world)) / world
                      for j in range(len(sizes))])
    return {"grads": out, "exact": exact, "wire": ddp.wire_format(),
            "mode": ddp._fp32_mode()}


class _DirectMul(torch.autograd.Function):
    """y = x * w whose weight gradient goes the own ops' direct way when DDP allows it
    (accumulated into the bucket view + announced; autograd gets None)."""
    DIRECT = [0]

    @staticmethod
    def forward(ctx, x, w):
        from apex_example_amd.ops import _ddp_direct

        ctx.save_for_backward(x, w)
        ctx.w = w
        if ctx.needs_input_grad[1]:
            _ddp_direct.note_use(w)
        return x * w

    @staticmethod
    def backward(ctx, g):
        from apex_example_amd.ops import _ddp_direct

        x, w = ctx.saved_tensors
        gw = (g * x).sum(0)
        sl = _ddp_direct.slots(ctx.w)
        if sl is not None:
            with torch.no_grad():
                ctx.w.grad.add_(gw)
            _ddp_direct.mark_ready(sl)
            _DirectMul.DIRECT[0] += 1
            gw = None
        return g * w, gw


class _DirectNet(nn.Module):
    def __init__(self, case):
        super().__init__()
        self.case = case
        self.a = nn.Parameter(torch.linspace(0.5, 1.5, 8))
        self.b = nn.Parameter(torch.linspace(-1.0, 1.0, 8))
        self.c = nn.Parameter(torch.linspace(2.0, 3.0, 8))   # always used once
        if case == "tied":
            self.sub = nn.Module()
            self.sub.w = self.a                                  # a listed twice

    def forward(self, x):
        h = _DirectMul.apply(x, self.c)
        if self.case == "twice":       # one module's weight used twice in a forward
            h = _DirectMul.apply(_DirectMul.apply(h, self.a), self.a)
        elif self.case == "tied":      # tied weight: used through both names
            h = _DirectMul.apply(_DirectMul.apply(h, self.a), self.sub.w)
        elif self.case == "plain":     # every weight used once per forward
            h = _DirectMul.apply(h, self.a)
        else:                          # "functional": a direct use + a plain autograd use
            h = _DirectMul.apply(h, self.a) + h * self.a
        return (_DirectMul.apply(h, self.b) ** 2).sum()


def ddp_direct_shared(rank, world, case="twice", iters=3, two_forwards=False):
    """Shared / multiply-used parameters on the direct-gradient path: grads
    must equal the full-batch autograd reference, or (functional use after a launched
    bucket) the reducer raises its explicit error; the parameter is then excluded."""
    from apex_example_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    net = _DirectNet(case)
    ref = _DirectNet(case)
    ref.load_state_dict(net.state_dict())
    ddp = DistributedDataParallel(net, message_size=1)  # one bucket per parameter
    _DirectMul.DIRECT[0] = 0
    out, refs, err = [], [], None
    for it in range(iters):
        xs = [torch.randn(4, 8, generator=torch.Generator().manual_seed(50 * it + r))
              for r in range(world)]
        for p in net.parameters():  # (bucket views: zeroed in place)
            if p.grad is not None:
                p.grad.zero_()
        try:
            if two_forwards:  # siamese / contrastive: two DDP forwards, one backward
                (ddp(xs[rank]) + ddp(2.0 * xs[rank])).backward()
            else:
                ddp(xs[rank]).backward()
        except RuntimeError as e:
            err = str(e)
            break
        out.append({k: v.grad.clone() for k, v in net.named_parameters()})
        if two_forwards:
            loss = sum(ref(x) + ref(2.0 * x) for x in xs) / world
        else:
            loss = sum(ref(x) for x in xs) / world
        ref.zero_grad()
        loss.backward()
        refs.append({k: v.grad.clone() for k, v in ref.named_parameters()})
    red = ddp.reducer
    idx = {id(p): i for i, p in enumerate(ddp.active_params)}
    return {"grads": out, "refs": refs, "err": err, "direct": _DirectMul.DIRECT[0],
            "direct_ok": {k: bool(red.direct_ok(idx[id(p)])) for k, p in net.named_parameters()}}


def ddp_layout(rank, world, tapered=True, message_size=4000):
    """Bucket layout (in launch order) and numels of a chain of linear layers whose
    gradients arrive last-layer first, plus the gradients of one backward."""
    from apex_example_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    layers = [nn.Linear(32, 32) for _ in range(12)]
    net = nn.Sequential(*layers)
    ddp = DistributedDataParallel(net, message_size=message_size, tapered_buckets=tapered)
    x = torch.randn(4, 32, generator=torch.Generator().manual_seed(rank))
    for _ in range(2):  # iteration 1 records the arrival order, 2 runs the new layout
        for p in net.parameters():
            if p.grad is not None:
                p.grad.zero_()
        ddp(x).square().sum().backward()
    return {"numels": [int(n) for n in ddp.reducer.bucket_numels()],
            "grads": [p.grad.clone() for p in net.parameters()]}


def ddp_train_amp(rank, world, inject_rank=-1):
    """amp O2 (bf16, CPU) + DDP + FusedSGD: training + overflow consensus."""
    from apex_example_amd import amp
    from apex_example_amd.optimizers import FusedSGD
    from apex_example_amd.parallel import DistributedDataParallel

    model = _mlp()
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.bfloat16,
                                verbosity=0)
    ddp = DistributedDataParallel(model, message_size=200)
    x, y = _data(8 * world, seed=7)
    xs, ys = x.chunk(world)[rank], y.chunk(world)[rank]
    losses = []
    for it in range(4):
        loss = F.cross_entropy(ddp(xs), ys)
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        if it == 2:
            before = [p.detach().clone() for p in amp.master_params(opt)]
        opt.step()
        if it == 2:
            after = [p.detach().clone() for p in amp.master_params(opt)]
        losses.append(loss.item())
        if it == 1 and rank == inject_rank:
            xs = xs.clone()
            xs[0, 0] = float("inf")
        elif it == 2:
            xs = x.chunk(world)[rank]
    return {"losses": losses, "scale": amp.state_dict()["loss_scaler0"]["loss_scale"],
            "skipped_unchanged": all(torch.equal(a, b) for a, b in zip(before, after)),
            "masters": [p.detach().clone() for p in amp.master_params(opt)]}


def reducer_manual(rank, world):
    from apex_example_amd.parallel import Reducer

    model = _mlp()
    if rank == 1:
        with torch.no_grad():
            for p in model.parameters():
                p.mul_(3.0)
    red = Reducer(model)
    for p in model.parameters():
        p.grad = torch.full_like(p, float(rank + 1))
    red.reduce()
    return {"params": [p.detach().clone() for p in model.parameters()],
            "grads": [p.grad.clone() for p in model.parameters()]}


# ---------------------------------------------------------------------- SyncBN
def syncbn_step(rank, world, sizes=(4, 6), channel_last=False, fuse_relu=False, python=False,
                fmt="nchw"):
    from apex_example_amd.parallel import SyncBatchNorm, SyncBatchNormPython

    cls = SyncBatchNormPython if python else SyncBatchNorm
    torch.manual_seed(0)
    C = 8
    full = torch.randn(sum(sizes), C, 5, 5) * 2 + 1
    off = sum(sizes[:rank])
    x = full[off:off + sizes[rank]].clone()
    if fmt == "nhwc":
        x = x.to(memory_format=torch.channels_last)
    if channel_last:
        x = x.permute(0, 2, 3, 1).contiguous()
    x.requires_grad_(True)
    bn = cls(C, channel_last=channel_last, fuse_relu=fuse_relu)
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, C))
        bn.bias.copy_(torch.linspace(-1, 1, C))
    y = bn(x)
    g = torch.Generator().manual_seed(99)
    dy_full = torch.randn(sum(sizes), C, 5, 5, generator=g)
    dy = dy_full[off:off + sizes[rank]]
    if channel_last:
        dy = dy.permute(0, 2, 3, 1)
    (y * dy).sum().backward()
    return {"y": y.detach(), "dx": x.grad.detach(), "dw": bn.weight.grad.clone(),
            "db": bn.bias.grad.clone(), "rm": bn.running_mean.clone(),
            "rv": bn.running_var.clone()}


def gpu_syncbn_step(rank, world, sizes=(4, 6), fuse_relu=True):
    """The GPU SyncBN path (packed stats, one all_gather, device-scaled backward
    sums, one all_reduce) with two ranks sharing cuda:0 over gloo, channels-last
    bf16 with residual + ReLU, vs. BN over the concatenated batch in fp32."""
    from apex_example_amd.ops import batch_norm as bnmod
    from apex_example_amd.parallel import SyncBatchNorm

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    slots0 = bnmod.SLOT_GATHER_CALLS[0]
    C = 16
    full = torch.randn(sum(sizes), C, 6, 6) * 2 + 1
    zfull = torch.randn(sum(sizes), C, 6, 6)
    off = sum(sizes[:rank])
    x = full[off:off + sizes[rank]].cuda().to(torch.bfloat16).to(
        memory_format=torch.channels_last).requires_grad_(True)
    z = zfull[off:off + sizes[rank]].cuda().to(torch.bfloat16).to(
        memory_format=torch.channels_last).requires_grad_(True)
    bn = SyncBatchNorm(C, fuse_relu=fuse_relu).cuda()
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, C))
        bn.bias.copy_(torch.linspace(-1, 1, C))
    y = bn(x, z)
    g = torch.Generator().manual_seed(99)
    dy_full = torch.randn(sum(sizes), C, 6, 6, generator=g)
    dy = dy_full[off:off + sizes[rank]].cuda()
    (y.float() * dy).sum().backward()
    torch.cuda.synchronize()
    return {"y": y.detach().float().cpu(), "dx": x.grad.detach().float().cpu(),
            "dz": z.grad.detach().float().cpu(), "dw": bn.weight.grad.cpu(),
            "db": bn.bias.grad.cpu(), "rm": bn.running_mean.cpu(), "rv": bn.running_var.cpu(),
            "nbt": int(bn.num_batches_tracked),
            "slot_calls": bnmod.SLOT_GATHER_CALLS[0] - slots0}


def syncbn_groups(rank, world):
    from apex_example_amd.parallel import create_syncbn_process_group

    g = create_syncbn_process_group(2)
    return {"group_size": dist.get_world_size(g), "group_rank": dist.get_rank(g)}


def ddp_amp_vs_local(rank, world, opt_level="O2", fused=False, iters=3):
    """Identical data on every rank: apex-DDP-averaged grads must equal the grads
    of an undistributed copy, for the fp32 params amp stashes between
    backward passes (bucket-view grads must not alias the stash)."""
    from apex_example_amd import amp
    from apex_example_amd.optimizers import FusedAdam
    from apex_example_amd.parallel import DistributedDataParallel

    def make():
        torch.manual_seed(0)
        return nn.Sequential(nn.Linear(16, 32), nn.BatchNorm1d(32), nn.ReLU(), nn.Linear(32, 4))

    ma, mb = make(), make()
    if fused:
        oa, ob = FusedAdam(ma.parameters(), lr=1e-2), FusedAdam(mb.parameters(), lr=1e-2)
    else:
        oa = torch.optim.SGD(ma.parameters(), lr=0.1, momentum=0.9)
        ob = torch.optim.SGD(mb.parameters(), lr=0.1, momentum=0.9)
    [ma, mb], [oa, ob] = amp.initialize([ma, mb], [oa, ob], opt_level=opt_level,
                                        half_dtype=torch.bfloat16, num_losses=2, verbosity=0)
    ddp = DistributedDataParallel(ma, message_size=100)
    x, y = _data(8, seed=11)
    diffs = []
    for it in range(iters):
        for lid, (mod, opt) in enumerate(((ddp, oa), (mb, ob))):
            loss = F.cross_entropy(mod(x).float(), y)
            opt.zero_grad()
            with amp.scale_loss(loss, opt, loss_id=lid) as s:
                s.backward()
        ga = [p.grad.float().clone() for p in amp.master_params(oa)]
        gb = [p.grad.float().clone() for p in amp.master_params(ob)]
        diffs.append(max(float((a - b).abs().max() / (b.abs().max() + 1e-6))
                         for a, b in zip(ga, gb)))
        oa.step()
        ob.step()
    return {"diffs": diffs}


def gpu_ddp_resnet(rank, world, steps=4, syncbn=False, lr=0.05, opt_level="O2", hw=32):
    """Two ranks sharing cuda:0 over gloo (RCCL refuses two ranks on one GPU): the
    GPU-side DDP path of bench.py - amp O2 bf16, fused BN, GEMM convs, FusedSGD,
    bucket views - must keep replicas identical and match a one-process run on
    the concatenated batch."""
    from apex_example_amd import amp
    from apex_example_amd.models import resnet18
    from apex_example_amd.optimizers import FusedSGD
    from apex_example_amd.parallel import DistributedDataParallel, convert_syncbn_model

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    m = resnet18(num_classes=10, fused_bn=True, gemm_1x1=True)
    if syncbn:  # bench.py's N > 1 default
        m = convert_syncbn_model(m)
    m = m.cuda().to(memory_format=torch.channels_last)
    opt = FusedSGD(m.parameters(), lr=lr, momentum=0.9, materialize_master_grads=False)
    m, opt = amp.initialize(m, opt, opt_level=opt_level, half_dtype=torch.bfloat16, verbosity=0)
    ddp = DistributedDataParallel(m, message_size=200_000)
    x, y = _resnet_batch(rank, hw=hw)
    losses, masters1 = [], None
    for i in range(steps):
        loss = F.cross_entropy(ddp(x), y)
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
        losses.append(loss.item())
        if i == 0:
            masters1 = [p.detach().float().cpu() for p in amp.master_params(opt)]
    torch.cuda.synchronize()
    return {"params": [p.detach().float().cpu() for p in m.parameters()], "losses": losses,
            "masters": [p.detach().float().cpu() for p in amp.master_params(opt)],
            "masters1": masters1,
            "views": all(getattr(p, "_amd_grad_is_bucket_view", False) for p in m.parameters())}


def _resnet_batch(rank, bs=8, hw=32):
    g = torch.Generator().manual_seed(5 + rank)
    x = torch.randn(bs, 3, hw, hw, generator=g).cuda().to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (bs,), generator=g).cuda()
    return x, y


def gpu_resnet_reference(world=2, steps=4, lr=0.05, opt_level="O2", hw=32):
    """One process, the concatenated per-rank batches of ``gpu_ddp_resnet``,
    local BN (= SyncBN statistics over the global batch), no DDP."""
    from apex_example_amd import amp
    from apex_example_amd.models import resnet18
    from apex_example_amd.optimizers import FusedSGD

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    m = resnet18(num_classes=10, fused_bn=True, gemm_1x1=True)
    m = m.cuda().to(memory_format=torch.channels_last)
    p0 = [p.detach().float().cpu().clone() for p in m.parameters()]
    opt = FusedSGD(m.parameters(), lr=lr, momentum=0.9, materialize_master_grads=False)
    m, opt = amp.initialize(m, opt, opt_level=opt_level, half_dtype=torch.bfloat16, verbosity=0)
    batches = [_resnet_batch(r, hw=hw) for r in range(world)]
    x = torch.cat([b[0] for b in batches]).contiguous(memory_format=torch.channels_last)
    y = torch.cat([b[1] for b in batches])
    losses, masters1 = [], None
    for i in range(steps):
        loss = F.cross_entropy(m(x), y)
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
        losses.append(loss.item())
        if i == 0:
            masters1 = [p.detach().float().cpu() for p in amp.master_params(opt)]
    torch.cuda.synchronize()
    return {"masters": [p.detach().float().cpu() for p in amp.master_params(opt)],
            "masters1": masters1, "losses": losses, "params0": p0}


# ---------------------------------------------------------------------- ZeRO Adam
def dfa_train(rank, world, dtype="fp32", clip=0.0, nb=2, steps=3, scale=1.0):
    from apex_example_amd.contrib.optimizers import DistributedFusedAdam

    model = _mlp()
    if rank == 1:  # DistributedFusedAdam broadcasts rank 0's parameters
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.5)
    if dtype == "bf16":
        model = model.to(torch.bfloat16)
    opt = DistributedFusedAdam(model.parameters(), lr=1e-2, weight_decay=0.01,
                               max_grad_norm=clip, dwu_num_blocks=nb, align=8)
    opt.set_global_scale(scale)
    x, y = _data(8 * world)
    xs, ys = x.chunk(world)[rank], y.chunk(world)[rank]
    for _ in range(steps):
        opt.zero_grad()
        out = model(xs.to(next(model.parameters()).dtype)).float()
        (F.cross_entropy(out, ys) * scale).backward()
        opt.step()
    sd = opt.state_dict()
    return {"params": [p.detach().float().clone() for p in model.parameters()],
            "step": sd["param_groups"][0]["step"], "shard_numel": sd["shards"][0]["master"].numel()}


def gpu_dfa(rank, world, steps=5):
    """Two ranks sharing cuda:0 over gloo: DistributedFusedAdam's HIP path (fused
    Adam on shard views, 16-bit param slice written in-kernel, device-side
    overflow check + step counter under a loss scale) on a bf16 GPT-2 block."""
    from apex_example_amd.contrib.optimizers import DistributedFusedAdam
    from apex_example_amd.models.gpt2 import GPT2Block, GPT2Config

    torch.cuda.set_device(0)
    torch.manual_seed(0)
    cfg = GPT2Config(n_embd=256, n_head=4, resid_pdrop=0.0, attn_pdrop=0.0)
    m = GPT2Block(cfg).cuda().to(torch.bfloat16)
    opt = DistributedFusedAdam(m.parameters(), lr=1e-3, weight_decay=0.01, max_grad_norm=1.0,
                               dwu_num_blocks=3)
    opt.set_global_scale(torch.tensor([1024.0], device="cuda"))
    g = torch.Generator().manual_seed(7 + rank)
    x = torch.randn(2, 128, 256, generator=g).cuda().to(torch.bfloat16)
    losses = []
    for it in range(steps):
        opt.zero_grad()
        loss = m(x).float().pow(2).mean()
        (loss * 1024.0).backward()
        if it == 2 and rank == 1:  # overflow on one rank: every rank must skip
            next(m.parameters()).grad.view(-1)[0] = float("inf")
        before = [p.detach().clone() for p in m.parameters()] if it == 2 else None
        opt.step()
        if it == 2:
            torch.cuda.synchronize()
            skipped = all(torch.equal(a, p.detach()) for a, p in zip(before, m.parameters()))
        losses.append(loss.item())
    torch.cuda.synchronize()
    return {"params": [p.detach().float().cpu() for p in m.parameters()], "losses": losses,
            "skipped": skipped, "step": opt.state_dict()["param_groups"][0]["step"]}


def replica_digests(rank, world, desync=-1):
    """utils/consistency.py on gloo: identical replicas match; one rank with one bit of
    one weight flipped is caught in that group only; comm_info reports the world."""
    from apex_example_amd.utils.consistency import (comm_info, cross_rank_match,
                                                    model_state_groups)

    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(8, 16), nn.BatchNorm1d(16), nn.Linear(16, 4))
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    model(torch.randn(4, 8)).sum().backward()
    opt.step()
    if rank == desync:
        with torch.no_grad():
            model[2].weight.view(-1)[:1].view(torch.int32).add_(1)
    res = cross_rank_match(model_state_groups(model, opt))
    return {"match": {k: v["match"] for k, v in res.items()},
            "digest": {k: v["digest"] for k, v in res.items()},
            "comm": comm_info(dist.group.WORLD)}
