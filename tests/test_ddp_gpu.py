"""DDP on the GPU over RCCL (world_size 1 on the single-GPU test box): the
apex ddp_race_condition_test pattern - many iterations
with many small buckets whose all-reduces run on RCCL's stream while backward
keeps producing grads, every grad checked against a closed form right after
backward, and the bucket buffers consumed immediately by an in-place op."""
import os

import pytest
import torch
import torch.distributed as dist

import dist_workers as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(W.free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


class _Model(torch.nn.Module):
    def __init__(self, n=24, numel=4096 * 64):
        super().__init__()
        self.ps = torch.nn.ParameterList(
            [torch.nn.Parameter(torch.full((numel,), float(i + 1), device="cuda"))
             for i in range(n)])

    def forward(self, x):
        # d(loss)/d(p_i) = x * (i + 1): a closed form per param and iteration
        return sum((p * x * (i + 1)).sum() for i, p in enumerate(self.ps))


@pytest.mark.parametrize("streams", [1, 2])
def test_ddp_race_condition(pg, streams):
    from apex_example_amd.parallel import DistributedDataParallel

    model = _Model()
    ddp = DistributedDataParallel(model, message_size=4096 * 64 * 2,
                                  num_allreduce_streams=streams)
    bad = torch.zeros((), device="cuda")
    for it in range(60):
        x = torch.tensor(float(it % 7 + 1), device="cuda")
        for p in model.ps:
            if p.grad is not None:
                p.grad.zero_()
        ddp(x).backward()
        for i, p in enumerate(model.ps):
            bad += (p.grad - x * (i + 1)).abs().max()
            p.grad.mul_(0.5)  # consume the bucket in place right away
    torch.cuda.synchronize()
    assert bad.item() == 0.0
    assert len(ddp.bucket_layout()) >= 6


def test_ddp_resnet_amp_step(pg):
    """ResNet-18 amp O2 + apex DDP + FusedSGD on RCCL: grads are bucket views and
    the step is sync-free."""
    from apex_example_amd import amp
    from apex_example_amd.models import resnet18
    from apex_example_amd.optimizers import FusedSGD
    from apex_example_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, materialize_master_grads=False)
    m, opt = amp.initialize(m, opt, opt_level="O2", half_dtype=torch.bfloat16, verbosity=0)
    ddp = DistributedDataParallel(m, message_size=2_000_000)
    x = torch.randn(16, 3, 64, 64, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")
    losses = []
    for _ in range(8):
        loss = torch.nn.functional.cross_entropy(ddp(x), y)
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
        losses.append(loss.item())
    assert all(getattr(p, "_amd_grad_is_bucket_view", False) for p in m.parameters())
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("syncbn", [False, True])
def test_two_ranks_one_gpu_gloo(tmp_path, syncbn):
    """bench.py's N>1 code path (apex DDP over a process group, bucket views, fused
    kernels, SyncBN by default) with two processes on the one test GPU."""
    res = W.run("gpu_ddp_resnet", 2, str(tmp_path), syncbn=syncbn)
    for a, b in zip(res[0]["params"], res[1]["params"]):
        assert torch.equal(a, b)
    assert res[0]["views"] and res[1]["views"]
    assert res[0]["losses"][-1] < res[0]["losses"][0]


def test_distributed_fused_adam_two_ranks_one_gpu(tmp_path):
    res = W.run("gpu_dfa", 2, str(tmp_path))
    for a, b in zip(res[0]["params"], res[1]["params"]):
        assert torch.equal(a, b)
    for r in res:
        assert r["skipped"]          # the injected overflow skipped the step on both ranks
        assert r["step"] == 4        # 5 steps, one skipped
    assert res[0]["losses"][-1] < res[0]["losses"][0]


def test_syncbn_gpu_two_ranks_matches_global_batch(tmp_path):
    """GPU SyncBN (bench.py's N>1 default) == BN + residual + ReLU over the global batch."""
    sizes = (4, 6)
    res = W.run("gpu_syncbn_step", 2, str(tmp_path), sizes=sizes)
    torch.manual_seed(0)
    C = 16
    full = torch.randn(sum(sizes), C, 6, 6) * 2 + 1
    zfull = torch.randn(sum(sizes), C, 6, 6)
    x = full.to(torch.bfloat16).float().requires_grad_(True)
    z = zfull.to(torch.bfloat16).float().requires_grad_(True)
    bn = torch.nn.BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, C))
        bn.bias.copy_(torch.linspace(-1, 1, C))
    y = torch.relu(bn(x) + z)
    g = torch.Generator().manual_seed(99)
    dy = torch.randn(sum(sizes), C, 6, 6, generator=g)
    (y * dy).sum().backward()
    ys = torch.cat([r["y"] for r in res])
    torch.testing.assert_close(ys, y.detach(), rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(torch.cat([r["dx"] for r in res]), x.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(torch.cat([r["dz"] for r in res]), z.grad, rtol=3e-2, atol=3e-2)
    # dgamma / dbeta are per-rank partial sums (DDP all-reduces them as gradients)
    torch.testing.assert_close(res[0]["dw"] + res[1]["dw"], bn.weight.grad, rtol=3e-2, atol=5e-2)
    torch.testing.assert_close(res[0]["db"] + res[1]["db"], bn.bias.grad, rtol=3e-2, atol=5e-2)
    for r in res:
        torch.testing.assert_close(r["rm"], bn.running_mean, rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(r["rv"], bn.running_var, rtol=2e-2, atol=2e-2)
        assert r["nbt"] == 1
