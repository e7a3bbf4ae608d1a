"""One-launch (persistent, grid-barrier) BatchNorm kernels (csrc/hip/bn_persist.hip)
against an fp32 PyTorch reference of the same op and against the split-kernel path.

Covers the four ResNet-50 variants (BN+ReLU, BN+residual+ReLU with the 1-bit mask,
plain BN, BN+residual without ReLU), channel counts that leave idle lanes (C/8 not
a multiple of the lane tile), rows that do not fill the last row block, and many
launches back to back with different grids (the barrier's generation / parity
state), with the barrier's error word checked at the end.
"""
import pytest
import torch

from apex_example_amd import _native

pytestmark = pytest.mark.gpu

dev = torch.device("cuda", 0)


def _C():
    return _native.require().bn


def _ref(x, z, w, b, eps, relu):
    xf = x.float()
    dims = (0, 2, 3)
    mean = xf.mean(dims)
    var = xf.var(dims, unbiased=False)
    y = (xf - mean[None, :, None, None]) * torch.rsqrt(var + eps)[None, :, None, None]
    y = y * w[None, :, None, None] + b[None, :, None, None]
    if z is not None:
        y = y + z.float()
    if relu:
        y = torch.relu(y)
    return y, mean, var


def _run(shape, with_z, relu, seed=0, persist=True):
    from apex_example_amd.ops.batch_norm import BatchNorm2dReLU
    torch.manual_seed(seed)
    N, C, H, W = shape
    x = (torch.randn(shape, device=dev) * 2 + 0.5).to(torch.bfloat16).to(
        memory_format=torch.channels_last).requires_grad_(True)
    z = None
    if with_z:
        z = torch.randn(shape, device=dev).to(torch.bfloat16).to(
            memory_format=torch.channels_last).requires_grad_(True)
    bn = BatchNorm2dReLU(C, fuse_relu=relu).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    prev = _C().persist_mode()
    _C().persist_enable(int(persist))
    try:
        y = bn(x, z) if with_z else bn(x)
        g = torch.randn(shape, device=dev).to(torch.bfloat16).to(memory_format=torch.channels_last)
        y.backward(g)
        torch.cuda.synchronize()
    finally:
        _C().persist_enable(prev)
    return x, z, bn, y, g


SHAPES = [(64, 256, 14, 14), (32, 512, 7, 7), (4, 200, 9, 7), (3, 2048, 7, 7), (16, 64, 28, 28)]
VARIANTS = [(False, True), (True, True), (False, False), (True, False)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("with_z,relu", VARIANTS)
def test_persist_matches_fp32_reference(shape, with_z, relu):
    n0 = _C().persist_launches()
    x, z, bn, y, g = _run(shape, with_z, relu)
    assert _C().persist_launches() >= n0 + 2, "persistent kernels did not run"
    # reference forward / backward in fp32 on the same bf16 inputs
    xr = x.detach().float().requires_grad_(True)
    zr = z.detach().float().requires_grad_(True) if z is not None else None
    w = bn.weight.detach().clone().requires_grad_(True)
    b = bn.bias.detach().clone().requires_grad_(True)
    yr, mean, var = _ref(xr, zr, w, b, bn.eps, relu)
    yr.backward(g.float())
    scale = yr.abs().max().item()
    assert (y.float() - yr).abs().max().item() <= 1e-2 * scale
    # running statistics (momentum 0.1, unbiased variance)
    M = x.numel() // x.size(1)
    torch.testing.assert_close(bn.running_mean, 0.1 * mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.running_var, 0.9 + 0.1 * var * M / (M - 1), rtol=1e-3,
                               atol=1e-4)
    assert int(bn.num_batches_tracked) == 1
    gs = xr.grad.abs().max().item()
    assert (x.grad.float() - xr.grad).abs().max().item() <= 2e-2 * gs
    if z is not None:
        assert (z.grad.float() - zr.grad).abs().max().item() <= 1e-2 * zr.grad.abs().max().item()
    torch.testing.assert_close(bn.weight.grad, w.grad, rtol=2e-3, atol=2e-3 * w.grad.abs().max().item())
    torch.testing.assert_close(bn.bias.grad, b.grad, rtol=2e-3, atol=2e-3 * b.grad.abs().max().item())
    assert _C().persist_error() == 0


@pytest.mark.parametrize("with_z,relu", VARIANTS)
def test_persist_matches_split_path(with_z, relu):
    shape = (64, 256, 14, 14)
    a = _run(shape, with_z, relu, seed=3, persist=True)
    s = _run(shape, with_z, relu, seed=3, persist=False)
    # same math, different summation order: agree to a few bf16 ulps
    assert (a[3].float() - s[3].float()).abs().max().item() <= 2e-2 * s[3].float().abs().max().item()
    assert (a[0].grad.float() - s[0].grad.float()).abs().max().item() <= \
        2e-2 * s[0].grad.float().abs().max().item()
    torch.testing.assert_close(a[2].weight.grad, s[2].weight.grad, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(a[2].running_var, s[2].running_var, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("mode", [1, 2])
def test_persist_many_launches_alternating_grids(mode):
    # the barrier state (generation parity, counter reset, accumulator zeroing) across
    # 40 launches whose grids differ; mode 2 = the barrier without release/acquire fences
    C = _C()
    shapes = [(64, 256, 14, 14), (32, 512, 7, 7), (8, 128, 14, 14), (4, 200, 9, 7)]
    for i in range(40):
        shape = shapes[i % len(shapes)]
        x, z, bn, y, g = _run(shape, i % 3 == 0, i % 2 == 0, seed=i, persist=mode)
        yr, _, _ = _ref(x.detach().float(), z.detach().float() if z is not None else None,
                        bn.weight.detach(), bn.bias.detach(), bn.eps, i % 2 == 0)
        assert (y.float() - yr).abs().max().item() <= 1e-2 * yr.abs().max().item(), i
    assert C.persist_error() == 0


def test_persist_falls_back_when_too_large():
    # more rows than the resident grid can hold: the split kernels run instead
    C = _C()
    n0 = C.persist_launches()
    x, z, bn, y, g = _run((128, 256, 28, 28), False, True)
    assert C.persist_launches() == n0
    yr, _, _ = _ref(x.detach().float(), None, bn.weight.detach(), bn.bias.detach(), bn.eps, True)
    assert (y.float() - yr).abs().max().item() <= 1e-2 * yr.abs().max().item()
