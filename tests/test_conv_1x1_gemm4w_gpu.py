"""Stride-1 1x1 conv forwards on gemm4w (csrc/hip/gemm4w.hip EPI 3: bf16 store + the
consuming BatchNorm's channel-major statistics slab): outputs against fp32 F.conv2d and
against the own implicit-GEMM kernel (the path with the switch off), the slab's sums
against fp64 sums of the stored bf16 output, ragged M (partial last 256-row tile), and
bitwise stability across calls.  The slab width tells which kernel ran (ceil(M / 256)
gemm4w tiles vs ceil(M / 128))."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)
CL = torch.channels_last


def _C():
    from apex_example_amd import _native
    return _native.require()


@pytest.fixture
def g4w_switch():
    C = _C()
    yield C.conv.set_1x1_gemm4w
    C.conv.set_1x1_gemm4w(0)


@pytest.mark.parametrize("shape", [
    # (N, C_in, H, W, C_out)
    (4, 256, 14, 14, 1024),
    (2, 128, 28, 28, 512),
    (3, 512, 7, 7, 2048),
    (2, 64, 30, 17, 256),     # M = 1020: partial last tile
    (1, 1024, 9, 9, 256),     # M = 81 < one tile
])
def test_conv1x1_gemm4w_matches_fp32_and_own(shape, g4w_switch):
    N, Ci, H, W, Co = shape
    C = _C()
    torch.manual_seed(7)
    x = torch.randn(N, Ci, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(Co, Ci, 1, 1, device=dev) / Ci ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=CL)
    shift = torch.randn(Co, device=dev) * 0.1
    M = N * H * W

    g4w_switch(2)                       # every eligible shape (the default takes the winners)
    y = C.conv.conv_fwd(x, w, 1)
    ys, slab = C.conv.conv_fwd_stats(x, w, 1, shift)
    y0, slab0 = C.conv.conv_fwd_stats(x, w, 1, None)
    assert slab.shape == (2, Co, (M + 255) // 256), "gemm4w did not run"
    g4w_switch(0)
    yo, slabo = C.conv.conv_fwd_stats(x, w, 1, shift)
    assert slabo.shape[2] == (M + 127) // 128

    ref = F.conv2d(x.float(), w.float())
    scale = float(ref.abs().max())
    for t in (y, ys, y0, yo):
        assert float((t.float() - ref).abs().max()) / scale < 1e-2
    assert torch.equal(y, ys) and torch.equal(y, y0)
    d = (y.float() - yo.float()).abs()
    assert float((d > 0).float().mean()) < 0.05          # fp32 accumulation order only
    yv = ys.double() - shift.double().view(1, -1, 1, 1)
    s = slab.double().sum(2)
    torch.testing.assert_close(s[0], yv.sum((0, 2, 3)), rtol=1e-5, atol=1e-2)
    torch.testing.assert_close(s[1], (yv ** 2).sum((0, 2, 3)), rtol=1e-5, atol=1e-2)
    s0 = slab0.double().sum(2)
    torch.testing.assert_close(s0[0], y0.double().sum((0, 2, 3)), rtol=1e-5, atol=1e-2)
    # bitwise stable
    g4w_switch(2)
    ys2, slab2 = C.conv.conv_fwd_stats(x, w, 1, shift)
    assert torch.equal(ys, ys2) and torch.equal(slab, slab2)


def test_conv1x1_gemm4w_default_table(g4w_switch):
    """Mode 1 routes exactly the measured winners."""
    C = _C()
    g4w_switch(1)
    on = C.conv.on_gemm4w_1x1
    assert on(12544, 512, 2048) and on(50176, 1024, 256) and on(802816, 64, 256)
    assert not on(200704, 128, 512) and not on(50176, 256, 1024) and not on(12544, 2048, 512)
    assert not on(50176, 256, 64)       # Cout % 256 != 0
    g4w_switch(0)
    assert not on(12544, 512, 2048)
