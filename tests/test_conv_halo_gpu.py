"""3x3 stride-1 forward with the LDS-resident input halo (csrc/hip/conv_igemm.hip
conv3h_k): every output of the halo kernel - plain forward, forward + BN statistics,
forward + BN-backward epilogue - against fp32 and against the per-tap kernel
(conv_tap_k, the path with the halo switched off), on shapes whose 256-pixel tiles cross
image rows, images and the padded border in every way (tiny images many per tile, odd
widths, partial last tiles).  The statistics slab's width tells which kernel ran
(ceil(M / 256) halo tiles vs ceil(M / 128)).  Both tile widths (128 and 64 output
channels) run: automatically by shape and forced through the A/B switch.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)
CL = torch.channels_last


def _C():
    from apex_example_amd import _native
    return _native.require()


def _bf(t):
    return t.to(torch.bfloat16).contiguous(memory_format=CL)


@pytest.fixture
def halo_switch():
    C = _C()
    was = C.conv.halo_enabled()
    yield C.conv.set_halo
    C.conv.set_halo(was)
    C.conv.set_halo_mtile(0)


SHAPES = [
    # (N, C_in, H, W, C_out)
    (2, 128, 28, 28, 128),
    (2, 256, 14, 14, 256),
    (4, 512, 7, 7, 512),      # 5 images per tile
    (3, 64, 9, 11, 128),      # odd width, M = 297: partial last tile
    (5, 128, 5, 3, 256),      # 15-pixel images: 17 per tile
    (1, 64, 56, 56, 128),
    (2, 96 * 2, 13, 17, 128),
    (2, 64, 56, 56, 64),      # 500-row window: the 64-wide tile's 512-row buffer
    (2, 128, 20, 20, 192),    # Cout % 128 != 0: 64-wide tiles
]


def _run(C, x, w, shift, xb, add, mean, invstd, bw, bb):
    y = C.conv.conv_fwd(x, w, 1)
    ys, slab = C.conv.conv_fwd_stats(x, w, 1, shift)
    g0, s0 = C.conv.conv_fwd_bnbwd(x, w, None, xb, None, mean, invstd, bw, bb, 2)
    g1, s1 = C.conv.conv_fwd_bnbwd(x, w, add, xb, None, mean, invstd, bw, bb, 0)
    return y, ys, slab, g0, s0, g1, s1


@pytest.mark.parametrize("mode,bm", [(1, 256), (1, 224), (64, 256)])
@pytest.mark.parametrize("shape", SHAPES)
def test_halo_conv_matches_fp32_and_tap_kernel(shape, mode, bm, halo_switch):
    N, Ci, H, W, Co = shape
    C = _C()
    torch.manual_seed(3)
    x = _bf(torch.randn(N, Ci, H, W, device=dev))
    w = _bf(torch.randn(Co, Ci, 3, 3, device=dev) / (Ci * 9) ** 0.5)
    xb = _bf(torch.randn(N, Co, H, W, device=dev) * 1.3 + 0.2)
    add = _bf(torch.randn(N, Co, H, W, device=dev))
    mean = torch.randn(Co, device=dev) * 0.1
    invstd = torch.rand(Co, device=dev) + 0.5
    bw, bb = torch.randn(Co, device=dev), torch.randn(Co, device=dev) * 0.2
    shift = torch.randn(Co, device=dev) * 0.1
    args = (x, w, shift, xb, add, mean, invstd, bw, bb)
    M = N * H * W

    C.conv.set_halo_mtile(bm)           # 224-pixel tiles exist for the 128-wide kernel only
    halo_switch(mode)
    h = _run(C, *args)
    halo_switch(0)
    t = _run(C, *args)
    halo_switch(mode)
    assert t[2].shape[2] == (M + 127) // 128
    halo = not (bm == 224 and Co % 128 != 0)
    tiles = (M + bm - 1) // bm if halo else (M + 127) // 128
    assert h[2].shape[2] == tiles, "the halo kernel did not run" if halo else "unexpected"

    ref = F.conv2d(x.float(), w.float(), padding=1)
    scale = float(ref.abs().max())
    for y in (h[0], t[0]):
        err = float((y.float() - ref).abs().max()) / scale
        assert err < 1e-2, err
    # both kernels accumulate in fp32 (different order): their bf16 outputs agree to one
    # rounding step almost everywhere
    d = (h[0].float() - t[0].float()).abs()
    assert float(d.max()) <= 2 * float(ref.abs().max()) * 2 ** -8
    assert float((d > 0).float().mean()) < 0.05
    assert torch.equal(h[0], h[1])                       # stats variant stores the same y

    yv = h[1].float() - shift.view(1, -1, 1, 1)
    sums = h[2].double().sum(2)
    torch.testing.assert_close(sums[0], yv.double().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(sums[1], (yv.double() ** 2).sum((0, 2, 3)), rtol=1e-4, atol=1e-2)

    # BN-backward epilogue: mode 2 (ReLU recomputed from x) and mode 0 with a residual add,
    # both against the halo kernel's own plain output
    sc = invstd * bw
    pre = xb.float() * sc.view(1, -1, 1, 1) + (bb - mean * sc).view(1, -1, 1, 1)
    keep, border = pre > 0, pre.abs() < 1e-4
    ref0 = torch.where(keep, h[0].float(), torch.zeros_like(ref))
    ok = ~border
    torch.testing.assert_close(h[3].float()[ok], ref0[ok], rtol=0, atol=0)
    ref1 = (h[0].float() + add.float()).to(torch.bfloat16).float()
    torch.testing.assert_close(h[5].float(), ref1, rtol=0, atol=0)
    for g, s in ((h[3], h[4]), (h[5], h[6])):
        assert s.shape[2] == tiles
        gd = g.double().permute(0, 2, 3, 1).reshape(-1, Co)
        xd = xb.double().permute(0, 2, 3, 1).reshape(-1, Co)
        ss = s.double().sum(2)
        torch.testing.assert_close(ss[0], gd.sum(0), rtol=1e-5, atol=1e-3)
        torch.testing.assert_close(ss[1], (gd * (xd - mean.double())).sum(0), rtol=1e-5, atol=1e-3)

    # deterministic: a second run is bitwise identical
    for i, (a, b) in enumerate(zip(h, _run(C, *args))):
        assert torch.equal(a, b), i


def test_halo_window_limit_falls_back(halo_switch):
    """A 256-pixel tile of 120-wide rows that crosses an image needs a ~750-row window (>
    512): such shapes keep the per-tap kernel (128-pixel tiles) and stay correct."""
    C = _C()
    halo_switch(1)
    torch.manual_seed(4)
    x = _bf(torch.randn(2, 64, 40, 120, device=dev))
    w = _bf(torch.randn(128, 64, 3, 3, device=dev) / 24.0)
    y, slab = C.conv.conv_fwd_stats(x, w, 1, None)
    assert slab.shape[2] == (2 * 40 * 120 + 127) // 128
    ref = F.conv2d(x.float(), w.float(), padding=1)
    assert float((y.float() - ref).abs().max() / ref.abs().max()) < 1e-2
