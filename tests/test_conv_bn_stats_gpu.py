"""BatchNorm statistics computed in the producing conv's epilogue:
the own MFMA conv kernels (csrc/hip/conv_igemm.hip) write per-M-tile shifted sums of
their bf16 output for the consuming BN, which then finalizes from that slab instead of
re-reading the activation.  Checked against an fp64 reference of the same output, the
conv output itself must be bitwise unchanged, and a ResNet training step with the fusion
must match the unfused one to rounding."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _C():
    from apex_example_amd import _native
    return _native.require()


@pytest.mark.parametrize("shape", [
    # (N, Cin, H, W, Cout, k, stride)
    (4, 64, 56, 56, 64, 3, 1),     # 3x3, 64-wide tiles
    (2, 128, 28, 28, 128, 3, 1),   # 3x3, 128-wide tiles
    (3, 128, 14, 14, 128, 3, 2),   # strided 3x3, M = 147 (partial last tile)
    (4, 64, 56, 56, 256, 1, 1),    # channel-expanding 1x1
    (2, 256, 28, 28, 512, 1, 2),   # strided 1x1 projection
    (1, 512, 7, 7, 2048, 1, 1),    # M = 49 < one tile
    (96, 64, 56, 56, 64, 1, 1),    # S = 2,352 tiles: one channel per finalize workgroup
])
@pytest.mark.parametrize("use_shift", [False, True])
def test_conv_epilogue_stats_match_reference(shape, use_shift):
    N, Cin, H, W, Cout, k, s = shape
    C = _C()
    torch.manual_seed(0)
    x = torch.randn(N, Cin, H, W, device=dev).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, k, k, device=dev) / (Cin * k * k) ** 0.5 + 0.01).to(
        torch.bfloat16).contiguous(memory_format=torch.channels_last)
    shift = (torch.randn(Cout, device=dev) * 0.1 + 0.02) if use_shift else None
    y_ref = C.conv.conv_fwd(x, w, s)
    y, slab = C.conv.conv_fwd_stats(x, w, s, shift)
    assert torch.equal(y, y_ref)                   # the epilogue does not touch y
    count = y.numel() // Cout
    rm = shift.clone() if use_shift else torch.zeros(Cout, device=dev)
    rv = torch.ones(Cout, device=dev)
    nbt = torch.zeros((), dtype=torch.long, device=dev)
    mean, invstd = C.bn.slab_train_stats(slab, count, rm if use_shift else None, rm, rv, nbt,
                                         1e-5, 0.1)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, Cout)
    m_ref = yd.mean(0)
    v_ref = yd.var(0, unbiased=False)
    torch.testing.assert_close(mean.double(), m_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(invstd.double(), (v_ref + 1e-5).rsqrt(), rtol=1e-4, atol=1e-5)
    base = shift if use_shift else torch.zeros(Cout, device=dev)
    torch.testing.assert_close(rm.double(), 0.9 * base.double() + 0.1 * m_ref, rtol=1e-5,
                               atol=1e-5)
    unb = v_ref * count / max(count - 1, 1)
    torch.testing.assert_close(rv.double(), 0.9 + 0.1 * unb, rtol=1e-5, atol=1e-5)
    assert int(nbt) == 1
    # SyncBN packed form: [mean | biased var | count]
    packed = C.bn.slab_packed_stats(slab, count, shift)
    torch.testing.assert_close(packed[:Cout].double(), m_ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(packed[Cout:2 * Cout].double(), v_ref, rtol=1e-4, atol=1e-5)
    assert float(packed[-1]) == count


@pytest.mark.parametrize("arch", ["resnet50", "resnet18"])
def test_every_bn_in_resnet_gets_its_own_statistics(arch):
    """One training-mode forward of a whole ResNet with the epilogue statistics on: for
    EVERY BatchNorm, the running-stat update must equal the fp64 statistics of the
    tensor that BN actually received (so no slab is attached to the wrong layer), and
    the slab path must really have been taken for the own-kernel convs."""
    from apex_example_amd.models import resnet18, resnet50
    from apex_example_amd.ops import batch_norm as bnmod
    from apex_example_amd.ops.batch_norm import BatchNorm2dReLU

    torch.manual_seed(0)
    ctor = {"resnet50": resnet50, "resnet18": resnet18}[arch]
    m = ctor(fused_bn=True, gemm_1x1=True).to(dev).to(torch.bfloat16)
    for mod in m.modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            mod.float()
    m = m.to(memory_format=torch.channels_last).train()
    seen = {}
    took = []
    orig_take = bnmod.take_slab

    def spy_take(x, bn):
        r = orig_take(x, bn)
        if r[0] is not None:
            took.append(bn)
        return r
    bnmod.take_slab = spy_take
    hooks = []
    for name, mod in m.named_modules():
        if isinstance(mod, BatchNorm2dReLU):
            def pre(mo, args, n=name):
                x = args[0]
                seen[n] = (x.detach().double().permute(0, 2, 3, 1).reshape(-1, x.size(1)),
                           mo.running_mean.clone(), mo.running_var.clone())
            hooks.append(mod.register_forward_pre_hook(pre))
    try:
        x = torch.randn(8, 3, 96, 96, device=dev).to(torch.bfloat16).to(
            memory_format=torch.channels_last)
        with torch.no_grad():
            m(x)
    finally:
        bnmod.take_slab = orig_take
        for h in hooks:
            h.remove()
    mods = dict(m.named_modules())
    assert len(took) >= (30 if arch == "resnet50" else 14), len(took)
    for n, (xd, rm0, rv0) in seen.items():
        bn = mods[n]
        mean = xd.mean(0)
        var = xd.var(0, unbiased=True)
        torch.testing.assert_close(bn.running_mean.double(), 0.9 * rm0.double() + 0.1 * mean,
                                   rtol=1e-4, atol=1e-5, msg=n)
        torch.testing.assert_close(bn.running_var.double(), 0.9 * rv0.double() + 0.1 * var,
                                   rtol=1e-3, atol=1e-5, msg=n)


def _resnet_step(fused_stats, arch="resnet50", steps=3):
    from apex_example_amd import amp
    from apex_example_amd.models import resnet18, resnet50
    from apex_example_amd.ops import conv as convmod
    from apex_example_amd.optimizers import FusedSGD

    prev = convmod._CONV_BN_STATS
    convmod._CONV_BN_STATS = fused_stats
    try:
        torch.manual_seed(0)
        ctor = {"resnet50": resnet50, "resnet18": resnet18}[arch]
        # zero-init residual branches: a non-chaotic network at init, so two runs that
        # differ only in the rounding of the BN statistics stay close (with random
        # residual weights the 1-ulp output differences grow ~10x per stage:
        # tools/diag/bn_stats_diff.py)
        m = ctor(fused_bn=True, gemm_1x1=True, num_classes=100, zero_init_residual=True).to(
            dev).to(memory_format=torch.channels_last)
        opt = FusedSGD(m.parameters(), lr=0.02, momentum=0.9, materialize_master_grads=False)
        m, opt = amp.initialize(m, opt, opt_level="O2", half_dtype=torch.bfloat16, verbosity=0)
        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.randn(16, 3, 128, 128, device=dev, generator=g).to(
            memory_format=torch.channels_last)
        y = torch.randint(0, 100, (16,), device=dev, generator=g)
        losses = []
        for _ in range(steps):
            loss = F.cross_entropy(m(x), y)
            opt.zero_grad()
            with amp.scale_loss(loss, opt) as sl:
                sl.backward()
            opt.step()
            losses.append(float(loss))
        bufs = {n: b.detach().clone() for n, b in m.named_buffers()}
        return losses, bufs
    finally:
        convmod._CONV_BN_STATS = prev


@pytest.mark.parametrize("arch", ["resnet50", "resnet18"])
def test_resnet_training_with_epilogue_stats_matches_stats_pass(arch, monkeypatch):
    from apex_example_amd import _native

    calls = {"n": 0}
    bn = _native.require().bn
    orig = bn.slab_train_stats

    class Spy:
        def __getattr__(self, k):
            return getattr(bn, k)

        def slab_train_stats(self, *a, **k):
            calls["n"] += 1
            return orig(*a, **k)
    from apex_example_amd.ops import batch_norm as bnmod
    monkeypatch.setattr(bnmod, "_C", lambda: Spy())
    l1, b1 = _resnet_step(True, arch)
    used = calls["n"]
    l0, b0 = _resnet_step(False, arch)
    assert used > 0 and calls["n"] == used       # only the fused run took slabs
    assert abs(l1[0] - l0[0]) <= 1e-3 * abs(l0[0]), (l1, l0)   # same forward to rounding
    for a, b in zip(l1, l0):
        assert abs(a - b) <= 2e-2 * abs(b) + 2e-3, (l1, l0)
    for k in b0:
        if k.endswith("num_batches_tracked"):
            assert torch.equal(b0[k], b1[k]), k
        else:
            torch.testing.assert_close(b1[k], b0[k], rtol=2e-2, atol=2e-3, msg=k)
