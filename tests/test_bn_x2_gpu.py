"""The downsample BN's backward sums formed in the consuming BN's elementwise pass
(ops/batch_norm.py _X2_BWD, csrc/hip/bn_nhwc.hip backward_k<..., X2>): the kernel's sums
vs an fp64 reference, and a ResNet-50 step's gradients with the fusion on vs off."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_backward_elemt_x2_sums_match_reference():
    from apex_example_amd import _native

    C = _native.require().bn
    torch.manual_seed(0)
    n, c, h, w = 8, 256, 14, 14
    cl = torch.channels_last
    dy = torch.randn(n, c, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=cl)
    x = torch.randn(n, c, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=cl)
    x2 = (torch.randn(n, c, h, w, device=DEV) * 2 + 1).to(torch.bfloat16).contiguous(memory_format=cl)
    mean, invstd = torch.randn(c, device=DEV) * 0.1, torch.rand(c, device=DEV) + 0.5
    mean2, invstd2 = torch.randn(c, device=DEV), torch.rand(c, device=DEV) + 0.5
    wt, bs = torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV)
    wt2 = torch.rand(c, device=DEV) + 0.5
    sdy, sdx = torch.randn(c, device=DEV), torch.randn(c, device=DEV)
    cnt = float(n * h * w)
    assert C.backward_x2_ok(dy, x, x2)
    dx, s1, s2, gw2, gb2 = C.backward_elemt_x2(dy, x, mean, invstd, wt, bs, sdy, sdx, cnt, x2,
                                               mean2, invstd2, wt2, True)
    dx_ref, _ = C.backward_elemt(dy, x, mean, invstd, wt, bs, sdy, sdx, cnt, None, False, False)
    assert torch.equal(dx, dx_ref)
    d = dy.double().permute(0, 2, 3, 1).reshape(-1, c)
    xd = x2.double().permute(0, 2, 3, 1).reshape(-1, c)
    r1 = d.sum(0)
    r2 = (d * (xd - mean2.double())).sum(0)
    torch.testing.assert_close(s1.double(), r1, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s2.double(), r2, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(gb2.double(), r1, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(gw2.double(), r2 * invstd2.double(), rtol=1e-4, atol=1e-2)


def test_resnet50_step_grads_with_x2_fusion(monkeypatch):
    from apex_example_amd.models import resnet50
    from apex_example_amd.ops import batch_norm as B

    # the separate-module downsample path (the fused bn3 + downsample-BN pass replaces it)
    monkeypatch.setattr(B, "_FUSE_DS", False)

    torch.manual_seed(0)
    m = resnet50(fused_bn=True, gemm_1x1=True).to(DEV).to(memory_format=torch.channels_last)
    m = m.to(torch.bfloat16)
    for mod in m.modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            mod.float()
    x = torch.randn(8, 3, 96, 96, device=DEV).to(torch.bfloat16).to(
        memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    grads = []
    for on in (True, False):
        m.load_state_dict(state)
        m.zero_grad(set_to_none=True)
        old = B._X2_BWD
        B._X2_BWD = on
        before = B.X2_BWD_CALLS[0]
        try:
            m(x).float().square().mean().backward()
        finally:
            B._X2_BWD = old
        used = B.X2_BWD_CALLS[0] - before
        assert (used > 0) == on, used
        grads.append({n: p.grad.float().clone() for n, p in m.named_parameters()})
    # the fusion changes only fp32 summation order; bf16 roundings downstream of it then
    # spread the difference through the earlier layers: the first fused BN (layer4's
    # downsample, whose dy is still identical in both runs) matches to fp32 rounding,
    # every gradient matches in direction
    for n in grads[0]:
        a, b = grads[0][n].flatten(), grads[1][n].flatten()
        if n.startswith("layer4.0.downsample.bn."):
            scale = b.abs().max().clamp_min(1e-6)
            assert float((a - b).abs().max() / scale) < 1e-3, n
        cos = float(torch.nn.functional.cosine_similarity(a.double(), b.double(), dim=0))
        assert cos > 0.99 or float(b.abs().max()) < 1e-6, (n, cos)


def test_apply2_bitwise_equals_two_passes():
    """apply2_mask: relu(bn(x) + bnd(xd)) with the downsample BN applied on load is bitwise
    the output and mask of bnd's apply pass followed by bn's apply with z."""
    from apex_example_amd import _native

    C = _native.require().bn
    torch.manual_seed(3)
    n, c, h, w = 4, 512, 14, 14
    cl = torch.channels_last
    x = torch.randn(n, c, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=cl)
    xd = (torch.randn(n, c, h, w, device=DEV) * 3).to(torch.bfloat16).contiguous(memory_format=cl)
    m, i = torch.randn(c, device=DEV) * 0.1, torch.rand(c, device=DEV) + 0.5
    md, idd = torch.randn(c, device=DEV), torch.rand(c, device=DEV) + 0.2
    wt, bs = torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV)
    wd, bd = torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV)
    y, mask = C.apply2_mask(x, m, i, wt, bs, xd, md, idd, wd, bd)
    z = C.apply(xd, md, idd, wd, bd, None, False)
    y2, mask2 = C.apply_mask(x, m, i, wt, bs, z, True)
    assert torch.equal(y, y2) and torch.equal(mask, mask2)


def test_resnet50_step_with_fused_downsample_bn():
    """ResNet-50 train step with the downsample BN fused into bn3's pass vs the two module
    calls: identical output and running stats, gradients to bf16 noise."""
    from apex_example_amd.models import resnet50
    from apex_example_amd.ops import batch_norm as B

    torch.manual_seed(0)
    m = resnet50(fused_bn=True, gemm_1x1=True).to(DEV).to(memory_format=torch.channels_last)
    m = m.to(torch.bfloat16)
    for mod in m.modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            mod.float()
    x = torch.randn(8, 3, 96, 96, device=DEV).to(torch.bfloat16).to(
        memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    runs = []
    for on in (True, False):
        m.load_state_dict(state)
        m.zero_grad(set_to_none=True)
        old = B._FUSE_DS
        B._FUSE_DS = on
        before = B.FUSED_DS_CALLS[0]
        try:
            out = m(x)
            out.float().square().mean().backward()
        finally:
            B._FUSE_DS = old
        assert (B.FUSED_DS_CALLS[0] - before == 4) == on
        runs.append((out.detach().clone(), {k: v.clone() for k, v in m.state_dict().items()},
                     {n: p.grad.float().clone() for n, p in m.named_parameters()}))
    (oa, sa, ga), (ob, sb, gb) = runs
    assert torch.equal(oa, ob)
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    for n in ga:
        a, b = ga[n].flatten(), gb[n].flatten()
        cos = float(torch.nn.functional.cosine_similarity(a.double(), b.double(), dim=0))
        assert cos > 0.99 or float(b.abs().max()) < 1e-6, (n, cos)
        if n.startswith("layer4.") or n.startswith("fc."):
            scale = b.abs().max().clamp_min(1e-6)
            assert float((a - b).abs().max() / scale) < 2e-2, n
