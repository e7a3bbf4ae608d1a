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


def test_resnet50_step_grads_with_x2_fusion():
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
