"""amp_C / multi_tensor_applier semantics on the C++ CPU path (the GPU kernels are
checked against the same references in test_kernels_gpu.py)."""
import math

import pytest
import torch

from apex_example_amd import amp_C
from apex_example_amd.multi_tensor_apply import multi_tensor_applier


def _lists(sizes, dtype=torch.float32, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(n, generator=g).to(dtype) for n in sizes]


SIZES = [1, 7, 100, 8193, 70000]


def test_applier_available_and_chunk_size():
    assert multi_tensor_applier.available
    assert multi_tensor_applier.chunk_size == 2048 * 32


@pytest.mark.parametrize("tin", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("tout", [torch.float32, torch.bfloat16])
def test_scale(tin, tout):
    xs = _lists(SIZES, tin)
    ys = [torch.empty(x.shape, dtype=tout) for x in xs]
    noop = torch.zeros(1, dtype=torch.int32)
    multi_tensor_applier(amp_C.multi_tensor_scale, noop, [xs, ys], 0.5)
    for x, y in zip(xs, ys):
        torch.testing.assert_close(y, (x.float() * 0.5).to(tout))
    assert noop.item() == 0


@pytest.mark.parametrize("bad", [float("inf"), float("-inf"), float("nan")])
def test_scale_overflow_flag(bad):
    xs = _lists(SIZES)
    xs[3][4000] = bad
    ys = [torch.empty_like(x) for x in xs]
    noop = torch.zeros(1, dtype=torch.int32)
    multi_tensor_applier(amp_C.multi_tensor_scale, noop, [xs, ys], 2.0)
    assert noop.item() == 1


def test_scale_device_scalar_reciprocal():
    xs = _lists(SIZES)
    ys = [torch.empty_like(x) for x in xs]
    noop = torch.zeros(1, dtype=torch.int32)
    s = torch.tensor([4.0])
    amp_C.multi_tensor_scale(65536, noop, [xs, ys], s, scale_inv=True)
    for x, y in zip(xs, ys):
        torch.testing.assert_close(y, x / 4)


def test_axpby_and_check_arg():
    xs = _lists(SIZES, seed=1)
    ys = _lists(SIZES, seed=2)
    out = [torch.empty_like(x) for x in xs]
    noop = torch.zeros(1, dtype=torch.int32)
    multi_tensor_applier(amp_C.multi_tensor_axpby, noop, [xs, ys, out], 2.0, -1.0, -1)
    for x, y, o in zip(xs, ys, out):
        torch.testing.assert_close(o, 2 * x - y)
    ys[0][0] = float("nan")
    multi_tensor_applier(amp_C.multi_tensor_axpby, noop, [xs, ys, out], 2.0, -1.0, 0)
    assert noop.item() == 0
    multi_tensor_applier(amp_C.multi_tensor_axpby, noop, [xs, ys, out], 2.0, -1.0, 1)
    assert noop.item() == 1


def test_l2norm_global_and_per_tensor():
    xs = _lists(SIZES, seed=3)
    noop = torch.zeros(1, dtype=torch.int32)
    n, per = multi_tensor_applier(amp_C.multi_tensor_l2norm, noop, [xs], True)
    ref = torch.cat([x.double() for x in xs]).norm().item()
    assert math.isclose(n.item(), ref, rel_tol=1e-6)
    for x, p in zip(xs, per):
        assert math.isclose(p.item(), x.double().norm().item(), rel_tol=1e-6)
    n2, per2 = multi_tensor_applier(amp_C.multi_tensor_l2norm, noop, [xs], False)
    assert per2.numel() == 0


def test_norm_out_blend():
    xs = _lists([10, 20])
    out = torch.tensor([1.0, 2.0])
    noop = torch.zeros(1, dtype=torch.int32)
    amp_C.multi_tensor_norm_out_cuda(65536, noop, [xs], out, 0.9, 0.1, 2)
    exp = [math.sqrt(0.9 * o * o + 0.1 * x.norm().item() ** 2) for o, x in zip([1.0, 2.0], xs)]
    torch.testing.assert_close(out, torch.tensor(exp))


def test_zero_and_flatten():
    from apex_example_amd import apex_C

    xs = _lists([5, 6, 7])
    flat = apex_C.flatten(xs)
    assert flat.numel() == 18
    back = apex_C.unflatten(flat, xs)
    for a, b in zip(xs, back):
        torch.testing.assert_close(a, b)
    amp_C.multi_tensor_zero(65536, None, [xs])
    assert all(float(x.abs().sum()) == 0 for x in xs)


def test_sgd_matches_torch_cpu():
    torch.manual_seed(0)
    ps = [torch.randn(n) for n in [10, 300]]
    ref = [p.clone().requires_grad_(True) for p in ps]
    moms = [torch.zeros_like(p) for p in ps]
    opt = torch.optim.SGD(ref, lr=0.1, momentum=0.9, weight_decay=0.01)
    noop = torch.zeros(1, dtype=torch.int32)
    for it in range(3):
        gs = [torch.randn_like(p) for p in ps]
        for r, g in zip(ref, gs):
            r.grad = g.clone()
        opt.step()
        amp_C.multi_tensor_sgd(65536, noop, [gs, ps, moms], 0.01, 0.9, 0.0, 0.1, False, it == 0,
                               False, 1.0)
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p, r.detach())


def test_noop_flag_skips_optimizer():
    ps = [torch.randn(100)]
    gs = [torch.randn(100)]
    moms = [torch.zeros(100)]
    before = ps[0].clone()
    noop = torch.ones(1, dtype=torch.int32)
    amp_C.multi_tensor_sgd(65536, noop, [gs, ps, moms], 0.0, 0.9, 0.0, 0.1, False, True, False, 1.0)
    torch.testing.assert_close(ps[0], before)


def test_loss_scale_state_machine_kernel():
    from apex_example_amd import _native

    mt = _native.require().mt
    scale = torch.tensor([65536.0])
    unsk = torch.zeros(1, dtype=torch.int32)
    skipped = torch.zeros(1, dtype=torch.int32)
    ovf = torch.zeros(1, dtype=torch.int32)
    for _ in range(3):
        mt.update_loss_scale(scale, unsk, skipped, ovf, 2.0, 4, 0.0, 2.0 ** 24, True)
    assert unsk.item() == 3 and scale.item() == 65536.0
    mt.update_loss_scale(scale, unsk, skipped, ovf, 2.0, 4, 0.0, 2.0 ** 24, True)
    assert unsk.item() == 0 and scale.item() == 131072.0
    ovf.fill_(1)
    mt.update_loss_scale(scale, unsk, skipped, ovf, 2.0, 4, 0.0, 2.0 ** 24, True)
    assert scale.item() == 65536.0 and skipped.item() == 1 and unsk.item() == 0
    # min clamp
    scale.fill_(1.0)
    mt.update_loss_scale(scale, unsk, skipped, ovf, 2.0, 4, 1.0, 2.0 ** 24, True)
    assert scale.item() == 1.0
    # max clamp
    ovf.zero_()
    scale.fill_(2.0 ** 24)
    for _ in range(4):
        mt.update_loss_scale(scale, unsk, skipped, ovf, 2.0, 4, 0.0, 2.0 ** 24, True)
    assert scale.item() == 2.0 ** 24


def test_channels_last_tensors_accepted():
    a = torch.randn(4, 3, 5, 5).to(memory_format=torch.channels_last)
    b = torch.empty_like(a)
    noop = torch.zeros(1, dtype=torch.int32)
    amp_C.multi_tensor_scale(65536, noop, [[a], [b]], 3.0)
    torch.testing.assert_close(b, a * 3)


def test_legacy_lamb_stages_match_formula_and_honour_noop():
    """amp_C.multi_tensor_lamb_stage{1,2}_cuda (legacy two-stage LAMB API): values
    vs the textbook formula, and a set noop flag leaves every tensor untouched."""
    import torch

    from apex_example_amd import amp_C

    torch.manual_seed(0)
    shapes = [(7,), (3, 5)]
    g = [torch.randn(s) for s in shapes]
    p = [torch.randn(s) for s in shapes]
    m = [torch.randn(s) * 0.1 for s in shapes]
    v = [torch.rand(s) * 0.1 for s in shapes]
    u = [torch.zeros(s) for s in shapes]
    decay = [0.01, 0.0]
    b1, b2, eps, step, gn, mx, lr = 0.9, 0.999, 1e-6, 3, 4.0, 1.0, 0.1
    ref_m = [mi * b1 + (gi / 4.0) * (1 - b1) for gi, mi in zip(g, m)]
    ref_v = [vi * b2 + (gi / 4.0) ** 2 * (1 - b2) for gi, vi in zip(g, v)]
    ref_u = [(rm / (1 - b1 ** step)) / ((rv / (1 - b2 ** step)).sqrt() + eps) + d * pi
             for rm, rv, d, pi in zip(ref_m, ref_v, decay, p)]
    noop = torch.zeros(1, dtype=torch.int32)
    # noop set: nothing changes
    before = [t.clone() for t in m + v + u + p]
    amp_C.multi_tensor_lamb_stage1_cuda(0, noop + 1, [g, p, m, v, u], decay, step, b1, b2, eps,
                                        gn, mx)
    pn = [pi.norm() for pi in p]
    amp_C.multi_tensor_lamb_stage2_cuda(0, noop + 1, [p, u], pn, [torch.ones(())] * 2, lr, 0.01)
    for a, b in zip(before, m + v + u + p):
        assert torch.equal(a, b)
    amp_C.multi_tensor_lamb_stage1_cuda(0, noop, [g, p, m, v, u], decay, step, b1, b2, eps,
                                        torch.tensor([gn]), mx)
    for a, b in zip(m + v + u, ref_m + ref_v + ref_u):
        torch.testing.assert_close(a, b)
    un = [ui.norm() for ui in u]
    p0 = [pi.clone() for pi in p]
    amp_C.multi_tensor_lamb_stage2_cuda(0, noop, [p, u], pn, un, lr, 0.01)
    for a, b, ui, pni, uni in zip(p, p0, u, pn, un):
        torch.testing.assert_close(a, b - lr * (pni / uni) * ui)
