"""The own 256 x 256 one-wave-per-SIMD MFMA GEMM (csrc/hip/gemm4w.hip) against fp32 references:
plain C = A B^T at ragged M / several N, K; the FFN forward epilogue (bias + GELU, the
pre-activation kept) and the FFN backward epilogue (dGELU from the pre-activation + bias
gradient column sums), both GELU flavours."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _dn():
    from apex_example_amd import _native
    return _native.require().dense


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mnk", [(256, 256, 128), (1000, 512, 256), (4096, 1024, 1024),
                                 (333, 4096, 384), (16384, 256, 1024)])
def test_gemm4w_plain(mnk, dtype):
    m, n, k = mnk
    g = torch.Generator(device=DEV).manual_seed(m + n + k)
    a = torch.randn(m, k, device=DEV, generator=g).to(dtype)
    b = torch.randn(n, k, device=DEV, generator=g).to(dtype)
    assert _dn().gemm4w_ok(a, b)
    c, = _dn().gemm4w(a, b)
    ref = a.float() @ b.float().t()
    err = float((c.float() - ref).abs().max() / ref.abs().max())
    assert err < 1e-2, err
    # bitwise-stable across calls (no atomics, fixed order)
    assert torch.equal(c, _dn().gemm4w(a, b)[0])


@pytest.mark.parametrize("mnk", [(256, 256, 64), (300, 768, 192), (1000, 512, 1088)])
def test_gemm4w_odd_k_tiles(mnk):
    """gemm4w takes K % 64 == 0 (an odd number of 64-deep K-tiles, one K-tile)."""
    m, n, k = mnk
    g = torch.Generator(device=DEV).manual_seed(m + k)
    a = torch.randn(m, k, device=DEV, generator=g).to(torch.bfloat16)
    b = torch.randn(n, k, device=DEV, generator=g).to(torch.bfloat16)
    assert _dn().gemm4w_ok(a, b)
    c, = _dn().gemm4w(a, b)
    ref = a.float() @ b.float().t()
    assert float((c.float() - ref).abs().max() / ref.abs().max()) < 1e-2


def test_gemm4w_asymmetric_layout():
    """Exact small-integer data with A = I (rows) and an asymmetric B: catches a
    transposed or permuted C write (the C^T accumulators and the permuted B rows)."""
    m, n, k = 512, 512, 512
    a = torch.eye(m, k, device=DEV, dtype=torch.bfloat16)
    b = (torch.arange(n, device=DEV).view(n, 1) * 3 + torch.arange(k, device=DEV).view(1, k)) % 61
    b = b.to(torch.bfloat16)
    c, = _dn().gemm4w(a, b)
    assert torch.equal(c.float(), (a.float() @ b.float().t()))


def test_gemm4w_strided_rows():
    """Row strides larger than K (views of a wider matrix)."""
    g = torch.Generator(device=DEV).manual_seed(5)
    big = torch.randn(512, 640, device=DEV, generator=g).to(torch.bfloat16)
    a = big[:, :512]
    b = torch.randn(768, 640, device=DEV, generator=g).to(torch.bfloat16)[:, 128:]
    c, = _dn().gemm4w(a, b)
    ref = a.float() @ b.float().t()
    assert float((c.float() - ref).abs().max() / ref.abs().max()) < 1e-2


@pytest.mark.parametrize("tanh", [False, True])
@pytest.mark.parametrize("dtype,bias_dtype", [(torch.bfloat16, torch.bfloat16),
                                              (torch.bfloat16, torch.float32),
                                              (torch.float16, torch.float16)])
def test_gemm4w_gelu_epilogues(tanh, dtype, bias_dtype):
    m, n, k = 1536, 1024, 512
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(m, k, device=DEV, generator=g).to(dtype)
    w = (torch.randn(n, k, device=DEV, generator=g) / k ** 0.5).to(dtype)
    bias = (torch.randn(n, device=DEV, generator=g) * 0.1).to(bias_dtype)
    approx = "tanh" if tanh else "none"
    h, pre = _dn().gemm4w(x, w, 1, bias=bias, want_pre=True, tanh=tanh)
    pre_ref = (x.float() @ w.float().t() + bias.float())
    assert float((pre.float() - pre_ref).abs().max()) < 3e-2
    h_ref = F.gelu(pre.float(), approximate=approx)   # gelu of the rounded pre-activation
    assert float((h.float() - h_ref).abs().max()) < 2e-2
    # backward: dpre = dh * gelu'(pre), dh = dy @ W2^T computed by the GEMM
    dy = torch.randn(m, 768, device=DEV, generator=g).to(dtype)
    w2t = (torch.randn(n, 768, device=DEV, generator=g) / 768 ** 0.5).to(dtype)
    dpre, db = _dn().gemm4w(dy, w2t, 2, aux=pre, tanh=tanh, bias_grad_dtype=torch.float32)
    dh = (dy.float() @ w2t.float().t()).to(dtype).float()
    p = pre.float().requires_grad_(True)
    gref, = torch.autograd.grad(F.gelu(p, approximate=approx), p, dh)
    scale = float(gref.abs().max())
    assert float((dpre.float() - gref).abs().max()) / scale < 2e-2
    db_ref = dpre.float().sum(0)
    torch.testing.assert_close(db, db_ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("fused", [False, True])
def test_ffn_gemm4w_grads_after_inplace_weight_update(monkeypatch, fused):
    """the fused FFN backward must see W2 as it is NOW.  Fused
    optimizers write weights through their data pointers without bumping the version
    counter; run fwd/bwd, update W2 in place the way they do, then fwd/bwd again and
    compare the input gradient with the unfused F.linear path."""
    from apex_example_amd import fused_dense as fd
    if not fused:  # the unfused path (hipBLASLt GEMMs + GELU passes)
        monkeypatch.setattr(fd, "_g4w_ok", lambda *a: False)
    g = torch.Generator(device=DEV).manual_seed(11)
    m, d, f = 512, 256, 1024
    x = torch.randn(m, d, device=DEV, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(f, d, device=DEV, generator=g) / d ** 0.5).to(torch.bfloat16)
    b1 = (torch.randn(f, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    w2 = (torch.randn(d, f, device=DEV, generator=g) / f ** 0.5).to(torch.bfloat16)
    b2 = (torch.randn(d, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    dy = torch.randn(m, d, device=DEV, generator=g).to(torch.bfloat16)
    ws = [t.clone().requires_grad_(True) for t in (w1, b1, w2, b2)]  # the same leaves
    for step in range(2):
        xr = x.clone().requires_grad_(True)
        y = fd.fused_dense_gelu_dense_function(xr, *ws, approximate="tanh")
        y.backward(dy)
        xf = x.float().requires_grad_(True)
        h = F.gelu(F.linear(xf, w1.float(), b1.float()), approximate="tanh")
        F.linear(h, ws[2].detach().float(), b2.float()).backward(dy.float())
        err = float((xr.grad.float() - xf.grad).abs().max() / xf.grad.abs().max())
        assert err < 3e-2, (step, err)
        # in-place update that leaves _version alone (as a data_ptr-writing kernel does)
        with torch.no_grad():
            ws[2].data.mul_(-1.5)
