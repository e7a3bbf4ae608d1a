"""The dense weight-gradient GEMM (csrc/hip/wgrad4w.hip: dW = dY^T X with both operands
row-major over the tokens, transposed LDS fragment reads, fp32 partials per row split +
the slab reduction) against fp32 references: several shapes and split counts, bf16 and
fp16 operands, bf16 / fp32 results, accumulation into and overwrite of a given buffer
(the DDP bucket-view path), strided operand rows, and bitwise run-to-run stability."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _dn():
    from apex_example_amd import _native
    return _native.require().dense


def _ops(T, M, N, dtype, seed, ld_pad=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    dy = torch.randn(T, M + ld_pad, device=DEV, generator=g).to(dtype)[:, :M]
    x = torch.randn(T, N + ld_pad, device=DEV, generator=g).to(dtype)[:, :N]
    return dy, x


def _err(got, ref):
    return float((got.float().reshape(ref.shape) - ref).abs().max() / ref.abs().max())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("tmns", [(64, 256, 256, 1), (1024, 256, 512, 2), (4096, 512, 768, 4),
                                  (16384, 1024, 4096, 4), (8192, 3072, 1024, 8),
                                  (2048, 1024, 1024, 16)])
def test_wgrad4w_matches_fp32(tmns, dtype):
    T, M, N, S = tmns
    dy, x = _ops(T, M, N, dtype, T + M + N)
    assert _dn().wgrad4w_ok(dy, x, S)
    ref = dy.float().t() @ x.float()
    out_dt = torch.bfloat16 if dtype == torch.bfloat16 else torch.float32
    w = _dn().wgrad4w(dy, x, S, out_dt)
    assert w.shape == (M, N) and w.dtype == out_dt
    assert _err(w, ref) < (1e-2 if out_dt == torch.bfloat16 else 1e-3)
    # fixed reduction order: bitwise stable across calls
    assert torch.equal(w, _dn().wgrad4w(dy, x, S, out_dt))


@pytest.mark.parametrize("S", [1, 4])
def test_wgrad4w_fp32_out_accumulate_and_overwrite(S):
    T, M, N = 2048, 512, 256
    dy, x = _ops(T, M, N, torch.bfloat16, 7)
    ref = dy.float().t() @ x.float()
    base = torch.randn(M, N, device=DEV)
    acc = base.clone()
    r = _dn().wgrad4w(dy, x, S, torch.float32, out=acc, accumulate=True)
    assert r.data_ptr() == acc.data_ptr()
    assert _err(acc - base, ref) < 1e-4
    over = torch.full((M, N), 123.0, device=DEV)
    _dn().wgrad4w(dy, x, S, torch.float32, out=over, accumulate=False)
    assert _err(over, ref) < 1e-5


def test_wgrad4w_bf16_out_accumulate_flat_view():
    """A DDP bucket view: a flat bf16 slice of a larger buffer, accumulated into."""
    T, M, N = 4096, 256, 768
    dy, x = _ops(T, M, N, torch.bfloat16, 11)
    ref = dy.float().t() @ x.float()
    bucket = torch.zeros(M * N + 512, device=DEV, dtype=torch.bfloat16)
    view = bucket[256:256 + M * N]
    _dn().wgrad4w(dy, x, 4, torch.bfloat16, out=view, accumulate=False)
    assert _err(view, ref) < 1e-2
    _dn().wgrad4w(dy, x, 4, torch.bfloat16, out=view, accumulate=True)
    assert _err(view, 2 * ref) < 1e-2
    assert bucket[:256].abs().max() == 0 and bucket[256 + M * N:].abs().max() == 0


def test_wgrad4w_strided_rows():
    """Operands that are column slices of wider tensors (row stride > width)."""
    T, M, N = 1024, 256, 256
    dy, x = _ops(T, M, N, torch.bfloat16, 13, ld_pad=64)
    assert dy.stride(0) == M + 64 and x.stride(0) == N + 64
    ref = dy.float().t() @ x.float()
    assert _err(_dn().wgrad4w(dy, x, 2, torch.float32), ref) < 1e-3


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("tmns", [(64, 256, 256, 1), (128, 256, 512, 1), (192, 512, 256, 1),
                                  (4096, 512, 768, 4), (16384, 1024, 4096, 4),
                                  (2048, 1024, 1024, 16)])
def test_wgrad4w_vs_fp32_and_stable(tmns, dtype):
    """wgrad4w against fp32 from 1 to 64 K-tiles per split, bitwise stable across calls
    (the DMA / LDS layout variants it was once compared with were removed in round 6)."""
    T, M, N, S = tmns
    dy, x = _ops(T, M, N, dtype, 3 * T + M, ld_pad=64 if T <= 256 else 0)
    ref = dy.float().t() @ x.float()
    a = _dn().wgrad4w(dy, x, S, torch.float32)
    assert _err(a, ref) < 1e-3
    assert torch.equal(a, _dn().wgrad4w(dy, x, S, torch.float32))


def test_wgrad4w_rejects_unsupported():
    dn = _dn()
    dy, x = _ops(1024, 256, 256, torch.bfloat16, 3)
    assert not dn.wgrad4w_ok(dy, x, 3)                 # 1024 / 3 rows
    assert not dn.wgrad4w_ok(dy[:, :192], x, 1)        # M % 256
    assert not dn.wgrad4w_ok(dy, x[:1000], 1)          # T mismatch
    with pytest.raises(RuntimeError):
        dn.wgrad4w(dy, x, 3, torch.float32)


@pytest.mark.parametrize("w_dtype", [torch.bfloat16, torch.float32])
def test_dense_wgrad_routes_through_wgrad4w(monkeypatch, w_dtype):
    """fused_dense._wgrad with APEX_AMD_DENSE_W4W on takes the own kernel (bf16 weights:
    bf16 result; fp32 master-style weights: fp32 result, also accumulating into a
    given buffer) and matches the hipBLASLt split-K path within rounding."""
    from apex_example_amd import fused_dense as FD
    T, o, i = 4096, 3072, 1024   # 48 output tiles: routed (fewer stay on hipBLASLt)
    dy, x = _ops(T, o, i, torch.bfloat16, 21)
    ref = dy.float().t() @ x.float()
    monkeypatch.setattr(FD, "_DENSE_W4W", False)
    lib = FD._wgrad(dy, x, w_dtype)
    monkeypatch.setattr(FD, "_DENSE_W4W", True)
    called = []
    dn = _dn()
    real = dn.wgrad4w

    def spy(*a, **k):
        called.append(a[2])
        return real(*a, **k)
    monkeypatch.setattr(dn, "wgrad4w", spy, raising=False)
    own = FD._wgrad(dy, x, w_dtype)
    assert called == [FD._w4w_splits(T, o, i)]
    assert own.dtype == w_dtype and own.shape == (o, i)
    tol = 1e-2 if w_dtype == torch.bfloat16 else 1e-4
    assert _err(own, ref) < tol and _err(lib, ref) < tol
    acc = torch.ones(o, i, device=DEV, dtype=w_dtype)
    FD._wgrad(dy, x, w_dtype, out=acc, accumulate=True)
    assert _err(acc - 1, ref) < tol


def test_dense_wgrad_small_weights_stay_on_library(monkeypatch):
    from apex_example_amd import fused_dense as FD
    dy, x = _ops(4096, 1024, 1024, torch.bfloat16, 5)
    monkeypatch.setattr(FD, "_DENSE_W4W", True)
    assert FD._wgrad_w4w(dy, x, torch.bfloat16, None, True) is None


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(1024, 4096), (4096, 1024), (100, 200)])
def test_dense_weight_transpose_kernel(shape, dtype):
    """fused_dense._transposed: the tiled transpose kernel equals w.t() exactly."""
    from apex_example_amd import fused_dense as FD
    w = torch.randn(*shape, device=DEV).to(dtype)
    t = FD._transposed(w)
    assert t.is_contiguous() and t.shape == (shape[1], shape[0])
    assert torch.equal(t, w.t())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("tmns", [(64, 256, 256, 1), (1024, 256, 512, 2), (4096, 512, 768, 4),
                                  (8192, 3072, 1024, 2), (2048, 1024, 1024, 16)])
@pytest.mark.parametrize("b_dtype", [torch.float32, torch.bfloat16])
def test_wgrad4w_bias_column_sums(tmns, dtype, b_dtype):
    """wgrad4w_bias: the same dW as wgrad4w (bitwise) plus db = column sums of dy formed
    from the kernel's fragments (v_dot2 next to the MFMAs), against fp32."""
    T, M, N, S = tmns
    dy, x = _ops(T, M, N, dtype, 5 * T + N)
    out_dt = torch.bfloat16 if dtype == torch.bfloat16 else torch.float32
    w, db = _dn().wgrad4w_bias(dy, x, S, out_dt, bias_dtype=b_dtype)
    assert torch.equal(w, _dn().wgrad4w(dy, x, S, out_dt))
    ref = dy.double().sum(0)
    assert db.dtype == b_dtype and db.shape == (M,)
    assert _err(db, ref.float()) < (1e-2 if b_dtype == torch.bfloat16 else 1e-5)
    w2, db2 = _dn().wgrad4w_bias(dy, x, S, out_dt, bias_dtype=b_dtype)
    assert torch.equal(db, db2)  # fixed order


def test_wgrad4w_bias_into_bucket_view():
    T, M, N = 4096, 3072, 1024
    dy, x = _ops(T, M, N, torch.bfloat16, 19)
    ref = dy.float().t() @ x.float()
    acc = torch.ones(M, N, device=DEV)
    r, db = _dn().wgrad4w_bias(dy, x, 2, torch.float32, out=acc, accumulate=True,
                               bias_dtype=torch.float32)
    assert r.data_ptr() == acc.data_ptr()
    assert _err(acc - 1, ref) < 1e-4
    assert _err(db, dy.double().sum(0).float()) < 1e-5


@pytest.mark.parametrize("w_dtype", [torch.bfloat16, torch.float32])
def test_dense_wgrad_bgrad_routes_through_wgrad4w_bias(monkeypatch, w_dtype):
    from apex_example_amd import fused_dense as FD
    T, o, i = 4096, 3072, 1024
    dy, x = _ops(T, o, i, torch.bfloat16, 23)
    dn = _dn()
    real = dn.wgrad4w_bias
    called = []

    def spy(*a, **k):
        called.append(a[2])
        return real(*a, **k)
    monkeypatch.setattr(dn, "wgrad4w_bias", spy, raising=False)
    monkeypatch.setattr(FD, "_W4W_BIAS", True)
    dw, db = FD._wgrad_bgrad(dy, x, w_dtype, w_dtype)
    assert called and dw.dtype == w_dtype and db.dtype == w_dtype
    monkeypatch.setattr(FD, "_W4W_BIAS", False)
    dw0, db0 = FD._wgrad_bgrad(dy, x, w_dtype, w_dtype)
    assert torch.equal(dw, dw0)
    tol = 1e-2 if w_dtype == torch.bfloat16 else 1e-5
    assert _err(db, db0.float()) < tol
