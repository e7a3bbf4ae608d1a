"""Fused attention kernels (csrc/hip/attention.hip) vs fp32 torch references,
including the exact counter-hash dropout masks."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
M32 = 0xFFFFFFFF


def _C():
    from apex_example_amd import _native

    return _native.require().attn


def _mul32(a, c):
    return (a * c) & M32


def drop_keep_mask(B, H, S, seed, p):
    """[B, H, S(q), S(k)] keep mask of the kernels' hash (int64 torch arithmetic)."""
    thr = int(p * 65536 + 0.5)
    bh = torch.arange(B * H, dtype=torch.int64).view(B, H, 1, 1)
    q = torch.arange(S, dtype=torch.int64).view(1, 1, S, 1)
    key = torch.arange(S, dtype=torch.int64).view(1, 1, 1, S)
    kp = key >> 1
    x = (seed ^ _mul32(bh, 0x9E3779B1) ^ _mul32(q, 0x85EBCA77) ^ _mul32(kp, 0xC2B2AE3D)) & M32
    x = x ^ (x >> 16)
    x = _mul32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mul32(x, 0x846CA68B)
    x = x ^ (x >> 16)
    v = torch.where((key & 1) == 1, x >> 16, x & 0xFFFF)
    return (v >= thr), 65536.0 / (65536 - thr)


def ref_attention(q, k, v, causal, p=0.0, seed=0):
    """fp32 reference on [B, S, H, D] inputs -> ([B, S, H, D], lse [B, H, S] log2)."""
    B, S, H, D = q.shape
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) / math.sqrt(D)
    if causal:
        s = s.masked_fill(torch.ones(S, S, device=q.device).triu(1).bool(), float("-inf"))
    lse = torch.logsumexp(s, -1) / math.log(2.0)
    pr = torch.softmax(s, -1)
    if p > 0:
        keep, scale = drop_keep_mask(B, H, S, seed, p)
        pr = pr * keep.to(q.device) * scale
    return (pr @ vf).permute(0, 2, 1, 3), lse


def _qkv(B, S, H, dt, fused=True):
    torch.manual_seed(0)
    if fused:  # slices of a fused projection, as the models pass them
        qkv = torch.randn(B, S, 3, H, 64, device=DEV, dtype=dt)
        return qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    return tuple(torch.randn(B, S, H, 64, device=DEV, dtype=dt) for _ in range(3))


@pytest.mark.parametrize("B,S,H", [(2, 128, 2), (1, 200, 3), (2, 512, 4), (1, 64, 1)])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_attn_fwd(B, S, H, causal, dt):
    q, k, v = _qkv(B, S, H, dt)
    o, lse = _C().fwd(q, k, v, causal, 0.0, 0, 1.0 / 8.0)
    ro, rlse = ref_attention(q, k, v, causal)
    torch.testing.assert_close(o.float(), ro, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(lse, rlse, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("causal", [False, True])
def test_attn_fwd_dropout_exact_mask(causal):
    q, k, v = _qkv(2, 256, 2, torch.bfloat16, fused=False)
    o, _ = _C().fwd(q, k, v, causal, 0.1, 1234, 1.0 / 8.0)
    ro, _ = ref_attention(q, k, v, causal, p=0.1, seed=1234)
    torch.testing.assert_close(o.float(), ro, rtol=3e-2, atol=3e-2)
    keep, _ = drop_keep_mask(2, 2, 256, 1234, 0.1)
    assert abs(1 - keep.float().mean().item() - 0.1) < 0.01
