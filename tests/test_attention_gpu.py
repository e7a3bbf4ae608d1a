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


def _murmur32(x):
    x = x ^ (x >> 16)
    x = _mul32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mul32(x, 0x846CA68B)
    return x ^ (x >> 16)


def _umul24(x, c):
    return ((x & 0xFFFFFF) * (c & 0xFFFFFF)) & M32


def drop_keep_mask(B, H, S, seed, p, device="cpu"):
    """[B, H, S(q), S(k)] keep mask of the kernels' hash (int64 torch arithmetic):
    drop_mix(drop_base(seed, bh) + q * kDropQ + (key >> 2) * kDropK), byte (key & 3)
    against round(256 p) (csrc/hip/attention.hip)."""
    from dropout_hash import keep_mask
    return keep_mask(B, H, S, seed, p, device=device)


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
        # the mask mirror runs where the scores are (production shapes: 134 M entries)
        keep, scale = drop_keep_mask(B, H, S, seed, p, device=q.device)
        pr = pr * keep * scale
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


# ------------------------------------------------------------------ backward
def _ref_grads(q, k, v, do, causal, p=0.0, seed=0):
    qf, kf, vf = (t.detach().float().clone().requires_grad_(True) for t in (q, k, v))
    o, _ = ref_attention(qf, kf, vf, causal, p=p, seed=seed)
    o.backward(do.float())
    return qf.grad, kf.grad, vf.grad


def _close(a, b, rel):
    err = (a.float() - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err / scale < rel, (err, scale)


@pytest.mark.parametrize("B,S,H", [(2, 128, 2), (1, 200, 3), (2, 512, 2), (1, 64, 1)])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_attn_bwd(B, S, H, causal, dt):
    from apex_example_amd.ops import fused_attention

    q, k, v = (t.detach().clone().requires_grad_(True) for t in _qkv(B, S, H, dt, fused=False))
    o = fused_attention(q, k, v, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    rq, rk, rv = _ref_grads(q, k, v, do, causal)
    rel = 2e-2 if dt == torch.bfloat16 else 6e-3
    _close(q.grad, rq, rel)
    _close(k.grad, rk, rel)
    _close(v.grad, rv, rel)


@pytest.mark.parametrize("causal", [False, True])
def test_attn_qkv_packed_bwd_and_dropout_mask(causal):
    """Packed [B,S,3,H,64] input (the models' layout) with dropout: grads vs the
    fp32 reference using the kernels' exact keep mask."""
    from apex_example_amd.ops.attention import FusedQKVAttentionFunction

    B, S, H = 2, 256, 2
    torch.manual_seed(1)
    qkv = torch.randn(B, S, 3, H, 64, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = FusedQKVAttentionFunction.apply(qkv, causal, 0.1, 0.125, 4321)
    do = torch.randn_like(o)
    o.backward(do)
    q, k, v = qkv.detach().unbind(2)
    rq, rk, rv = _ref_grads(q, k, v, do, causal, p=0.1, seed=4321)
    g = qkv.grad
    assert g.shape == qkv.shape and g.is_contiguous()
    _close(g[:, :, 0], rq, 3e-2)
    _close(g[:, :, 1], rk, 3e-2)
    _close(g[:, :, 2], rv, 3e-2)


def test_attn_bwd_deterministic():
    from apex_example_amd.ops import fused_attention

    q, k, v = (t.detach().clone().requires_grad_(True) for t in _qkv(2, 384, 2, torch.bfloat16,
                                                                        fused=False))
    do = torch.randn(2, 384, 2, 64, device=DEV, dtype=torch.bfloat16)
    grads = []
    for _ in range(2):
        for t in (q, k, v):
            t.grad = None
        fused_attention(q, k, v, causal=True).backward(do)
        grads.append([t.grad.clone() for t in (q, k, v)])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


def test_bert_layer_fused_attention_matches_sdpa():
    from apex_example_amd.models.bert import BertConfig, BertLayer

    torch.manual_seed(0)
    cfg = BertConfig(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    a = BertLayer(cfg).to(DEV).to(torch.bfloat16)
    cfg_ref = BertConfig(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0,
                         fused_attention=False)
    r = BertLayer(cfg_ref).to(DEV).to(torch.bfloat16)
    r.load_state_dict(a.state_dict())
    x = torch.randn(4, 128, 1024, device=DEV, dtype=torch.bfloat16)
    xa, xr = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yr = a(xa), r(xr)
    _close(ya, yr.float(), 2e-2)
    dy = torch.randn_like(ya)
    ya.backward(dy)
    yr.backward(dy)
    _close(xa.grad, xr.grad.float(), 3e-2)
    _close(a.attention.qkv.weight.grad, r.attention.qkv.weight.grad.float(), 3e-2)


def test_contrib_self_mha_fast_matches_default():
    from apex_example_amd.contrib.multihead_attn import SelfMultiheadAttn

    torch.manual_seed(0)
    fast = SelfMultiheadAttn(1024, 16, bias=True, include_norm_add=True).to(DEV).to(
        torch.bfloat16)
    ref = SelfMultiheadAttn(1024, 16, bias=True, include_norm_add=True, impl="default").to(
        DEV).to(torch.bfloat16)
    ref.load_state_dict(fast.state_dict())
    x = torch.randn(128, 4, 1024, device=DEV, dtype=torch.bfloat16)
    xa, xr = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, _ = fast(xa, xa, xa, is_training=False)
    yr, _ = ref(xr, xr, xr, is_training=False)
    _close(ya, yr.float(), 2e-2)
    dy = torch.randn_like(ya)
    ya.backward(dy)
    yr.backward(dy)
    _close(xa.grad, xr.grad.float(), 3e-2)


# ---------------------------------------------------------- production shapes
# The models' own shapes under the heaviest-first causal tile order and the full dropout
# path: GPT-2-medium (B 8, S 1024, H 16, causal, fp16 - amp O1) and BERT-large (B 32,
# S 512, H 16, dropout 0.1, bf16, packed QKV as the model passes it), forward and all three
# gradients against the fp32 reference (with the kernels' exact keep mask).
def test_attn_production_gpt2_causal_s1024():
    from apex_example_amd.ops import fused_attention

    torch.manual_seed(5)
    B, S, H = 8, 1024, 16
    q, k, v = (torch.randn(B, S, H, 64, device=DEV, dtype=torch.float16).requires_grad_(True)
               for _ in range(3))
    o = fused_attention(q, k, v, causal=True)
    ro, _ = ref_attention(q.detach(), k.detach(), v.detach(), True)
    _close(o.detach(), ro, 1e-2)
    do = torch.randn_like(o)
    o.backward(do)
    rq, rk, rv = _ref_grads(q, k, v, do, True)
    _close(q.grad, rq, 1e-2)
    _close(k.grad, rk, 1e-2)
    _close(v.grad, rv, 1e-2)


def test_attn_production_bert_dropout_s512():
    from apex_example_amd.ops.attention import FusedQKVAttentionFunction

    torch.manual_seed(6)
    B, S, H = 32, 512, 16
    qkv = torch.randn(B, S, 3, H, 64, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    o = FusedQKVAttentionFunction.apply(qkv, False, 0.1, 0.125, 777)
    q, k, v = qkv.detach().unbind(2)
    ro, _ = ref_attention(q, k, v, False, p=0.1, seed=777)
    _close(o.detach(), ro, 3e-2)
    do = torch.randn_like(o)
    o.backward(do)
    rq, rk, rv = _ref_grads(q, k, v, do, False, p=0.1, seed=777)
    g = qkv.grad
    _close(g[:, :, 0], rq, 3e-2)
    _close(g[:, :, 1], rk, 3e-2)
    _close(g[:, :, 2], rv, 3e-2)
