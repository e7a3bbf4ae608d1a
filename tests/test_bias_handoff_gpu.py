"""The dense bias gradient handed over by the fused residual-join backward
(apex_example_amd/ops/_bias_handoff.py; csrc/hip/layer_norm.hip ln_bwd_fast<..., HS>):
the column sums of dh formed next to the dgamma / dbeta partials must equal the dense
layer's own column-sum pass over dh (and an fp32 reference), and the dense layers of a
BERT layer must actually take them."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("n2", [1024, 2048])
def test_join_dh_colsum_matches_reference(dtype, p, n2):
    """n2 = 2048 needs more than 64 KB of LDS for the third per-wave partial row: no
    column sums are offered there (the dense layer sums dh itself) unless the one-row-set
    combine (layer_norm.set_bwd_one_row, off by default) is on."""
    from apex_example_amd import _native
    from apex_example_amd.normalization import FusedLayerNorm, fused_add_dropout_layer_norm

    torch.manual_seed(1)
    ln = FusedLayerNorm(n2).to(DEV).to(dtype)
    x = torch.randn(2048, n2, device=DEV, dtype=dtype, requires_grad=True)
    h = torch.randn(2048, n2, device=DEV, dtype=dtype, requires_grad=True)
    y, s = fused_add_dropout_layer_norm(x, h, ln, p, True)
    dy = torch.randn_like(y)
    captured = {}
    from apex_example_amd.ops import _bias_handoff as H
    real = H.offer

    def spy(dh, cs):
        captured["dh"], captured["cs"] = dh, cs
        real(dh, cs)
    H.offer = spy
    try:
        y.backward(dy)
    finally:
        H.offer = real
        H.clear()
    assert _native.available()
    dh, cs = captured["dh"], captured["cs"]
    if n2 > 1365 and not _native.require().layer_norm.bwd_one_row():
        assert cs is None
        return
    assert cs is not None and cs.dtype == dtype and cs.shape == (n2,)
    assert torch.equal(dh, h.grad)
    ref = dh.double().sum(0)
    assert _rel(cs, ref) < (1e-2 if dtype == torch.bfloat16 else 1e-5)
    # the same numbers the dense layer's own pass (bias_grad.hip) produces, to rounding
    own = _native.require().dense.bias_grad(dh, dtype)
    assert _rel(cs, own) < (1e-2 if dtype == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_bert_layer_takes_handoff_and_matches(monkeypatch, p):
    from apex_example_amd import fused_dense as FD
    from apex_example_amd.models.bert import BertConfig, BertLayer
    from apex_example_amd.ops import _bias_handoff as H

    cfg = BertConfig(hidden_size=512, num_attention_heads=8, intermediate_size=2048,
                     hidden_dropout_prob=p, attention_probs_dropout_prob=0.0)
    torch.manual_seed(0)
    layer = BertLayer(cfg).to(DEV).to(torch.bfloat16)
    x0 = torch.randn(4, 256, 512, device=DEV, dtype=torch.bfloat16)
    dy = torch.randn_like(x0)

    def run(enabled):
        monkeypatch.setattr(H, "ENABLED", enabled)
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        torch.manual_seed(7)  # same dropout seeds both times
        layer(x).backward(dy)
        H.clear()
        return x.grad, {n: q.grad.clone() for n, q in layer.named_parameters()}

    taken = []
    real = H.take

    def spy(g2, dtype):
        r = real(g2, dtype)
        taken.append(r is not None)
        return r
    monkeypatch.setattr(H, "take", spy)
    dx_off, g_off = run(False)
    assert not any(taken)
    taken.clear()
    dx_on, g_on = run(True)
    # the attention-output and FFN-output biases come from the joins
    assert sum(taken) == 2, taken
    assert torch.equal(dx_on, dx_off)
    for n in g_off:
        if n.endswith("bias") and _rel(g_on[n], g_off[n]) > 0:
            assert _rel(g_on[n], g_off[n]) < 1e-2, n  # summation order only
        else:
            assert torch.equal(g_on[n], g_off[n]), n
    assert FD._bias_grad is not None


@pytest.mark.parametrize("xdt,hdt", [(torch.float32, torch.float16), (torch.bfloat16, torch.bfloat16)])
def test_join_one_row_combine_bitwise(xdt, hdt):
    """The one-row-set LDS combine of the LayerNorm backward partials (A/B switch) adds the
    waves in the per-wave rows' order: dgamma / dbeta / dx bitwise equal."""
    from apex_example_amd import _native
    from apex_example_amd.normalization import FusedLayerNorm
    from apex_example_amd.normalization.fused_layer_norm import AddDropoutLayerNormFunction

    L = _native.require().layer_norm
    torch.manual_seed(2)
    n2 = 1024
    ln = FusedLayerNorm(n2).to(DEV).to(xdt)
    x = torch.randn(4096, n2, device=DEV, dtype=xdt)
    h = torch.randn(4096, n2, device=DEV, dtype=hdt)

    def run(one):
        L.set_bwd_one_row(one)
        try:
            xa, ha = x.clone().requires_grad_(True), h.clone().requires_grad_(True)
            ln.weight.grad = ln.bias.grad = None
            torch.manual_seed(5)
            y, s = AddDropoutLayerNormFunction.apply(xa, ha, ln.weight, ln.bias,
                                                     ln.normalized_shape, ln.eps, 0.1, True)
            torch.manual_seed(6)
            (y.float() * torch.randn_like(y, dtype=torch.float32)).sum().backward()
            return [xa.grad, ha.grad, ln.weight.grad.clone(), ln.bias.grad.clone()]
        finally:
            L.set_bwd_one_row(0)

    for a, b in zip(run(0), run(1)):
        assert torch.equal(a, b)
