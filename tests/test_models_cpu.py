"""Model-zoo checks on CPU: parameter counts of the benchmark architectures
(BASELINE.md section 3), forward shapes and one amp training step of the
small variants through the fused optimizers' CPU path."""
import pytest
import torch

from apex_example_amd.models import resnet18, resnet50
from apex_example_amd.models.bert import (BertConfig, BertForPreTraining, bert_large,
                                          pretraining_loss, synthetic_batch)
from apex_example_amd.models.gpt2 import GPT2Config, GPT2LMHeadModel, gpt2_medium, lm_loss


def _count(m):
    ps = list(m.parameters())
    return sum(p.numel() for p in ps), len(ps)


def test_resnet50_param_count():
    assert _count(resnet50()) == (25_557_032, 161)


@pytest.mark.slow
def test_bert_large_param_count():
    # 398 tensors with separate q/k/v; the fused qkv projection makes it 302
    assert _count(bert_large()) == (336_226_108, 302)


@pytest.mark.slow
def test_gpt2_medium_param_count():
    assert _count(gpt2_medium()) == (354_823_168, 292)


def _tiny_bert():
    return BertConfig(vocab_size=128, hidden_size=32, num_hidden_layers=2, num_attention_heads=4,
                      intermediate_size=64, max_position_embeddings=32)


def _tiny_gpt():
    return GPT2Config(vocab_size=96, n_positions=32, n_embd=32, n_layer=2, n_head=4)


def test_bert_forward_shapes_and_fused_ln_parity():
    cfg = _tiny_bert()
    torch.manual_seed(0)
    m = BertForPreTraining(cfg).eval()
    cfg2 = _tiny_bert()
    cfg2.fused_layer_norm = False
    torch.manual_seed(0)
    m2 = BertForPreTraining(cfg2).eval()
    m2.load_state_dict(m.state_dict())
    b = synthetic_batch(cfg, 3, 16, 4, "cpu", seed=1)
    mlm, nsp = m(b[0], b[1], b[2])
    assert mlm.shape == (12, 128) and nsp.shape == (3, 2)
    mlm2, nsp2 = m2(b[0], b[1], b[2])
    torch.testing.assert_close(mlm, mlm2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(nsp, nsp2, rtol=1e-4, atol=1e-5)


def test_gpt2_causal():
    cfg = _tiny_gpt()
    m = GPT2LMHeadModel(cfg).eval()
    ids = torch.randint(0, 96, (2, 12))
    out = m(ids)
    ids2 = ids.clone()
    ids2[:, 8:] = (ids2[:, 8:] + 1) % 96
    out2 = m(ids2)
    # positions before the edit see no change
    torch.testing.assert_close(out[:, :8], out2[:, :8])
    assert not torch.allclose(out[:, 8:], out2[:, 8:])


def test_gpt2_joined_residual_ln_matches_blockwise():
    """fused_residual_ln (joins feed the next block's ln_1 / ln_f) computes the
    same function as the plain pre-LN block loop, same state dict."""
    cfg = _tiny_gpt()
    torch.manual_seed(0)
    m = GPT2LMHeadModel(cfg).eval()
    cfg2 = _tiny_gpt()
    cfg2.fused_residual_ln = False
    m2 = GPT2LMHeadModel(cfg2).eval()
    m2.load_state_dict(m.state_dict())
    ids = torch.randint(0, 96, (2, 12))
    torch.testing.assert_close(m(ids), m2(ids), rtol=1e-5, atol=1e-5)


def _train(model, opt, batch_fn, loss_fn, opt_level, steps=12):
    from apex_example_amd import amp

    model, opt = amp.initialize(model, opt, opt_level=opt_level, half_dtype=torch.bfloat16,
                                verbosity=0)
    losses = []
    for _ in range(steps):
        loss = loss_fn(model, batch_fn())
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
        losses.append(loss.item())
    return losses


def test_bert_o2_lamb_trains():
    from apex_example_amd.optimizers import FusedLAMB

    cfg = _tiny_bert()
    cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    torch.manual_seed(0)
    m = BertForPreTraining(cfg)
    b = synthetic_batch(cfg, 4, 16, 4, "cpu", seed=2)
    opt = FusedLAMB(m.parameters(), lr=3e-2)
    losses = _train(m, opt, lambda: b,
                    lambda mod, bb: pretraining_loss(*mod(bb[0], bb[1], bb[2]), bb[3], bb[4]),
                    "O2", steps=16)
    assert losses[-1] < losses[0] - 0.8


def test_gpt2_o2_adam_trains():
    from apex_example_amd.optimizers import FusedAdam

    cfg = _tiny_gpt()
    cfg.resid_pdrop = cfg.embd_pdrop = cfg.attn_pdrop = 0.0
    torch.manual_seed(0)
    m = GPT2LMHeadModel(cfg)
    ids = torch.randint(0, 96, (4, 16))
    opt = FusedAdam(m.parameters(), lr=3e-3)
    losses = _train(m, opt, lambda: ids, lambda mod, x: lm_loss(mod(x), x), "O2")
    assert losses[-1] < losses[0] - 0.5


def test_resnet18_o0_cpu_plumbing():
    """BASELINE.json config 1: ResNet-18 amp O0 (fp32 passthrough) SGD on CPU."""
    from apex_example_amd import amp

    torch.manual_seed(0)
    m = resnet18(num_classes=10)
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    m, opt = amp.initialize(m, opt, opt_level="O0", verbosity=0)
    x = torch.randn(8, 3, 32, 32)
    y = torch.randint(0, 10, (8,))
    losses = []
    for _ in range(6):
        loss = torch.nn.functional.cross_entropy(m(x), y)
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
        losses.append(loss.item())
    assert all(p.dtype == torch.float32 for p in m.parameters())
    assert losses[-1] < losses[0]
