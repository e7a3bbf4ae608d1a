"""amp API semantics on CPU: opt-level tables, overrides,
cast placement, the loss-scaler state machine with scripted overflow, skip-step,
num_losses / loss_id, checkpoint format, O1 registries."""
import copy
from collections import OrderedDict

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from apex_example_amd import amp
from apex_example_amd.models import ConvNet, resnet18


def test_opt_level_tables():
    from apex_example_amd.amp.frontend import Properties, opt_levels

    exp = {
        "O0": (torch.float32, False, None, False, 1.0),
        "O1": (None, True, None, None, "dynamic"),
        "O2": (torch.float16, False, True, True, "dynamic"),
        "O3": (torch.float16, False, False, False, 1.0),
    }
    for lvl, (cast, patch, kbn, mw, ls) in exp.items():
        p = opt_levels[lvl](Properties())
        assert p.opt_level == lvl and p.enabled
        assert p.cast_model_type == cast
        assert p.patch_torch_functions == patch
        assert p.keep_batchnorm_fp32 == kbn
        assert p.master_weights == mw
        assert p.loss_scale == ls


def test_bf16_half_dtype():
    from apex_example_amd.amp.frontend import Properties, opt_levels

    p = Properties()
    p.half_dtype = torch.bfloat16
    p = opt_levels["O2"](p)
    assert p.cast_model_type == torch.bfloat16
    with pytest.raises(ValueError):
        p.half_dtype = torch.float32


def test_invalid_opt_level_message():
    with pytest.raises(RuntimeError, match="letter O, not the number zero"):
        amp.initialize(nn.Linear(2, 2), opt_level="02", verbosity=0)


def test_keep_batchnorm_string_override():
    m = nn.Sequential(nn.Conv2d(3, 4, 3), nn.BatchNorm2d(4))
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    m, opt = amp.initialize(m, opt, opt_level="O2", keep_batchnorm_fp32="False",
                            half_dtype=torch.bfloat16, verbosity=0)
    assert m[1].weight.dtype == torch.bfloat16


def test_o2_casts_and_keeps_bn_fp32():
    m = ConvNet()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    m, opt = amp.initialize(m, opt, opt_level="O2", half_dtype=torch.bfloat16, verbosity=0)
    assert m.layer1[0].weight.dtype == torch.bfloat16
    assert m.layer1[1].weight.dtype == torch.float32  # BN kept fp32
    assert m.layer1[1].running_mean.dtype == torch.float32
    out = m(torch.randn(2, 1, 28, 28))
    assert out.dtype == torch.float32  # outputs cast back
    # masters are created lazily at the first backward (apex semantics)
    loss = out.sum()
    with amp.scale_loss(loss, opt) as s:
        s.backward()
    masters = list(amp.master_params(opt))
    assert all(p.dtype == torch.float32 for p in masters)
    assert len(masters) == 10


def test_parallel_wrapped_model_rejected():
    m = nn.Linear(2, 2)
    dp = torch.nn.DataParallel(m)
    with pytest.raises(RuntimeError, match="Parallel wrappers should only be applied"):
        amp.initialize(dp, opt_level="O0", verbosity=0)


def test_half_model_rejected():
    with pytest.raises(RuntimeError, match="expected torch.float32"):
        amp.initialize(nn.Linear(2, 2).half(), opt_level="O2", verbosity=0)


def test_o0_matches_fp32_training_bitwise():
    """BASELINE.json configs[0]: ResNet-18 amp O0 SGD on CPU == plain fp32 torch."""
    torch.manual_seed(0)
    base = resnet18(num_classes=10)
    x = torch.randn(4, 3, 32, 32)
    y = torch.randint(0, 10, (4,))
    m1 = copy.deepcopy(base)
    o1 = torch.optim.SGD(m1.parameters(), lr=0.05, momentum=0.9)
    m2 = copy.deepcopy(base)
    o2 = torch.optim.SGD(m2.parameters(), lr=0.05, momentum=0.9)
    m2, o2 = amp.initialize(m2, o2, opt_level="O0", verbosity=0)
    for _ in range(3):
        l1 = F.cross_entropy(m1(x), y)
        o1.zero_grad()
        l1.backward()
        o1.step()
        l2 = F.cross_entropy(m2(x), y)
        o2.zero_grad()
        with amp.scale_loss(l2, o2) as s:
            s.backward()
        o2.step()
        assert l1.item() == l2.item()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(a, b)


def _train_step(model, opt, x, y, loss_id=0, inject_inf=False):
    loss = F.cross_entropy(model(x), y)
    opt.zero_grad()
    with amp.scale_loss(loss, opt, loss_id=loss_id) as s:
        s.backward()
        if inject_inf:
            next(model.parameters()).grad.view(-1)[0] = float("inf")
    opt.step()
    return loss


def test_dynamic_scaler_overflow_skip_and_growth(capsys):
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(8, 16), nn.ReLU(), nn.Linear(16, 3))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.bfloat16,
                                verbosity=1)
    scaler = amp._amp_state.loss_scalers[0]
    scaler._scale_seq_len = 3  # shorten the growth window for the test
    assert scaler.loss_scale() == 2.0 ** 16
    x = torch.randn(4, 8)
    y = torch.randint(0, 3, (4,))
    _train_step(model, opt, x, y)
    before = [p.detach().clone() for p in model.parameters()]
    masters_before = [p.detach().clone() for p in amp.master_params(opt)]
    _train_step(model, opt, x, y, inject_inf=True)
    out = capsys.readouterr().out
    assert "Gradient overflow.  Skipping step, loss scaler 0 reducing loss scale to 32768.0" in out
    for a, b in zip(before, model.parameters()):
        assert torch.equal(a, b)
    for a, b in zip(masters_before, amp.master_params(opt)):
        assert torch.equal(a, b)
    assert scaler.loss_scale() == 2.0 ** 15
    assert amp.state_dict()["loss_scaler0"]["unskipped"] == 0
    for _ in range(3):
        _train_step(model, opt, x, y)
    assert scaler.loss_scale() == 2.0 ** 16  # doubled after scale_window clean steps


def test_min_max_loss_scale_clamps():
    model = nn.Linear(4, 2)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.bfloat16,
                                min_loss_scale=2.0 ** 15, max_loss_scale=2.0 ** 16,
                                verbosity=0)
    x, y = torch.randn(2, 4), torch.randint(0, 2, (2,))
    for _ in range(3):
        _train_step(model, opt, x, y, inject_inf=True)
    assert amp._amp_state.loss_scalers[0].loss_scale() == 2.0 ** 15


def test_static_loss_scale_never_skips():
    model = nn.Linear(4, 2)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O2", loss_scale=128.0,
                                half_dtype=torch.bfloat16, verbosity=0)
    scaler = amp._amp_state.loss_scalers[0]
    assert not scaler.dynamic and scaler.loss_scale() == 128.0
    x, y = torch.randn(2, 4), torch.randint(0, 2, (2,))
    _train_step(model, opt, x, y)
    assert scaler.loss_scale() == 128.0


def test_num_losses_and_loss_id():
    model = nn.Linear(4, 2)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O2", num_losses=2,
                                half_dtype=torch.bfloat16, verbosity=0)
    assert len(amp._amp_state.loss_scalers) == 2
    x, y = torch.randn(2, 4), torch.randint(0, 2, (2,))
    _train_step(model, opt, x, y, loss_id=1, inject_inf=True)
    sd = amp.state_dict()
    assert list(sd.keys()) == ["loss_scaler0", "loss_scaler1"]
    assert sd["loss_scaler0"]["loss_scale"] == 65536.0
    assert sd["loss_scaler1"]["loss_scale"] == 32768.0


def test_state_dict_golden_format_and_roundtrip(capsys):
    model = nn.Linear(4, 2)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.bfloat16,
                                verbosity=0)
    sd = amp.state_dict()
    assert isinstance(sd, OrderedDict)
    assert sd == OrderedDict([("loss_scaler0", {"loss_scale": 65536.0, "unskipped": 0})])
    # an Apex-written checkpoint entry loads as-is
    amp.load_state_dict({"loss_scaler0": {"loss_scale": 1024.0, "unskipped": 17}})
    assert amp.state_dict()["loss_scaler0"] == {"loss_scale": 1024.0, "unskipped": 17}
    amp.load_state_dict({"loss_scaler0": {"loss_scale": 8.0, "unskipped": 1},
                         "loss_scaler1": {"loss_scale": 8.0, "unskipped": 1}})
    assert "contains 2 entries, while 1 loss_scalers are used" in capsys.readouterr().out
    with pytest.raises(RuntimeError, match="Unexpected key"):
        amp.load_state_dict({"bogus": 1})


def test_checkpoint_resume_bundle(tmp_path):
    torch.manual_seed(0)
    model = ConvNet()
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.bfloat16,
                                verbosity=0)
    x, y = torch.randn(4, 1, 28, 28), torch.randint(0, 10, (4,))
    for _ in range(2):
        _train_step(model, opt, x, y)
    ck = {"model": model.state_dict(), "optimizer": opt.state_dict(), "amp": amp.state_dict()}
    torch.save(ck, tmp_path / "ck.pt")
    ref_loss = _train_step(model, opt, x, y).item()

    ck = torch.load(tmp_path / "ck.pt", weights_only=True)
    torch.manual_seed(1)
    model2 = ConvNet()
    opt2 = torch.optim.SGD(model2.parameters(), lr=0.05, momentum=0.9)
    model2, opt2 = amp.initialize(model2, opt2, opt_level="O2", half_dtype=torch.bfloat16,
                                  verbosity=0)
    model2.load_state_dict(ck["model"])
    opt2.load_state_dict(ck["optimizer"])
    amp.load_state_dict(ck["amp"])
    assert _train_step(model2, opt2, x, y).item() == pytest.approx(ref_loss, rel=1e-2)


def test_o1_cpu_autocast_and_registries():
    from apex_example_amd.amp import amp as amp_mod

    model = nn.Linear(8, 8)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O1", verbosity=0)
    x = torch.randn(4, 8)
    y = model(x)
    assert y.dtype == torch.bfloat16  # CPU autocast policy is bf16
    with amp.disable_casts():
        assert model(x).dtype == torch.float32

    @amp.float_function
    def f(a):
        return a.dtype

    @amp.half_function
    def h(a):
        return a.dtype

    @amp.promote_function
    def p(a, b):
        return (a + b).dtype

    assert f(x.bfloat16()) == torch.float32
    assert h(x) == torch.bfloat16
    assert p(x.bfloat16(), x) == torch.float32

    class Mod:
        @staticmethod
        def g(a):
            return a.dtype

    amp.register_float_function(Mod, "g")
    assert Mod.g(x.bfloat16()) == torch.float32
    with pytest.raises(ValueError):
        amp.register_half_function(Mod, "nope")
    amp_mod.deinit()
    assert Mod.g(x.bfloat16()) == torch.bfloat16  # restored


def test_disabled_returns_inputs():
    m = nn.Linear(2, 2)
    o = torch.optim.SGD(m.parameters(), lr=0.1)
    m2, o2 = amp.initialize(m, o, enabled=False)
    assert m2 is m and o2 is o
    loss = m(torch.randn(1, 2)).sum()
    with amp.scale_loss(loss, o) as s:
        assert s is loss


def test_fp16_utils_convert_network():
    from apex_example_amd.fp16_utils import convert_network, network_to_half, prep_param_lists

    m = nn.Sequential(nn.Conv2d(1, 2, 3), nn.BatchNorm2d(2), nn.Linear(2, 2))
    convert_network(m, torch.bfloat16)
    assert m[0].weight.dtype == torch.bfloat16 and m[1].weight.dtype == torch.float32
    assert m[2].weight.dtype == torch.bfloat16
    n = network_to_half(nn.Sequential(nn.Linear(2, 2), nn.BatchNorm1d(2)))
    assert n[1][1].weight.dtype == torch.float32
    mp, masters = prep_param_lists(nn.Linear(3, 3).half())
    assert all(p.dtype == torch.float32 for p in masters)


def test_fp16_optimizer_legacy():
    from apex_example_amd.fp16_utils import FP16_Optimizer

    torch.manual_seed(0)
    model = nn.Linear(4, 2).to(torch.bfloat16)
    opt = FP16_Optimizer(torch.optim.SGD(model.parameters(), lr=0.1), dynamic_loss_scale=True,
                         verbose=False)
    x = torch.randn(3, 4).to(torch.bfloat16)
    w0 = model.weight.detach().clone()
    loss = model(x).float().sum()
    opt.zero_grad()
    opt.backward(loss)
    opt.step()
    assert not torch.equal(w0, model.weight)
    sd = opt.state_dict()
    assert "fp32_from_fp16" in sd
