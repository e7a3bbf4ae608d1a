"""amp on the GPU: sync-free dynamic loss scaling, overflow skip, O1/O2/O3 end to end."""
import copy
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _small_resnet():
    from apex_example_amd.models import resnet18

    torch.manual_seed(0)
    return resnet18(num_classes=10, fused_bn=True, gemm_1x1=True).to(DEV).to(
        memory_format=torch.channels_last)


def _step(model, opt, x, y):
    from apex_example_amd import amp

    loss = F.cross_entropy(model(x), y)
    opt.zero_grad()
    with amp.scale_loss(loss, opt) as s:
        s.backward()
    opt.step()
    return loss


def test_o2_sync_free_step_has_no_host_sync():
    from apex_example_amd import amp
    from apex_example_amd.optimizers import FusedSGD

    model = _small_resnet()
    opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, materialize_master_grads=False)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.bfloat16,
                                verbosity=0)
    assert amp._amp_state.loss_scalers[0].sync_free
    x = torch.randn(8, 3, 64, 64, device=DEV).to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=DEV)
    for _ in range(2):  # warm caches (plan tables, allocator)
        _step(model, opt, x, y)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for _ in range(3):
            _step(model, opt, x, y)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()


def test_o2_training_reduces_loss():
    from apex_example_amd import amp
    from apex_example_amd.optimizers import FusedSGD

    model = _small_resnet()
    opt = FusedSGD(model.parameters(), lr=0.02, momentum=0.9, materialize_master_grads=False)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.bfloat16,
                                verbosity=0)
    x = torch.randn(16, 3, 32, 32, device=DEV).to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device=DEV)
    losses = [_step(model, opt, x, y).item() for _ in range(15)]
    assert losses[-1] < losses[0] * 0.7, losses
    # model params stay bf16, masters fp32, and equal after the in-kernel copy
    for mp, ms in zip(opt._amp_stash.all_fp16_params, opt._amp_stash.all_fp32_from_fp16_params):
        assert mp.dtype == torch.bfloat16 and ms.dtype == torch.float32
        torch.testing.assert_close(mp, ms.to(torch.bfloat16), rtol=0, atol=0)


@pytest.mark.parametrize("materialize", [False, True])
def test_overflow_skips_step_and_halves_scale(materialize, capsys):
    from apex_example_amd import amp
    from apex_example_amd.optimizers import FusedSGD

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(),
                                torch.nn.Linear(64, 4)).to(DEV)
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9,
                   materialize_master_grads=materialize)
    model, opt = amp.initialize(model, opt, opt_level="O2", verbosity=1)
    x = torch.randn(8, 32, device=DEV)
    y = torch.randint(0, 4, (8,), device=DEV)
    _step(model, opt, x, y)
    before = [p.detach().clone() for p in model.parameters()]
    masters = [p.detach().clone() for p in amp.master_params(opt)]
    scaler = amp._amp_state.loss_scalers[0]
    s0 = scaler.loss_scale()

    loss = F.cross_entropy(model(x), y)
    opt.zero_grad()
    with amp.scale_loss(loss, opt) as s:
        s.backward()
        # inject an overflow into one gradient
        next(iter(model.parameters())).grad[0].fill_(float("inf"))
    opt.step()
    torch.cuda.synchronize()
    for b, p in zip(before, model.parameters()):
        torch.testing.assert_close(b, p.detach(), rtol=0, atol=0)
    for b, p in zip(masters, amp.master_params(opt)):
        torch.testing.assert_close(b, p.detach(), rtol=0, atol=0)
    assert scaler.loss_scale() == s0 / 2
    assert amp.state_dict()["loss_scaler0"]["unskipped"] == 0
    # next clean step proceeds
    _step(model, opt, x, y)
    torch.cuda.synchronize()
    changed = any(not torch.equal(b, p.detach()) for b, p in zip(before, model.parameters()))
    assert changed
    torch.cuda.synchronize()
    scaler.poll()
    # the Apex message is printed: immediately in sync mode; in sync-free mode from
    # the pinned report the overflow step queued, once it reached the host
    out = capsys.readouterr().out
    assert ("Gradient overflow.  Skipping step, loss scaler 0 reducing loss scale to %s"
            % float(s0 / 2)) in out, out
    assert out.count("Gradient overflow.") == 1, out


def test_o1_fp16_autocast_and_o3():
    from apex_example_amd import amp
    from apex_example_amd.optimizers import FusedAdam

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.GELU(),
                                torch.nn.Linear(64, 8)).to(DEV)
    opt = FusedAdam(model.parameters(), lr=1e-2)
    model, opt = amp.initialize(model, opt, opt_level="O1", verbosity=0)
    x = torch.randn(32, 64, device=DEV)
    y = torch.randint(0, 8, (32,), device=DEV)
    out = model(x)
    assert out.dtype == torch.float16  # linear runs in half under O1
    assert next(model.parameters()).dtype == torch.float32
    losses = [_step(model, opt, x, y).item() for _ in range(20)]
    assert losses[-1] < losses[0]
    with amp.disable_casts():
        assert model(x).dtype == torch.float32


def test_o3_pure_half():
    from apex_example_amd import amp
    from apex_example_amd.optimizers import FusedSGD

    model = torch.nn.Linear(16, 4).to(DEV)
    opt = FusedSGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O3", half_dtype=torch.bfloat16,
                                verbosity=0)
    assert model.weight.dtype == torch.bfloat16
    x = torch.randn(8, 16, device=DEV)
    y = torch.randint(0, 4, (8,), device=DEV)
    _step(model, opt, x, y)
    assert model(x).dtype == torch.float32  # output cast back


def test_fused_adam_lamb_o2_model_copy_in_kernel():
    from apex_example_amd import amp
    from apex_example_amd.optimizers import FusedAdam, FusedLAMB

    for cls in (FusedAdam, FusedLAMB):
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(128, 256), torch.nn.LayerNorm(256),
                                    torch.nn.Linear(256, 10)).to(DEV)
        opt = cls(model.parameters(), lr=1e-3, materialize_master_grads=False)
        model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.bfloat16,
                                    verbosity=0)
        x = torch.randn(16, 128, device=DEV)
        y = torch.randint(0, 10, (16,), device=DEV)
        l0 = _step(model, opt, x, y).item()
        for _ in range(10):
            l1 = _step(model, opt, x, y).item()
        assert l1 < l0
        st = opt._amp_stash
        for mp, ms in zip(st.all_fp16_params, st.all_fp32_from_fp16_params):
            torch.testing.assert_close(mp, ms.to(torch.bfloat16), rtol=0, atol=0)
        sd = opt.state_dict()
        assert sd["param_groups"][0]["step"] == 11


@pytest.mark.parametrize("min_scale", [None, 2.0 ** 14])
def test_sync_free_scaler_trajectory_matches_sync_mode(min_scale):
    """The device-resident scaler (update_loss_scale kernel) follows Apex's
    sync-mode state machine step for step - scale and clean-step counter - over
    4,200 steps with injected overflows: back-to-back overflows (floored at
    min_loss_scale), 2,000-step growth windows, an overflow right after growth."""
    from apex_example_amd.amp.scaler import LossScaler

    sync = LossScaler("dynamic", device=DEV, min_loss_scale=min_scale)
    dev = LossScaler("dynamic", device=DEV, min_loss_scale=min_scale, sync_free=True)
    assert not sync.sync_free and dev.sync_free
    overflows = {3, 4, 5, 6, 700, 2706, 2707, 4100}
    n = 4200
    hist = torch.empty(n, 2, device=DEV)
    ref = []
    for i in range(n):
        for s in (sync, dev):
            s.clear_overflow_state()
            if i in overflows:
                s._overflow_buf.fill_(1)
        skip = sync.update_scale()
        assert skip == (i in overflows)
        ref.append((sync.loss_scale(), sync._unskipped))
        assert dev.update_scale() is False  # never a host decision in sync-free mode
        hist[i, 0] = dev._scale_dev[0]
        hist[i, 1] = dev._unskipped_dev[0].float()
    got = hist.cpu().tolist()
    for i, ((s_ref, u_ref), (s_dev, u_dev)) in enumerate(zip(ref, got)):
        assert (s_ref, u_ref) == (s_dev, int(u_dev)), (i, (s_ref, u_ref), (s_dev, u_dev))
    assert dev.skipped_steps() == len(overflows)
    # the run crossed at least one full 2,000-step growth window (707..2706)
    assert max(r[0] for r in ref[707:2706]) > ref[706][0]


@pytest.mark.parametrize("opt_level", ["O1", "O2"])
@pytest.mark.parametrize("sync_free", [True, False])
def test_folded_unscale_matches_materialized_across_growth(opt_level, sync_free):
    """Folded unscale (materialize_master_grads=False: the fused optimizer divides
    by the loss scale in-kernel, AFTER update_scale ran) vs the materialized path
    (grads unscaled before update_scale), with scale_window=2 so the scale GROWS
    every other step: the folded path must divide by the scale the grads were
    produced with, not the grown one.  O1 also covers the pending-grad unscale of
    a second backward before a step (gradient accumulation)."""
    from apex_example_amd import amp
    from apex_example_amd.amp import amp as amp_mod
    from apex_example_amd.optimizers import FusedAdam

    def run(materialize):
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(),
                                    torch.nn.Linear(64, 4)).to(DEV)
        opt = FusedAdam(model.parameters(), lr=1e-2, materialize_master_grads=materialize)
        model, opt = amp.initialize(model, opt, opt_level=opt_level, verbosity=0,
                                    loss_scale="dynamic")
        sc = amp._amp_state.loss_scalers[0]
        sc._scale_seq_len = 2
        if not sync_free and sc.sync_free:
            sc.sync_free = False
            opt._amp_stash.sync_free = False
        torch.manual_seed(1)
        scales = []
        for it in range(6):
            x = torch.randn(16, 32, device=DEV)
            y = torch.randint(0, 4, (16,), device=DEV)
            opt.zero_grad()
            n_acc = 2 if (opt_level == "O1" and it == 3) else 1
            for _ in range(n_acc):
                loss = F.cross_entropy(model(x), y)
                with amp.scale_loss(loss, opt) as s:
                    s.backward()
            opt.step()
            scales.append(sc.loss_scale())
        out = [p.detach().float().clone() for p in amp.master_params(opt)]
        amp_mod.deinit()
        amp._amp_state.handle = None
        return out, scales

    a, sa = run(True)
    b, sb = run(False)
    assert sa == sb and sa[-1] > sa[0], (sa, sb)
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_fused_sgd_native_plan_and_pair_launch_match_python_path(monkeypatch):
    """FusedSGD's steady-state native path (StepPlan per launch set, and the amp O2
    16-bit-copy + fp32 BatchNorm sets in ONE launch, mt_sgd_pair) is bitwise the
    per-step Python launch path."""
    from apex_example_amd import amp
    from apex_example_amd.models import resnet18
    from apex_example_amd.optimizers import FusedSGD
    from apex_example_amd.optimizers import _base
    from apex_example_amd.optimizers import fused_sgd as fs

    x = torch.randn(8, 3, 32, 32, device="cuda").to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    out, pairs = {}, {"n": 0}
    orig_pair = fs.FusedSGD._step_pair

    def counting(self, *a):
        r = orig_pair(self, *a)
        pairs["n"] += int(bool(r))
        return r
    monkeypatch.setattr(fs.FusedSGD, "_step_pair", counting)
    for plan in (False, True):
        monkeypatch.setattr(_base, "_STEP_PLAN", plan)
        torch.manual_seed(0)
        m = resnet18(num_classes=10, fused_bn=True, gemm_1x1=True).cuda().to(
            memory_format=torch.channels_last)
        opt = FusedSGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4,
                       materialize_master_grads=False)
        m, opt = amp.initialize(m, opt, opt_level="O2", half_dtype=torch.bfloat16, verbosity=0)
        n0 = pairs["n"]
        for _ in range(4):
            loss = torch.nn.functional.cross_entropy(m(x).float(), y)
            opt.zero_grad()
            with amp.scale_loss(loss, opt) as s:
                s.backward()
            opt.step()
        torch.cuda.synchronize()
        out[plan] = [p.detach().clone() for p in amp.master_params(opt)] + \
            [p.detach().clone() for p in m.parameters()]
        if plan:
            assert pairs["n"] - n0 >= 2   # steps 3 and 4 (plans exist from step 2's end)
        else:
            assert pairs["n"] == n0
    for a, b in zip(out[False], out[True]):
        assert torch.equal(a, b)


def test_folded_unscale_clip_through_master_params():
    """amp O1 + FusedAdam(materialize_master_grads=False) keeps the grads loss-scaled
    after scale_loss; Apex's documented clip between backward and step,
    clip_grad_norm_(amp.master_params(opt), max_norm), must still see unscaled grads
    (master_params removes the pending scale once, in place) and match the
    materialized path step for step."""
    from apex_example_amd import amp
    from apex_example_amd.amp import amp as amp_mod
    from apex_example_amd.optimizers import FusedAdam

    def run(materialize):
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.ReLU(),
                                    torch.nn.Linear(64, 4)).to(DEV)
        opt = FusedAdam(model.parameters(), lr=1e-2, materialize_master_grads=materialize)
        model, opt = amp.initialize(model, opt, opt_level="O1", verbosity=0,
                                    loss_scale="dynamic")
        torch.manual_seed(1)
        norms = []
        for _ in range(6):
            x = torch.randn(16, 32, device=DEV) * 10
            y = torch.randint(0, 4, (16,), device=DEV)
            opt.zero_grad()
            loss = F.cross_entropy(model(x), y)
            with amp.scale_loss(loss, opt) as s:
                s.backward()
            norms.append(float(torch.nn.utils.clip_grad_norm_(amp.master_params(opt), 0.05)))
            opt.step()
        out = [p.detach().float().clone() for p in amp.master_params(opt)]
        amp_mod.deinit()
        amp._amp_state.handle = None
        return out, norms

    a, na = run(True)
    b, nb = run(False)
    # overflowed steps (inf norm: skipped by both paths) aside, the clip is active
    fin = [i for i, n in enumerate(na) if math.isfinite(n)]
    assert len(fin) >= 2 and all(na[i] > 0.05 for i in fin), na
    for x, y in zip(na, nb):
        assert (x == y) if not math.isfinite(x) else abs(x - y) <= 1e-4 * abs(x), (na, nb)
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)
