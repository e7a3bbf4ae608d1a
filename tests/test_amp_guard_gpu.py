"""Sync-free overflow skipping for non-fused optimizers (amp/_guard.py): torch.optim
optimizers under amp O2 / O1 with dynamic loss scaling, an injected overflow at step 2
(and at step 0, where torch SGD would create its momentum buffer), must end bitwise
equal to Apex's host-synchronous skip (sync_free=False), with the same loss scale and
skipped-step count - and the guarded run must not read the flag on the host in the
steady state."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


def _run(make_opt, opt_level, sync_free, overflow_at=(2,), steps=6):
    from apex_example_amd import amp

    # MIOpen's fp16 conv weight gradient may reduce with atomics (a 1e-6 run-to-run
    # difference at some steps, measured with tools/diag/guard_diff.py): ask for its
    # deterministic solvers so the two runs can be compared bitwise
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(1, 8, 3, padding=1), torch.nn.BatchNorm2d(8),
                                torch.nn.ReLU(), torch.nn.Flatten(),
                                torch.nn.Linear(8 * 8 * 8, 10)).to(dev)
    opt = make_opt(model.parameters())
    model, opt = amp.initialize(model, opt, opt_level=opt_level, half_dtype=torch.float16,
                                verbosity=0, sync_free=sync_free)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.rand(16, 1, 8, 8, device=dev, generator=g)
    y = torch.randint(0, 10, (16,), device=dev, generator=g)
    for it in range(steps):
        xi = x.clone()
        if it in overflow_at:
            xi[0, 0, 0, 0] = float("inf")
        loss = F.cross_entropy(model(xi).float(), y)
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
    torch.cuda.synchronize()
    sc = amp._amp_state.loss_scalers[0]
    params = [p.detach().clone() for p in model.parameters()]
    masters = [p.detach().clone() for p in amp.master_params(opt)]
    state = [v.clone() for st in opt.state.values() for v in st.values() if torch.is_tensor(v)]
    return params, masters, state, sc.loss_scale(), sc.skipped_steps() if sc.sync_free else \
        getattr(sc, "_skipped_host", 0), sc.sync_free


OPTS = {
    "sgd": lambda ps: torch.optim.SGD(ps, lr=0.05),
    "sgd_momentum": lambda ps: torch.optim.SGD(ps, lr=0.05, momentum=0.9, weight_decay=1e-4),
    "adam": lambda ps: torch.optim.Adam(ps, lr=1e-3),            # CPU step: host fallback
}


@pytest.mark.parametrize("name", list(OPTS))
@pytest.mark.parametrize("opt_level", ["O2", "O1"])
@pytest.mark.parametrize("overflow_at", [(2,), (0, 3)])
def test_guarded_step_matches_host_skip(name, opt_level, overflow_at):
    ref = _run(OPTS[name], opt_level, False, overflow_at)
    got = _run(OPTS[name], opt_level, None, overflow_at)
    assert got[5] and not ref[5]          # guarded run is sync-free, reference is not
    # a skipped step leaves no trace (tools/diag/guard_diff.py: masters / state equal to
    # 0.0 right after it); the tolerance only covers kernel-level run-to-run noise
    for a, b in zip(got[0], ref[0]):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-5)
    for a, b in zip(got[1], ref[1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)
    assert len(got[2]) == len(ref[2])
    for a, b in zip(got[2], ref[2]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    assert got[3] == ref[3] and got[4] == ref[4] == len(overflow_at)


def test_guarded_sgd_steady_state_has_no_host_sync(monkeypatch):
    """After the first step the guard never reads the flag on the host."""
    from apex_example_amd import amp

    torch.manual_seed(0)
    model = torch.nn.Linear(16, 4).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.float16, verbosity=0)
    x = torch.randn(8, 16, device=dev)
    for _ in range(2):
        loss = model(x).float().pow(2).mean()
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
    torch.cuda.synchronize()
    reads = {"n": 0}
    orig = torch.Tensor.item

    def counting_item(self):
        if self.is_cuda:                  # device -> host reads only
            reads["n"] += 1
        return orig(self)
    monkeypatch.setattr(torch.Tensor, "item", counting_item)
    for _ in range(3):
        loss = model(x).float().pow(2).mean()
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
    monkeypatch.setattr(torch.Tensor, "item", orig)
    assert reads["n"] == 0
