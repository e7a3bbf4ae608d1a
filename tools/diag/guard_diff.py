#!/usr/bin/env python3
"""Per-step master-weight / momentum differences between amp's host-synchronous skip
and the device-side step guard (amp/_guard.py) for torch SGD with momentum."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

dev = torch.device("cuda", 0)


def run(sync_free, overflow_at=(2,), steps=5):
    from apex_example_amd import amp

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(1, 8, 3, padding=1), torch.nn.BatchNorm2d(8),
                                torch.nn.ReLU(), torch.nn.Flatten(),
                                torch.nn.Linear(8 * 8 * 8, 10)).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    model, opt = amp.initialize(model, opt, opt_level="O2", half_dtype=torch.float16,
                                verbosity=0, sync_free=sync_free)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.rand(16, 1, 8, 8, device=dev, generator=g)
    y = torch.randint(0, 10, (16,), device=dev, generator=g)
    trace = []
    for it in range(steps):
        xi = x.clone()
        if it in overflow_at:
            xi[0, 0, 0, 0] = float("inf")
        loss = F.cross_entropy(model(xi).float(), y)
        opt.zero_grad()
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        grads = [None if p.grad is None else p.grad.detach().clone()
                 for p in amp.master_params(opt)]
        opt.step()
        torch.cuda.synchronize()
        trace.append(([p.detach().clone() for p in amp.master_params(opt)],
                      [v.clone() for st in opt.state.values() for v in st.values()
                       if torch.is_tensor(v)], grads,
                      float(amp._amp_state.loss_scalers[0].loss_scale())))
    return trace


a = run(False)
b = run(None)
for it, (ta, tb) in enumerate(zip(a, b)):
    dm = max((x - y).abs().max().item() for x, y in zip(ta[0], tb[0]))
    ds = max([(x - y).abs().max().item() for x, y in zip(ta[1], tb[1])] or [0.0])
    dg = max([(x - y).abs().max().item() for x, y in zip(ta[2], tb[2])
              if x is not None and y is not None] or [float("nan")])
    print("step %d: master %.3e state %.3e (n %d/%d) grad %.3e scale %s/%s" % (
        it, dm, ds, len(ta[1]), len(tb[1]), dg, ta[3], tb[3]))
