#!/usr/bin/env python3
"""Numerical check of a committed TunableOp table on ResNet-50: one forward + backward
(no optimizer step) with TunableOp off, then with tuning/resnet50.csv loaded, same
weights and batch; per-parameter gradient and logits relative differences.  A
selection that returns wrong or non-finite results shows up as a large difference."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import bench  # noqa: E402


def run(model, x, y):
    for p in model.parameters():
        p.grad = None
    out = model(x)
    loss = F.cross_entropy(out.float(), y)
    loss.backward()
    torch.cuda.synchronize()
    return out.float().clone(), {n: p.grad.float().clone() for n, p in model.named_parameters()
                                 if p.grad is not None}


def main():
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    w = bench.build_resnet(args, dev, 1)
    model = [c.cell_contents for c in w.step.__closure__
             if isinstance(c.cell_contents, torch.nn.Module)][0]
    x, y = w.batch
    torch.cuda.tunable.enable(False)
    o0, g0 = run(model, x, y)
    from apex_example_amd.utils.gemm_tuning import use_tuned_gemms
    print("table:", use_tuned_gemms("resnet50"), torch.cuda.tunable.is_enabled(), flush=True)
    o1, g1 = run(model, x, y)
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-30))  # noqa: E731
    print("logits rel diff %.2e finite %s" % (rel(o1, o0), bool(torch.isfinite(o1).all())))
    worst = sorted(((rel(g1[n], g0[n]), n, bool(torch.isfinite(g1[n]).all())) for n in g0),
                   reverse=True)
    for r, n, fin in worst[:12]:
        print("  %-40s rel %.2e finite %s" % (n, r, fin))
    # run-to-run noise of the untuned path for scale
    torch.cuda.tunable.enable(False)
    o2, g2 = run(model, x, y)
    noise = max(rel(g2[n], g0[n]) for n in g0)
    print("untuned run-to-run max rel diff %.2e" % noise)


if __name__ == "__main__":
    main()
