#!/usr/bin/env python3
"""Which layer goes non-finite under the committed TunableOp GEMM selections?
One ResNet-50 forward + backward with the table loaded: non-finite module outputs
(forward hooks) and non-finite parameter gradients, by name and shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import bench  # noqa: E402


def main():
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if args.gemm_tuning == "auto":
        from apex_example_amd.utils.gemm_tuning import use_tuned_gemms
        print("table:", use_tuned_gemms(args.model), flush=True)
    w = bench.build_resnet(args, dev, 1)
    model = None
    # find the model through the step closure
    for c in w.step.__closure__ or []:
        v = c.cell_contents
        if isinstance(v, torch.nn.Module):
            model = v
    bad_fwd = []

    def hook(name):
        def f(m, inp, out):
            if isinstance(out, torch.Tensor) and not torch.isfinite(out).all():
                bad_fwd.append((name, tuple(out.shape), tuple(inp[0].shape)))
        return f
    for name, m in model.named_modules():
        if len(list(m.children())) == 0:
            m.register_forward_hook(hook(name))
    x, y = w.batch
    out = model(x)
    loss = F.cross_entropy(out.float(), y)
    loss.backward()
    torch.cuda.synchronize()
    print("loss", loss.item())
    print("non-finite forward outputs:", bad_fwd[:10])
    bad = [(n, tuple(p.shape)) for n, p in model.named_parameters()
           if p.grad is not None and not torch.isfinite(p.grad).all()]
    print("non-finite grads (%d):" % len(bad), bad[:20])
    big = sorted(((float(p.grad.float().abs().max()), n) for n, p in model.named_parameters()
                  if p.grad is not None), reverse=True)[:8]
    print("largest |grad|:", big)


if __name__ == "__main__":
    main()
